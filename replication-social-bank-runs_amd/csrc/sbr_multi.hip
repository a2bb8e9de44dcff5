// sbr_multi.hip — multi-GPU fan-out behind the C ABI (SURVEY.md §8(b) threading
// contract, §8(e) partitioning): an n-device context holds one single-device
// context per GPU; every host-pointer sweep on it
//   1. deals the β (or parameter) columns cyclically — column i to rank i mod N,
//      which balances the β-dependent knot counts and run lengths (sbr_shard.h);
//   2. runs each shard on its own GPU from its own host thread (the single-device
//      *_dev entry points on that child context's own stream, inputs staged into that
//      GPU's HBM);
//   3. returns the results to the caller's host arrays by one of two transports:
//      * direct (the default): each rank copies its own packed block in one DMA into its
//        own pinned landing buffer (from its own thread, so the N GPUs' PCIe links carry
//        the result in parallel and no collective runs — the results of a host-pointer
//        sweep are bound for host memory, which a gather to one GPU would funnel through a
//        single link); once every rank has succeeded, host threads copy the blocks into the
//        caller's u-fastest arrays (column i of the grid is block row i / N of rank
//        i mod N).  A failed call leaves the caller's arrays untouched;
//      * RCCL gather (SBR_FLAG_RCCL_GATHER): after every shard has finished, and after
//        every fallible per-rank step of the gather (device selection, rank 0's gather
//        buffer, its local copy) has succeeded, the packed blocks go to rank 0's HBM with
//        RCCL point-to-point (ncclSend/ncclRecv over xGMI, posted as one group over all
//        communicators from one thread).  If the group or a stream fails after posting,
//        every communicator is aborted (ncclCommAbort: no rank stays blocked) and rebuilt
//        on the next call; rank 0 then scatters the blocks into the caller's arrays.
//      Only the loopback tests (N = 2, 3, 8, 20) and N = 1 hardware runs have exercised
//      the N > 1 layouts so far: the RCCL transport is unverified on multi-GPU hardware.
// Steps 1, 3 and 4 are sbr_shard.h's, shared with the host loopback of
// sbr_shard_host_run (the CPU tests' N = 2, 3, 8 layouts).  Per-point results do not
// depend on the partitioning, so a multi-GPU sweep is bit-identical to a single-device
// one.  librccl.so.1 is loaded, and the communicators created, only when a sweep asks
// for the RCCL gather (reusing an already-loaded copy, e.g. torch's), so libsbr has no
// link-time dependency on it and the default transport never touches it.
#include <dlfcn.h>
#include <math.h>
#include <string.h>

#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/sbr.h"
#include "sbr_hostcopy.h"
#include "sbr_multi.h"
#include "sbr_shard.h"

namespace {

struct Rccl {
    bool ok = false;
    std::string err;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclCommAbort) CommAbort = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

const Rccl& rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (h) break;
        }
        if (!h) {
            r.err = std::string("librccl.so.1 not loadable: ") + dlerror();
            return;
        }
        r.CommInitAll = (decltype(r.CommInitAll))dlsym(h, "ncclCommInitAll");
        r.CommDestroy = (decltype(r.CommDestroy))dlsym(h, "ncclCommDestroy");
        r.CommAbort = (decltype(r.CommAbort))dlsym(h, "ncclCommAbort");
        r.Send = (decltype(r.Send))dlsym(h, "ncclSend");
        r.Recv = (decltype(r.Recv))dlsym(h, "ncclRecv");
        r.GroupStart = (decltype(r.GroupStart))dlsym(h, "ncclGroupStart");
        r.GroupEnd = (decltype(r.GroupEnd))dlsym(h, "ncclGroupEnd");
        r.GetErrorString = (decltype(r.GetErrorString))dlsym(h, "ncclGetErrorString");
        r.ok = r.CommInitAll && r.CommDestroy && r.CommAbort && r.Send && r.Recv && r.GroupStart && r.GroupEnd && r.GetErrorString;
        if (!r.ok) r.err = "librccl.so.1 lacks a required symbol";
    });
    return r;
}

// per-rank device state, kept across calls (grow-only)
struct Rank {
    int device = 0;
    sbr_ctx* kid = nullptr;
    hipStream_t stream = nullptr; // the child context's own stream (sbr_ctx_stream)
    ncclComm_t comm = nullptr;
    void* in = nullptr;     // staged inputs
    size_t in_bytes = 0;
    void* out = nullptr;    // packed result block
    size_t out_bytes = 0;
    void* gather = nullptr; // rank 0: every rank's block
    size_t gather_bytes = 0;
    void* pin = nullptr;    // pinned landing buffer of the direct transport
    size_t pin_bytes = 0;
};

int grow_pinned(void** p, size_t* have, size_t need)
{
    if (need <= *have) return 0;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *have = 0;
    if (hipHostMalloc(p, need) != hipSuccess) return -1;
    *have = need;
    return 0;
}

double ms_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int grow(void** p, size_t* have, size_t need)
{
    if (need <= *have) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    if (hipMalloc(p, need) != hipSuccess) return -1;
    *have = need;
    return 0;
}

}  // namespace

struct sbr_multi {
    std::vector<Rank> ranks;
    std::string err;
    bool comms_ok = false; // false after an abort (or before the first gather): (re)built by the next gather
    bool shared = false;   // rank rehearsal: ranks may share a device (SBR_MULTI_SHARED_DEVICES=1)
    // phases of the last sweep, ms: [0] slowest rank's staging + sweep, [1] slowest rank's D2H
    // into its landing buffer, [2] the host copy into the caller's arrays (direct transport) or
    // the RCCL gather + scatter, [3] unused, [4] the whole call
    double ph[5] = {};
};

namespace {

int init_comms(sbr_multi* m, std::string& err)
{
    const Rccl& R = rccl();
    const int n = (int)m->ranks.size();
    std::vector<ncclComm_t> comms(n);
    std::vector<int> dl(n);
    for (int r = 0; r < n; r++) dl[r] = m->ranks[r].device;
    const ncclResult_t nr = R.CommInitAll(comms.data(), n, dl.data());
    if (nr != ncclSuccess) {
        err = std::string("ncclCommInitAll: ") + R.GetErrorString(nr);
        return SBR_EDEVICE;
    }
    for (int r = 0; r < n; r++) m->ranks[r].comm = comms[r];
    m->comms_ok = true;
    return SBR_OK;
}

void abort_comms(sbr_multi* m)
{
    const Rccl& R = rccl();
    for (Rank& k : m->ranks) {
        if (k.comm) (void)R.CommAbort(k.comm);
        k.comm = nullptr;
    }
    m->comms_ok = false;
}

// RCCL transport of the gather: one group over every rank's communicator, posted from one
// thread; any failure after a send or receive was posted aborts every communicator, so that
// no stream is left waiting for a peer.
struct RcclTransport : sbr_shard::Transport {
    sbr_multi* m;
    const Rccl& R;
    std::string err;
    bool posted = false, failed = false;
    explicit RcclTransport(sbr_multi* m_) : m(m_), R(rccl()) {}
    int bad(const char* what, ncclResult_t nr)
    {
        failed = true;
        err = std::string(what) + ": " + R.GetErrorString(nr);
        return SBR_EDEVICE;
    }
    int begin() override
    {
        const ncclResult_t nr = R.GroupStart();
        return nr == ncclSuccess ? SBR_OK : bad("ncclGroupStart", nr);
    }
    int local_copy(void* dst, const void* src, size_t bytes) override
    {
        Rank& k0 = m->ranks[0];
        if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, k0.stream) != hipSuccess) {
            failed = true;
            err = "gather: rank 0 local copy";
            return SBR_EDEVICE;
        }
        return SBR_OK;
    }
    int recv(int from, void* dst, size_t bytes) override
    {
        posted = true;
        const ncclResult_t nr = R.Recv(dst, bytes, ncclUint8, from, m->ranks[0].comm, m->ranks[0].stream);
        return nr == ncclSuccess ? SBR_OK : bad("ncclRecv", nr);
    }
    int send(int from, const void* src, size_t bytes) override
    {
        posted = true;
        Rank& k = m->ranks[from];
        const ncclResult_t nr = R.Send(src, bytes, ncclUint8, 0, k.comm, k.stream);
        return nr == ncclSuccess ? SBR_OK : bad("ncclSend", nr);
    }
    int end() override
    {
        const ncclResult_t nr = R.GroupEnd();
        return nr == ncclSuccess ? SBR_OK : bad("ncclGroupEnd", nr);
    }
    int wait() override
    {
        // poll every rank's stream; on the first failure (or one already seen while
        // posting) abort all communicators, then drain the streams (aborted kernels exit)
        if (failed && posted) abort_comms(m);
        std::vector<char> done(m->ranks.size(), 0);
        size_t left = m->ranks.size();
        while (left) {
            for (size_t r = 0; r < m->ranks.size(); r++) {
                if (done[r]) continue;
                const hipError_t e = hipStreamQuery(m->ranks[r].stream);
                if (e == hipErrorNotReady) continue;
                done[r] = 1;
                left--;
                if (e != hipSuccess && !failed) {
                    failed = true;
                    err = std::string("gather: rank ") + std::to_string(r) + ": " + hipGetErrorString(e);
                    if (posted) abort_comms(m);
                }
            }
            if (left) std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        return failed ? SBR_EDEVICE : SBR_OK;
    }
};

}  // namespace

namespace sbr_multi_impl {

int create(int n_gpus, const int* devices, sbr_multi** out, std::vector<sbr_ctx*>& kids, std::string& err)
{
    *out = nullptr;
    int ndev = 0;
    // Rank rehearsal (diagnostic): with SBR_MULTI_SHARED_DEVICES=1 in the environment, ranks may
    // share a device (explicit duplicate ids; without a device list, rank r on device r mod
    // ndev), so the n-rank fan-out — host threads, per-rank streams and pinned landing buffers,
    // strided D2H, the all-or-nothing scatter — runs on a one-GPU box.  The RCCL gather needs
    // distinct devices and is refused on such a context.
    const char* sh = getenv("SBR_MULTI_SHARED_DEVICES");
    const bool shared = sh && sh[0] == '1' && sh[1] == 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || n_gpus <= 0 || (!shared && n_gpus > ndev) ||
        n_gpus > 64) {
        err = "n_gpus exceeds the visible HIP devices";
        return SBR_EDEVICE;
    }
    std::vector<int> dl(n_gpus);
    for (int r = 0; r < n_gpus; r++) {
        dl[r] = devices ? devices[r] : r % ndev;
        if (dl[r] < 0 || dl[r] >= ndev) { err = "device id out of range"; return SBR_EDEVICE; }
        for (int q = 0; q < r && !shared; q++)
            if (dl[q] == dl[r]) { err = "duplicate device id"; return SBR_EARG; }
    }
    // no RCCL here: the communicators are created by the first sweep that asks for the gather
    sbr_multi* m = new sbr_multi();
    m->shared = shared;
    m->ranks.resize(n_gpus);
    for (int r = 0; r < n_gpus; r++) m->ranks[r].device = dl[r];
    int rc = SBR_OK;
    for (int r = 0; r < n_gpus; r++) {
        Rank& k = m->ranks[r];
        rc = sbr_init(dl[r], &k.kid);
        if (rc != SBR_OK) {
            err = "per-device context";
            destroy(m);
            return rc;
        }
        k.stream = sbr_ctx_stream(k.kid);
        kids.push_back(k.kid);
    }
    *out = m;
    return SBR_OK;
}

void destroy(sbr_multi* m)
{
    if (!m) return;
    for (Rank& k : m->ranks) {
        (void)hipSetDevice(k.device);
        if (k.stream) (void)hipStreamSynchronize(k.stream);
        if (k.comm) (void)rccl().CommDestroy(k.comm); // a communicator implies a loaded librccl
        for (void* p : {k.in, k.out, k.gather})
            if (p) (void)hipFree(p);
        if (k.pin) (void)hipHostFree(k.pin);
        if (k.kid) (void)sbr_free(k.kid); // owns k.stream
    }
    delete m;
}

int size(const sbr_multi* m) { return m ? (int)m->ranks.size() : 1; }

sbr_ctx* child(sbr_multi* m, int r) { return (m && r >= 0 && r < (int)m->ranks.size()) ? m->ranks[r].kid : nullptr; }

const char* last_error(const sbr_multi* m) { return m ? m->err.c_str() : ""; }

const double* phases(const sbr_multi* m) { return m ? m->ph : nullptr; }

// One sweep over the ranks (plan, deal, pack, gather, scatter: sbr_shard.h).  For rank r
// with cols_r columns:
//   stage(r, cols_r, in_dev, stream) -> int   stages its inputs into in_dev (device)
//   run(r, cols_r, kid, stream, in_dev, out_fields)  enqueues the single-device sweep, writing
//                                              field f of the block at out_fields[f]
int run_sharded(sbr_multi* m, int64_t n_col, int64_t n_u, const std::vector<sbr_shard::Field>& fields,
                size_t in_bytes, const StageFn& stage, const RunFn& run, bool rccl_gather)
{
    m->err.clear();
    const auto t_call = std::chrono::steady_clock::now();
    for (double& x : m->ph) x = 0.0;
    const int N = (int)m->ranks.size();
    const sbr_shard::Plan plan = sbr_shard::make_plan(N, n_col, n_u, fields);
    std::vector<int> rcs(N, SBR_OK);
    std::vector<std::string> errs(N);
    std::vector<double> t_run(N, 0.0), t_d2h(N, 0.0);

    // phase 1: every shard on its GPU, to completion (no collective is entered and no caller array
    // is written unless all succeed); direct transport: each rank's block lands in its pinned buffer
    {
        std::vector<std::thread> th;
        for (int r = 0; r < N; r++)
            th.emplace_back([&, r] {
                Rank& k = m->ranks[r];
                if (plan.cols[r] == 0) return;
                const auto t0 = std::chrono::steady_clock::now();
                if (hipSetDevice(k.device) != hipSuccess) { rcs[r] = SBR_EDEVICE; errs[r] = "hipSetDevice"; return; }
                if (grow(&k.in, &k.in_bytes, in_bytes + 256) || grow(&k.out, &k.out_bytes, plan.block_bytes(r) + 256) ||
                    (!rccl_gather && grow_pinned(&k.pin, &k.pin_bytes, plan.block_bytes(r) + 256))) {
                    rcs[r] = SBR_ENOMEM;
                    errs[r] = "rank buffers";
                    return;
                }
                int rc = stage(r, plan.cols[r], k.in, k.stream);
                std::vector<void*> fp;
                for (size_t o : sbr_shard::field_offsets(plan, r, fields)) fp.push_back((char*)k.out + o);
                if (rc == SBR_OK) rc = run(r, plan.cols[r], k.kid, k.stream, k.in, fp);
                if (rc == SBR_OK && hipStreamSynchronize(k.stream) != hipSuccess) rc = SBR_EDEVICE;
                t_run[r] = ms_since(t0);
                // direct transport: the rank's packed block in one DMA over its own PCIe link
                if (rc == SBR_OK && !rccl_gather) {
                    const auto t1 = std::chrono::steady_clock::now();
                    if (hipMemcpyAsync(k.pin, k.out, plan.block_bytes(r), hipMemcpyDeviceToHost, k.stream) != hipSuccess ||
                        hipStreamSynchronize(k.stream) != hipSuccess)
                        rc = SBR_EDEVICE;
                    t_d2h[r] = ms_since(t1);
                }
                if (rc != SBR_OK) { rcs[r] = rc; errs[r] = sbr_last_error(k.kid); }
            });
        for (auto& t : th) t.join();
    }
    for (int r = 0; r < N; r++) {
        m->ph[0] = t_run[r] > m->ph[0] ? t_run[r] : m->ph[0];
        m->ph[1] = t_d2h[r] > m->ph[1] ? t_d2h[r] : m->ph[1];
    }
    for (int r = 0; r < N; r++)
        if (rcs[r] != SBR_OK) {
            m->err = "rank " + std::to_string(r) + ": " + errs[r];
            return rcs[r];
        }
    if (!rccl_gather) {
        // every rank succeeded: its columns from the landing buffers into the caller's arrays
        const auto t2 = std::chrono::steady_clock::now();
        std::vector<std::array<size_t, 3>> pieces;
        for (int r = 0; r < N; r++) {
            if (plan.cols[r] == 0) continue;
            const std::vector<size_t> fo = sbr_shard::field_offsets(plan, r, fields);
            for (size_t i = 0; i < fields.size(); i++) {
                const sbr_shard::Field& f = fields[i];
                if (!f.host) continue;
                const size_t row = (size_t)n_u * f.per_pt * f.esz;
                for (int64_t c = 0; c < plan.cols[r]; c++)
                    pieces.push_back({(size_t)((char*)f.host + (size_t)sbr_shard::global_col(r, c, N) * row),
                                      (size_t)((const char*)m->ranks[r].pin + fo[i] + (size_t)c * row), row});
            }
        }
        sbr_host::parallel_copy(pieces, 16);
        m->ph[2] = ms_since(t2);
        m->ph[4] = ms_since(t_call);
        return SBR_OK;
    }

    // phase 2, pre-checks: everything fallible before a send or receive is posted
    Rank& k0 = m->ranks[0];
    for (int r = 0; r < N; r++)
        if (hipSetDevice(m->ranks[r].device) != hipSuccess) { m->err = "hipSetDevice"; return SBR_EDEVICE; }
    if (hipSetDevice(k0.device) != hipSuccess) { m->err = "hipSetDevice"; return SBR_EDEVICE; }
    if (grow(&k0.gather, &k0.gather_bytes, plan.gather_bytes() + 256)) { m->err = "gather buffer"; return SBR_ENOMEM; }
    const auto t2 = std::chrono::steady_clock::now();
    if (!rccl().ok) { m->err = rccl().err; return SBR_EDEVICE; }
    if (m->shared && N > 1) { m->err = "the RCCL gather needs distinct devices (shared-device rehearsal)"; return SBR_EARG; }
    if (N > 1 && !m->comms_ok) {
        int rc = init_comms(m, m->err);
        if (rc) return rc;
        (void)hipSetDevice(k0.device);
    }
    // phase 2: the RCCL gather of the packed blocks to rank 0 …
    {
        RcclTransport tr(m);
        std::vector<const void*> blocks;
        for (const Rank& k : m->ranks) blocks.push_back(k.out);
        const int rc = sbr_shard::gather(plan, tr, blocks, k0.gather);
        if (rc) { m->err = tr.err.empty() ? "gather" : tr.err; return rc; }
    }
    // … and the strided scatter into the caller's arrays
    if (hipSetDevice(k0.device) != hipSuccess) { m->err = "hipSetDevice"; return SBR_EDEVICE; }
    const int rc = sbr_shard::scatter(plan, fields, k0.gather,
                                      [&](void* d, size_t dp, const void* src, size_t sp, size_t w, size_t h) {
                                          return hipMemcpy2DAsync(d, dp, src, sp, w, h, hipMemcpyDeviceToHost,
                                                                  k0.stream) == hipSuccess ? 0 : SBR_EDEVICE;
                                      });
    if (rc) { m->err = "result copy"; return rc; }
    if (hipStreamSynchronize(k0.stream) != hipSuccess) { m->err = "result sync"; return SBR_EDEVICE; }
    m->ph[2] = ms_since(t2);
    m->ph[4] = ms_since(t_call);
    return SBR_OK;
}

}  // namespace sbr_multi_impl

// ---------------------------------------------------------------------------
// sbr_shard_host_run: the same plan / deal / pack / gather / scatter on host memory with the
// loopback transport, the per-rank sweep supplied by the caller (tests: the CPU oracle).
// ---------------------------------------------------------------------------
extern "C" int sbr_shard_host_run(int32_t n_ranks, int64_t n_col, int64_t n_u, int32_t n_fields, const int64_t* esz,
                                  const int64_t* per_pt, void* const* host_out, sbr_shard_compute_fn compute, void* user,
                                  int32_t rccl_gather)
{
    if (n_ranks <= 0 || n_col <= 0 || n_u <= 0 || n_fields <= 0 || !esz || !per_pt || !host_out || !compute)
        return SBR_EARG;
    std::vector<sbr_shard::Field> fields;
    for (int f = 0; f < n_fields; f++) {
        if (esz[f] <= 0 || per_pt[f] <= 0) return SBR_EARG;
        fields.push_back({host_out[f], (size_t)esz[f], (size_t)per_pt[f]});
    }
    const sbr_shard::Plan plan = sbr_shard::make_plan(n_ranks, n_col, n_u, fields);
    std::vector<std::vector<char>> blocks(n_ranks);
    std::vector<const void*> bp(n_ranks, nullptr);
    for (int r = 0; r < n_ranks; r++) {
        blocks[r].assign(plan.block_bytes(r) + 1, 0);
        bp[r] = blocks[r].data();
        if (plan.cols[r] == 0) continue;
        std::vector<int64_t> ids(plan.cols[r]);
        for (int64_t c = 0; c < plan.cols[r]; c++) ids[c] = sbr_shard::global_col(r, c, n_ranks);
        std::vector<void*> fp;
        for (size_t o : sbr_shard::field_offsets(plan, r, fields)) fp.push_back(blocks[r].data() + o);
        const int rc = compute(user, r, plan.cols[r], ids.data(), fp.data());
        if (rc) return rc;
    }
    if (!rccl_gather) { // direct transport: every rank copies its own block into the caller's arrays
        for (int r = 0; r < n_ranks; r++) {
            const int rc = sbr_shard::scatter_rank(plan, r, fields, blocks[r].data(), sbr_shard::host_copy2d);
            if (rc) return rc;
        }
        return SBR_OK;
    }
    std::vector<char> gathered(plan.gather_bytes() + 1, 0);
    sbr_shard::LoopbackTransport tr;
    int rc = sbr_shard::gather(plan, tr, bp, gathered.data());
    if (rc) return SBR_EARG;
    return sbr_shard::scatter(plan, fields, gathered.data(), sbr_shard::host_copy2d);
}
