// sbr_multi.hip — multi-GPU fan-out behind the C ABI (SURVEY.md §8(b) threading
// contract, §8(e) partitioning): an n-device context holds one single-device
// context per GPU; every host-pointer sweep on it
//   1. deals the β (or parameter) columns cyclically — column i to rank i mod N,
//      which balances the β-dependent knot counts and run lengths;
//   2. runs each shard on its own GPU from its own host thread (the single-device
//      *_dev entry points on a per-rank stream, inputs staged into that GPU's HBM);
//   3. after every shard has finished (no collective is entered unless all ranks
//      succeeded, so a failing rank cannot leave the others blocked), gathers the
//      packed result blocks to rank 0 with RCCL point-to-point (ncclSend/ncclRecv over
//      xGMI) — the only communication of the path;
//   4. rank 0 scatters the blocks into the caller's u-fastest arrays (strided
//      copies: column i of the grid is block row i / N of rank i mod N).
// Per-point results do not depend on the partitioning, so a multi-GPU sweep is
// bit-identical to a single-device one.  librccl.so.1 is loaded at run time
// (reusing an already-loaded copy, e.g. torch's), so libsbr has no link-time
// dependency on it.
#include <dlfcn.h>
#include <math.h>
#include <string.h>

#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/sbr.h"
#include "sbr_multi.h"

namespace {

struct Rccl {
    bool ok = false;
    std::string err;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
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
        r.Send = (decltype(r.Send))dlsym(h, "ncclSend");
        r.Recv = (decltype(r.Recv))dlsym(h, "ncclRecv");
        r.GroupStart = (decltype(r.GroupStart))dlsym(h, "ncclGroupStart");
        r.GroupEnd = (decltype(r.GroupEnd))dlsym(h, "ncclGroupEnd");
        r.GetErrorString = (decltype(r.GetErrorString))dlsym(h, "ncclGetErrorString");
        r.ok = r.CommInitAll && r.CommDestroy && r.Send && r.Recv && r.GroupStart && r.GroupEnd && r.GetErrorString;
        if (!r.ok) r.err = "librccl.so.1 lacks a required symbol";
    });
    return r;
}

// per-rank device state, kept across calls (grow-only)
struct Rank {
    int device = 0;
    sbr_ctx* kid = nullptr;
    hipStream_t stream = nullptr;
    ncclComm_t comm = nullptr;
    void* in = nullptr;     // staged inputs
    size_t in_bytes = 0;
    void* out = nullptr;    // packed result block
    size_t out_bytes = 0;
    void* gather = nullptr; // rank 0: every rank's block
    size_t gather_bytes = 0;
};

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
};

namespace sbr_multi_impl {

int create(int n_gpus, const int* devices, sbr_multi** out, std::vector<sbr_ctx*>& kids, std::string& err)
{
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || n_gpus <= 0 || n_gpus > ndev) {
        err = "n_gpus exceeds the visible HIP devices";
        return SBR_EDEVICE;
    }
    std::vector<int> dl(n_gpus);
    for (int r = 0; r < n_gpus; r++) {
        dl[r] = devices ? devices[r] : r;
        if (dl[r] < 0 || dl[r] >= ndev) { err = "device id out of range"; return SBR_EDEVICE; }
        for (int q = 0; q < r; q++)
            if (dl[q] == dl[r]) { err = "duplicate device id"; return SBR_EARG; }
    }
    const Rccl& R = rccl();
    if (!R.ok) { err = R.err; return SBR_EDEVICE; }
    sbr_multi* m = new sbr_multi();
    m->ranks.resize(n_gpus);
    std::vector<ncclComm_t> comms(n_gpus);
    ncclResult_t nr = R.CommInitAll(comms.data(), n_gpus, dl.data());
    if (nr != ncclSuccess) {
        err = std::string("ncclCommInitAll: ") + R.GetErrorString(nr);
        delete m;
        return SBR_EDEVICE;
    }
    for (int r = 0; r < n_gpus; r++) {
        Rank& k = m->ranks[r];
        k.device = dl[r];
        k.comm = comms[r];
        int rc = sbr_init(dl[r], &k.kid);
        if (rc == SBR_OK && (hipSetDevice(dl[r]) != hipSuccess ||
                             hipStreamCreateWithFlags(&k.stream, hipStreamNonBlocking) != hipSuccess))
            rc = SBR_EDEVICE;
        if (rc != SBR_OK) {
            err = "per-device context";
            destroy(m);
            return rc;
        }
        kids.push_back(k.kid);
    }
    *out = m;
    return SBR_OK;
}

void destroy(sbr_multi* m)
{
    if (!m) return;
    const Rccl& R = rccl();
    for (Rank& k : m->ranks) {
        (void)hipSetDevice(k.device);
        if (k.stream) (void)hipStreamSynchronize(k.stream);
        if (k.comm && R.ok) (void)R.CommDestroy(k.comm);
        for (void* p : {k.in, k.out, k.gather})
            if (p) (void)hipFree(p);
        if (k.stream) (void)hipStreamDestroy(k.stream);
        if (k.kid) (void)sbr_free(k.kid);
    }
    delete m;
}

int size(const sbr_multi* m) { return m ? (int)m->ranks.size() : 1; }

sbr_ctx* child(sbr_multi* m, int r) { return (m && r >= 0 && r < (int)m->ranks.size()) ? m->ranks[r].kid : nullptr; }

const char* last_error(const sbr_multi* m) { return m ? m->err.c_str() : ""; }

// One sweep over the ranks.  For rank r with cols_r columns:
//   stage(r, cols_r, in_dev, stream) -> int   stages its inputs into in_dev (device)
//   run(r, kid, stream, in_dev, out_fields)    enqueues the single-device sweep, writing
//                                              field f of the block at out_fields[f]
// Fields: result arrays of n_col·n_u·per_pt elements of esz bytes, u-fastest per column
// (host == nullptr: not requested, still computed if the kernel needs a buffer).
int run_sharded(sbr_multi* m, int64_t n_col, int64_t n_u, const std::vector<FieldSpec>& fields, size_t in_bytes,
                const StageFn& stage, const RunFn& run)
{
    const int N = (int)m->ranks.size();
    const Rccl& R = rccl();
    std::vector<int> rcs(N, SBR_OK);
    std::vector<std::string> errs(N);
    std::vector<int64_t> cols(N), off(N + 1, 0);
    for (int r = 0; r < N; r++) cols[r] = n_col > r ? (n_col - r + N - 1) / N : 0;
    size_t per_col = 0; // packed bytes per column
    for (const FieldSpec& f : fields) per_col += (size_t)n_u * f.per_pt * f.esz;
    for (int r = 0; r < N; r++) off[r + 1] = off[r] + cols[r];

    // phase 1: every shard on its GPU, to completion
    {
        std::vector<std::thread> th;
        for (int r = 0; r < N; r++)
            th.emplace_back([&, r] {
                Rank& k = m->ranks[r];
                if (cols[r] == 0) return;
                if (hipSetDevice(k.device) != hipSuccess) { rcs[r] = SBR_EDEVICE; errs[r] = "hipSetDevice"; return; }
                if (grow(&k.in, &k.in_bytes, in_bytes + 256) ||
                    grow(&k.out, &k.out_bytes, (size_t)cols[r] * per_col + 256)) {
                    rcs[r] = SBR_ENOMEM;
                    errs[r] = "rank buffers";
                    return;
                }
                int rc = stage(r, cols[r], k.in, k.stream);
                std::vector<void*> fp;
                size_t o = 0;
                for (const FieldSpec& f : fields) {
                    fp.push_back((char*)k.out + o);
                    o += (size_t)cols[r] * n_u * f.per_pt * f.esz;
                }
                if (rc == SBR_OK) rc = run(r, cols[r], k.kid, k.stream, k.in, fp);
                if (rc == SBR_OK && hipStreamSynchronize(k.stream) != hipSuccess) rc = SBR_EDEVICE;
                if (rc != SBR_OK) { rcs[r] = rc; errs[r] = sbr_last_error(k.kid); }
            });
        for (auto& t : th) t.join();
    }
    for (int r = 0; r < N; r++)
        if (rcs[r] != SBR_OK) {
            m->err = "rank " + std::to_string(r) + ": " + errs[r];
            return rcs[r];
        }

    // phase 2: RCCL gather of the packed blocks to rank 0, then rank 0 scatters to the host
    {
        Rank& k0 = m->ranks[0];
        if (hipSetDevice(k0.device) != hipSuccess) { m->err = "hipSetDevice"; return SBR_EDEVICE; }
        if (grow(&k0.gather, &k0.gather_bytes, (size_t)n_col * per_col + 256)) { m->err = "gather buffer"; return SBR_ENOMEM; }
        std::vector<std::thread> th;
        for (int r = 0; r < N; r++)
            th.emplace_back([&, r] {
                Rank& k = m->ranks[r];
                if (hipSetDevice(k.device) != hipSuccess) { rcs[r] = SBR_EDEVICE; errs[r] = "hipSetDevice"; return; }
                ncclResult_t nr = ncclSuccess;
                if (r == 0) {
                    if (cols[0] > 0 &&
                        hipMemcpyAsync(k.gather, k.out, (size_t)cols[0] * per_col, hipMemcpyDeviceToDevice, k.stream) !=
                            hipSuccess) {
                        rcs[r] = SBR_EDEVICE; errs[r] = "gather copy"; return;
                    }
                    nr = R.GroupStart();
                    for (int q = 1; q < N && nr == ncclSuccess; q++)
                        if (cols[q] > 0)
                            nr = R.Recv((char*)k.gather + (size_t)off[q] * per_col, (size_t)cols[q] * per_col, ncclUint8,
                                        q, k.comm, k.stream);
                    const ncclResult_t ne = R.GroupEnd();
                    if (nr == ncclSuccess) nr = ne;
                } else if (cols[r] > 0) {
                    nr = R.Send(k.out, (size_t)cols[r] * per_col, ncclUint8, 0, k.comm, k.stream);
                }
                if (nr != ncclSuccess) { rcs[r] = SBR_EDEVICE; errs[r] = std::string("rccl: ") + R.GetErrorString(nr); return; }
                if (hipStreamSynchronize(k.stream) != hipSuccess) { rcs[r] = SBR_EDEVICE; errs[r] = "gather sync"; }
            });
        for (auto& t : th) t.join();
        for (int r = 0; r < N; r++)
            if (rcs[r] != SBR_OK) {
                m->err = "rank " + std::to_string(r) + ": " + errs[r];
                return rcs[r];
            }
        // scatter: block row c of rank r is grid column r + c·N
        for (int r = 0; r < N; r++) {
            if (cols[r] == 0) continue;
            const char* blk = (const char*)k0.gather + (size_t)off[r] * per_col;
            size_t o = 0;
            for (const FieldSpec& f : fields) {
                const size_t row = (size_t)n_u * f.per_pt * f.esz;
                if (f.host) {
                    hipError_t e = hipMemcpy2DAsync((char*)f.host + (size_t)r * row, (size_t)N * row, blk + o, row, row,
                                                    (size_t)cols[r], hipMemcpyDeviceToHost, k0.stream);
                    if (e != hipSuccess) { m->err = "result copy"; return SBR_EDEVICE; }
                }
                o += (size_t)cols[r] * row;
            }
        }
        if (hipStreamSynchronize(k0.stream) != hipSuccess) { m->err = "result sync"; return SBR_EDEVICE; }
    }
    return SBR_OK;
}

}  // namespace sbr_multi_impl
