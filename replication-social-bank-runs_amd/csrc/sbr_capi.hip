// sbr_capi.hip — the extern "C" boundary of libsbr (declared in include/sbr.h).
//
// A context owns one HIP device, one stream and a grow-only HBM workspace
// (knot slabs sized n_beta × knot_capacity).  Host-pointer entry points stage
// inputs, run the device pipeline and copy results back synchronously;
// *_dev entry points only enqueue on the caller's stream.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sbr.h"
#include "../../include/sbr_detmath.h"
#include "sbr_hostcopy.h"
#include "sbr_kernels.h"
#include "sbr_multi.h"

// Event flags. Timing events only time (no system-scope cache writeback/invalidate when they
// complete); dependency events between this device's queues release to device scope.
constexpr unsigned kTimingEventFlags = hipEventDisableSystemFence;
constexpr unsigned kSyncEventFlags = hipEventDisableTiming | hipEventReleaseToDevice;



struct sbr_ctx {
    int device = 0;
    // n-device context (sbr_init_multi): the per-device contexts, RCCL communicator and
    // rank buffers live in `multi`; the host-pointer sweeps fan out over them
    sbr_multi* multi = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    // learning workspaces: slot 0 for single sweeps; a pipelined batch rotates through
    // kLearnSlots slots, each learned on its own highest-priority stream, so the
    // learning of the next kLearnSlots-1 batches (latency-bound: 32 waves each) runs
    // concurrently with the equilibrium of the current one
    // (workspace slots and streams are separate counts: grid k learns into slot k mod
    // kLearnSlots on stream k mod kLearnStreams)
    static constexpr int kLearnSlots = 3; // slot 0: single sweeps; slots 0, 1: batch groups
    static constexpr int kLearnStreams = 3; // learning streams (with the context stream: within GPU_MAX_HW_QUEUES = 4)
    // the hetero batch pipeline alternates two of these slots' streams/events; single sweeps
    // run their column chunks on the streams with slot events 0..kLearnStreams-1
    static_assert(kLearnStreams >= 2 && kLearnSlots >= kLearnStreams, "kLearnSlots >= kLearnStreams >= 2");
    size_t ws_beta[kLearnSlots] = {}, ws_cap[kLearnSlots] = {};
    sbr::LearnBufs LW[kLearnSlots]{};
    int last_slot = 0;
    int64_t last_off = 0; // column offset of the last grid inside its (grouped) learning slot
    hipStream_t lstream[kLearnStreams] = {};
    hipEvent_t ev_in = nullptr, ev_learned[kLearnSlots] = {}, ev_eq[kLearnSlots] = {};
    // fork/join fences between HIP's null stream and `stream`, and the end of the last call
    // (whatever stream it ran on) that every call waits for (CallFence)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_last = nullptr;
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    // hetero learning workspace; H2 is the second slot of a pipelined hetero batch
    size_t hs_col = 0, hs_cap = 0, hs_K = 0;
    sbr::HeteroBufs H{};
    size_t hs2_col = 0, hs2_cap = 0, hs2_K = 0;
    sbr::HeteroBufs H2{};
    // social-learning workspace (sbr_social.hip): per point 5 knot buffers + n_cmp
    size_t so_pts = 0, so_cap = 0, so_cmp = 0;
    double *so_ws = nullptr, *so_cmpo = nullptr, *so_xi = nullptr;
    int32_t *so_n_old = nullptr, *so_live = nullptr, *so_work[2] = {nullptr, nullptr}, *so_count = nullptr;
    uint32_t *so_slots = nullptr, *so_bits = nullptr;
    int64_t* so_steps = nullptr;
    // promotion pool (sbr::SocialPool); so_count = [list 0, list 1, pool used, pool live]
    size_t pl_slots = 0, pl_cap = 0, pl_cmp = 0;
    double *pl_ws = nullptr, *pl_cmpo = nullptr, *pl_xi = nullptr;
    int32_t *pl_n_old = nullptr, *pl_live = nullptr, *pl_it = nullptr, *pl_ready = nullptr;
    uint32_t *pl_perm = nullptr, *pl_bits = nullptr;
    int64_t *pl_steps = nullptr, *pl_pts = nullptr;
    int32_t* so_count_host = nullptr; // pinned
    double* het_aw_path = nullptr;      // set only inside sbr_hetero_point_paths
    double *so_path_t = nullptr, *so_path_G = nullptr, *so_path_aw = nullptr; // set only inside sbr_social_point_paths
    int32_t* so_path_n = nullptr;
    int32_t so_path_cap = 0;
    sbr::SocialArgs* so_args_dev = nullptr;  // {main, pool} arguments of the iterate kernel
    sbr::SocialArgs* so_args_host = nullptr; // pinned staging for them
    int64_t so_promoted = 0, so_rerun = 0; // last sweep: points promoted into the pool / re-run larger
    int64_t so_budget = 0;            // workspace bytes (0: 60 % of free HBM)
    int64_t* so_prof = nullptr;       // SBR_FLAG_DIAG_SOCIAL_PROF: [pts][8]
    size_t so_prof_pts = 0;
    std::vector<int64_t> so_prof_acc; // host sums over the chunks of the last sweep
    // host-API staging
    void* stage = nullptr;
    size_t stage_bytes = 0;
    // pinned landing buffer of the host-pointer sweeps' results: one DMA copy at full PCIe rate,
    // then a multi-threaded host copy into the caller's (pageable) arrays
    void* res_pin = nullptr;
    size_t res_pin_bytes = 0;
    // sbr_equilibrium_on_knots: the caller's knot grid and its hazard path stay resident between
    // calls, keyed by value (n, t, G and β, η, p, λ); the device block and its pinned host mirror
    // share one layout (KnotLayout), so each transfer is one contiguous copy
    char* kn_dev = nullptr;
    char* kn_pin = nullptr;
    size_t kn_cap_k = 0, kn_cap_u = 0;
    bool kn_valid = false;
    int64_t kn_n = 0;
    double kn_key[4] = {};
    std::vector<double> kn_t, kn_G, kn_hr; // host copies of the resident knots and HR
    std::vector<double> kn_pdf;            // sbr_equilibrium_on_knots_pdf's pdf values (empty: βG(1 − G))
    int32_t kn_m = 0, kn_ntau = 0;         // knots <= η; τ̄ entries (0: the hazard's BoundsError)
    // single-u calls: mapped, coherent host memory the kernel reads t_end / u from and writes the
    // results and paths to (no copy launches per call) — host view and device view
    double* kn_zc = nullptr;
    double* kn_zc_dev = nullptr;
    size_t kn_zc_cap = 0; // doubles
    // sbr_hetero_equilibrium_on_knots: the same for a LearningResultsHetero (knots, K group CDFs,
    // the K hazard paths), keyed by K, n, t, G, βs, dist, η, p, λ
    char* hk_dev = nullptr;
    char* hk_pin = nullptr;
    size_t hk_cap_k = 0, hk_cap_u = 0;
    bool hk_valid = false;
    int64_t hk_n = 0;
    int32_t hk_K = 0, hk_ntau = 0;
    std::vector<double> hk_key, hk_t, hk_G, hk_hr;
    int lds_cap = 0, lds_cap_b = 0;
    int lds_smem = 0;
    // kernel timing (HIP event pairs on the launching stream), opt-in via sbr_timing_enable
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<hipEvent_t> ev_grid; // per grid of the last baseline batch: results complete
    std::vector<hipEvent_t> ev_hn;   // per equilibrium launch of a baseline batch: its hazards normalised
    int64_t n_grid = 0;
    int64_t bt_budget = 0; // baseline batch learning workspaces, bytes (0: 40 % of free + held HBM)
    size_t ev_used = 0;
    struct TRec {
        int kind; // 0 learning (+ hazard), 1 equilibrium
        hipEvent_t a, b;
        int count; // launches the span covers (a pipelined batch times its equilibria as one span)
    };
    std::vector<TRec> trec;
    // phases of the last host-pointer baseline sweep while timing is enabled (sbr_host_phases):
    // H2D, kernels, D2H (HIP events on the stream), the early-exit post-pass and the whole call
    // (host clock), milliseconds
    double ph_ms[5] = {};
    // the last chunked single sweep while timing is enabled: per chunk, events at its learning
    // end and its equilibrium end, and the sweep start (sbr_chunk_timeline)
    hipEvent_t ck_start = nullptr;
    std::vector<hipEvent_t> ck_ev;
    // readiness schedule of single sweeps: the learning kernel and the equilibrium workgroups
    // on streams with disjoint CU masks (hipExtStreamCreateWithCUMask), and the publication
    // queue [head, err, tail, pad, q[n_beta], hz_flag[n_beta]]
    hipStream_t rs_learn = nullptr, rs_eq = nullptr;
    int rs_state = 0; // 0 untried, 1 available, -1 unavailable (chunked schedule instead)
    bool rs_used = false; // the last run_baseline took the readiness schedule
    int32_t* rq = nullptr;
    size_t rq_cap = 0;
    hipEvent_t ev_rin = nullptr, ev_rq = nullptr, ev_rl = nullptr, ev_re = nullptr;
};

namespace {

constexpr int kDefaultCap = 65536; // the longest Fig 5 tail (β ≈ 2000) needs 20k knots below η

int fail(sbr_ctx* c, int code, const char* what, hipError_t e = hipSuccess)
{
    if (c) {
        c->err = what;
        if (e != hipSuccess) { c->err += ": "; c->err += hipGetErrorString(e); }
    }
    return code;
}

#define HIP_TRY(ctx, expr, code)                                  \
    do {                                                          \
        hipError_t _e = (expr);                                   \
        if (_e != hipSuccess) return fail((ctx), (code), #expr, _e); \
    } while (0)

// Every entry point runs inside a CallFence:
//  * it is ordered after the previous call on this context, whatever stream that one used
//    (a *_dev call on a caller stream X followed by a host-pointer call on the private
//    stream would otherwise let the learning kernel rewrite LW[0] while X still reads it);
//  * a NULL stream argument of a *_dev entry point names HIP's null stream (torch's default
//    stream): the work runs on the context's non-blocking stream, fenced to the null stream
//    on both sides (it starts after earlier null-stream work, and null-stream work enqueued
//    after the call starts after it) without putting the kernels on the null stream's queue.
// Fence failures are reported (SBR_EDEVICE), never dropped.
struct CallFence {
    sbr_ctx* c;
    bool null_stream;
    hipStream_t s;
    CallFence(sbr_ctx* c_, void* stream, bool dev)
        : c(c_), null_stream(dev && stream == nullptr), s(dev && stream ? (hipStream_t)stream : c_->stream)
    {
    }
    int begin()
    {
        if (null_stream) {
            HIP_TRY(c, hipEventRecord(c->ev_fork, nullptr), SBR_EDEVICE);
            HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_fork, 0), SBR_EDEVICE);
        }
        if (c->have_last && c->last_stream != s) HIP_TRY(c, hipStreamWaitEvent(s, c->ev_last, 0), SBR_EDEVICE);
        return SBR_OK;
    }
    int end(int rc)
    {
        // recorded after a failure too: later calls still order after whatever was enqueued
        hipError_t e = hipEventRecord(c->ev_last, s);
        if (e == hipSuccess) {
            c->have_last = true;
            c->last_stream = s;
        }
        if (null_stream && e == hipSuccess) {
            e = hipEventRecord(c->ev_join, c->stream);
            if (e == hipSuccess) e = hipStreamWaitEvent(nullptr, c->ev_join, 0);
        }
        if (rc == SBR_OK && e != hipSuccess) return fail(c, SBR_EDEVICE, "stream fence", e);
        return rc;
    }
};

// run body(stream) inside a CallFence (dev: `stream` is a caller stream or NULL = null stream;
// host-pointer entry points pass dev = false and run on the private stream)
template <class F>
int fenced(sbr_ctx* c, void* stream, bool dev, F&& body)
{
    CallFence f(c, stream, dev);
    int rc = f.begin();
    if (rc) return rc;
    rc = body(f.s);
    return f.end(rc);
}

void free_learn(sbr_ctx* c, int slot)
{
    sbr::LearnBufs& L = c->LW[slot];
    void* ps[] = {L.t, L.G, L.hr, L.hrI, L.n_knots, L.n_tau, L.n_le, L.status, L.n_accept, L.n_reject};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    L = sbr::LearnBufs{};
    c->ws_beta[slot] = c->ws_cap[slot] = 0;
}

// Row stride of a learning workspace for a knot capacity: the capacity rounded up to a 128-B line
// plus one line.  A wave's 64 lanes each stream their own column's row; with a power-of-two
// stride (65536 knots = 512 KiB) all 64 rows map to the same L2 set and channel, the partial
// lines are evicted before they fill, and every 8-B knot store costs a memory write.
size_t learn_ld(size_t cap) { return ((cap + 15) & ~(size_t)15) + 16; }

int ensure_learn(sbr_ctx* c, size_t n_beta, size_t cap, int slot = 0, bool hri = false)
{
    if (n_beta <= c->ws_beta[slot] && cap == c->ws_cap[slot] && (!hri || c->LW[slot].hrI)) return SBR_OK;
    free_learn(c, slot);
    sbr::LearnBufs& L = c->LW[slot];
    const size_t ld = learn_ld(cap);
    const size_t slab = n_beta * ld * sizeof(double);
    HIP_TRY(c, hipMalloc(&L.t, slab), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&L.G, slab), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&L.hr, slab), SBR_ENOMEM);
    L.hrI = nullptr; // the hazard kernel scans in LDS; the fused hazard (batch) parks I here
    if (hri) HIP_TRY(c, hipMalloc(&L.hrI, slab), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&L.n_knots, n_beta * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&L.n_tau, n_beta * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&L.n_le, n_beta * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&L.status, n_beta * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&L.n_accept, n_beta * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&L.n_reject, n_beta * 4), SBR_ENOMEM);
    L.cap = (int32_t)ld;
    L.lim = (int32_t)cap;
    c->ws_beta[slot] = n_beta;
    c->ws_cap[slot] = cap;
    return SBR_OK;
}

void free_hetero_bufs(sbr::HeteroBufs& H, size_t& col, size_t& cap, size_t& K)
{
    void* ps[] = {H.t, H.G, H.hr, H.hrI, H.n_knots, H.n_tau, H.n_le, H.status, H.n_accept, H.n_reject};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    H = sbr::HeteroBufs{};
    col = cap = K = 0;
}

void free_hetero(sbr_ctx* c)
{
    free_hetero_bufs(c->H, c->hs_col, c->hs_cap, c->hs_K);
    free_hetero_bufs(c->H2, c->hs2_col, c->hs2_cap, c->hs2_K);
}

int ensure_hetero_bufs(sbr_ctx* c, sbr::HeteroBufs& H, size_t& hcol, size_t& hcap, size_t& hK, size_t n_col,
                       size_t cap, size_t K)
{
    if (n_col <= hcol && cap == hcap && K == hK) return SBR_OK;
    free_hetero_bufs(H, hcol, hcap, hK);
    const size_t ld = learn_ld(cap); // padded rows, as for the baseline workspaces
    HIP_TRY(c, hipMalloc(&H.t, n_col * ld * 8), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&H.G, n_col * ld * K * 8), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&H.hr, n_col * ld * K * 8), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&H.hrI, n_col * ld * K * 8), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&H.n_knots, n_col * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&H.n_tau, n_col * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&H.n_le, n_col * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&H.status, n_col * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&H.n_accept, n_col * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&H.n_reject, n_col * 4), SBR_ENOMEM);
    H.cap = (int32_t)ld;
    H.lim = (int32_t)cap;
    hcol = n_col;
    hcap = cap;
    hK = K;
    return SBR_OK;
}

int ensure_hetero(sbr_ctx* c, size_t n_col, size_t cap, size_t K)
{
    return ensure_hetero_bufs(c, c->H, c->hs_col, c->hs_cap, c->hs_K, n_col, cap, K);
}

void free_social(sbr_ctx* c)
{
    void* ps[] = {c->so_ws, c->so_cmpo, c->so_xi, c->so_n_old, c->so_live, c->so_work[0], c->so_work[1],
                  c->so_count, c->so_slots, c->so_bits, c->so_steps};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    c->so_ws = c->so_cmpo = c->so_xi = nullptr;
    c->so_n_old = c->so_live = c->so_work[0] = c->so_work[1] = c->so_count = nullptr;
    c->so_slots = c->so_bits = nullptr;
    c->so_steps = nullptr;
    c->so_pts = c->so_cap = c->so_cmp = 0;
}

int ensure_social(sbr_ctx* c, size_t pts, size_t cap, size_t n_cmp)
{
    if (pts <= c->so_pts && cap == c->so_cap && n_cmp <= c->so_cmp) return SBR_OK;
    free_social(c);
    // wave-blocked layout (sbr_social.hip BView): whole 64-point groups
    HIP_TRY(c, hipMalloc(&c->so_ws, ((pts + 63) / 64) * 64 * 5 * cap * 8), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->so_cmpo, pts * n_cmp * 8), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->so_xi, pts * 8), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->so_n_old, pts * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->so_live, pts * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->so_work[0], pts * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->so_work[1], pts * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->so_count, 8 * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->so_slots, pts * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->so_bits, pts * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->so_steps, pts * 8), SBR_ENOMEM);
    if (!c->so_count_host) HIP_TRY(c, hipHostMalloc(&c->so_count_host, 8 * 4), SBR_ENOMEM);
    if (!c->so_args_dev) HIP_TRY(c, hipMalloc(&c->so_args_dev, 2 * sizeof(sbr::SocialArgs)), SBR_ENOMEM);
    if (!c->so_args_host) HIP_TRY(c, hipHostMalloc(&c->so_args_host, 2 * sizeof(sbr::SocialArgs)), SBR_ENOMEM);
    c->so_pts = pts;
    c->so_cap = cap;
    c->so_cmp = n_cmp;
    return SBR_OK;
}

void free_pool(sbr_ctx* c)
{
    void* ps[] = {c->pl_ws, c->pl_cmpo, c->pl_xi, c->pl_n_old, c->pl_live, c->pl_it, c->pl_ready,
                  c->pl_perm, c->pl_bits, c->pl_steps, c->pl_pts};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    c->pl_ws = c->pl_cmpo = c->pl_xi = nullptr;
    c->pl_n_old = c->pl_live = c->pl_it = c->pl_ready = nullptr;
    c->pl_perm = c->pl_bits = nullptr;
    c->pl_steps = c->pl_pts = nullptr;
    c->pl_slots = c->pl_cap = c->pl_cmp = 0;
}

int ensure_pool(sbr_ctx* c, size_t slots, size_t cap, size_t n_cmp)
{
    if (slots <= c->pl_slots && cap == c->pl_cap && n_cmp <= c->pl_cmp) return SBR_OK;
    free_pool(c);
    slots = (slots + 63) & ~(size_t)63;
    HIP_TRY(c, hipMalloc(&c->pl_ws, slots * 5 * cap * 8), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->pl_cmpo, slots * n_cmp * 8), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->pl_xi, slots * 8), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->pl_n_old, slots * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->pl_live, slots * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->pl_it, slots * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->pl_ready, slots * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->pl_perm, slots * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->pl_bits, slots * 4), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->pl_steps, slots * 8), SBR_ENOMEM);
    HIP_TRY(c, hipMalloc(&c->pl_pts, slots * 8), SBR_ENOMEM);
    c->pl_slots = slots;
    c->pl_cap = cap;
    c->pl_cmp = n_cmp;
    return SBR_OK;
}

int ensure_stage(sbr_ctx* c, size_t bytes)
{
    if (bytes <= c->stage_bytes) return SBR_OK;
    if (c->stage) (void)hipFree(c->stage);
    c->stage = nullptr;
    c->stage_bytes = 0;
    HIP_TRY(c, hipMalloc(&c->stage, bytes), SBR_ENOMEM);
    c->stage_bytes = bytes;
    return SBR_OK;
}

int ensure_res_pin(sbr_ctx* c, size_t bytes)
{
    if (bytes <= c->res_pin_bytes) return SBR_OK;
    if (c->res_pin) (void)hipHostFree(c->res_pin);
    c->res_pin = nullptr;
    c->res_pin_bytes = 0;
    HIP_TRY(c, hipHostMalloc(&c->res_pin, bytes), SBR_ENOMEM);
    c->res_pin_bytes = bytes;
    return SBR_OK;
}

// ξ_guess (solver.jl:413,441) is honoured by sbr_equilibrium_on_knots, which solves on the caller's
// whole knot grid; the sweeps' truncated learning (DESIGN.md §Truncated learning) and the
// extensions' own bisections start at the reference's defaults, so they refuse a guess
bool guess_set(const sbr_opts* o) { return o && (o->flags & SBR_FLAG_XI_GUESS); }

// EconomicParameters / LearningParameters scalar checks (model.jl:31-35, 71-76)
bool scalars_valid(double x0, double p, double kappa, double lambda)
{
    return x0 >= 0.0 && p >= 0.0 && p <= 1.0 && kappa > 0.0 && kappa < 1.0 && lambda > 0.0;
}

sbr_opts resolve(const sbr_opts* o)
{
    sbr_opts r;
    sbr_default_opts(&r);
    if (o) {
        r = *o;
        // a zero field is the default (a zero-filled sbr_opts is the reference's defaults)
        if (!(r.ode_reltol > 0.0)) r.ode_reltol = 2.220446049250313e-16;
        if (!(r.ode_abstol > 0.0)) r.ode_abstol = 2.220446049250313e-16;
        if (r.knot_capacity <= 0) r.knot_capacity = kDefaultCap;
        if (r.ode_maxiters <= 0) r.ode_maxiters = SBR_DEFAULT_ODE_MAXITERS;
        // the device ODE loops count a solve's steps in int32 (sbr_ode.h OdeOut)
        if (r.ode_maxiters > INT32_MAX) r.ode_maxiters = INT32_MAX;
        if (r.bisect_max_iters <= 0) r.bisect_max_iters = 100;
        if (r.hetero_max_iters <= 0) r.hetero_max_iters = 500;
    }
    return r;
}

hipEvent_t next_event(sbr_ctx* c)
{
    if (c->ev_used == c->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, kTimingEventFlags) != hipSuccess) return nullptr;
        c->ev_pool.push_back(e);
    }
    return c->ev_pool[c->ev_used++];
}

hipEvent_t tstart(sbr_ctx* c, hipStream_t s)
{
    if (!c->timing) return nullptr;
    hipEvent_t e = next_event(c);
    if (e) (void)hipEventRecord(e, s);
    return e;
}

void tend(sbr_ctx* c, hipStream_t s, int kind, hipEvent_t a, int count = 1)
{
    if (!c->timing || !a) return;
    hipEvent_t e = next_event(c);
    if (!e) return;
    (void)hipEventRecord(e, s);
    c->trec.push_back({kind, a, e, count});
}

int launch_eq(sbr_ctx* c, hipStream_t s, const sbr::LearnBufs& L, const double* eta, const double* t_end,
              const double* u, int64_t n_beta, int64_t n_u, double kappa, const sbr_opts& o,
              const sbr::ResultSoA& out, double* aw_path, int group = 1, bool timed = true)
{
    sbr::EqArgs ea{kappa, (int32_t)n_u, o.bisect_max_iters, c->lds_cap_b, aw_path,
                   (o.flags & SBR_FLAG_EXHAUSTIVE) ? 1 : 0, (o.flags >> 8) & 7};
    ea.group = group;
    hipEvent_t t0 = timed ? tstart(c, s) : nullptr;
    if (aw_path && n_beta == 1 && n_u == 1) { // single point with its path: the whole workgroup on it
        ea.lds_cap = c->lds_cap;
        HIP_TRY(c, sbr::launch_point_coop(L, eta, t_end, u, ea, out, s), SBR_EDEVICE);
        tend(c, s, 1, t0);
        return SBR_OK;
    }
    HIP_TRY(c, sbr::launch_equilibrium(L, eta, t_end, u, ea, out, (int)n_beta, s), SBR_EDEVICE);
    tend(c, s, 1, t0);
    return SBR_OK;
}

// highest-priority learning streams + events of the pipelined batch sweeps
int ensure_pipe_streams(sbr_ctx* c)
{
    if (c->lstream[0]) return SBR_OK;
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi); // hi = greatest priority
    for (int k = 0; k < sbr_ctx::kLearnStreams; k++)
        HIP_TRY(c, hipStreamCreateWithPriority(&c->lstream[k], hipStreamNonBlocking, hi), SBR_EDEVICE);
    for (int k = 0; k < sbr_ctx::kLearnSlots; k++) {
        HIP_TRY(c, hipEventCreateWithFlags(&c->ev_learned[k], kSyncEventFlags), SBR_EDEVICE);
        HIP_TRY(c, hipEventCreateWithFlags(&c->ev_eq[k], kSyncEventFlags), SBR_EDEVICE);
    }
    HIP_TRY(c, hipEventCreateWithFlags(&c->ev_in, kSyncEventFlags), SBR_EDEVICE);
    return SBR_OK;
}

// Pipelined batch plan (sbr_sweep_baseline_batch_dev).  The learning kernel is latency-bound
// (one serial ODE per lane, ≈32 waves per 2048-column grid) and a launch lasts as long as its
// slowest column whatever its width; run beside the equilibrium kernel a learning wave holds
// an equilibrium workgroup slot of its CU (169 VGPRs next to 6 × 80) and issues ahead of it.
// So the batch learns as many grids as it can in ONE launch — up to SBR_BATCH_LEARN_WAVES waves,
// at most one per SIMD — while the chip has nothing else to do, and then runs the equilibria
// back to back with nothing beside them; a batch longer than that learns its next group into
// the second workspace beside the first group's equilibria.
#ifndef SBR_BATCH_LEARN_WAVES
#define SBR_BATCH_LEARN_WAVES 768 // learning waves per batch learning launch (of 1,024 SIMDs)
#endif
#ifndef SBR_BATCH_EQ_COLS
#define SBR_BATCH_EQ_COLS 4096 // columns per equilibrium launch of a batch (two full grids: one tail per two)
#endif
struct BatchPlan {
    int64_t L = 1;  // grids per learning launch (and workspace slot)
    int64_t E = 1;  // grids per equilibrium launch
    int nslot = 1;  // workspace slots in rotation (1 when one group holds the batch, else 2)
};

// bytes of one learning column of a batch workspace: t, G, the HR numerators and the running
// integrals (cap doubles each) and six counters
size_t batch_col_bytes(size_t cap) { return learn_ld(cap) * 4 * sizeof(double) + 6 * sizeof(int32_t); }

// Size the plan and its workspaces.  L is capped by the wave budget and by the memory budget
// (c->bt_budget, default 40 % of the free plus the already held HBM); if an allocation fails
// anyway the slots are released and L is halved, down to one grid (then SBR_ENOMEM).
int batch_alloc(sbr_ctx* c, int64_t n_batch, int64_t n_beta, size_t cap, BatchPlan& P)
{
    const int64_t wpg = (n_beta + 63) / 64; // learning waves per grid
    int64_t L = SBR_BATCH_LEARN_WAVES / wpg;
    if (L < 1) L = 1;
    if (L > n_batch) L = n_batch;
    size_t freeb = 0, total = 0;
    (void)hipMemGetInfo(&freeb, &total);
    size_t held = 0;
    for (int k = 0; k < 2; k++) held += c->ws_beta[k] * batch_col_bytes(c->ws_cap[k]);
    const double budget = c->bt_budget > 0 ? (double)c->bt_budget : 0.4 * (double)(freeb + held);
    const double per_grid = (double)n_beta * (double)batch_col_bytes(cap);
    for (;;) {
        int nslot = n_batch > L ? 2 : 1;
        while (L > 1 && (double)(L * nslot) * per_grid > budget) {
            L = L > 2 ? (L + 1) / 2 : 1;
            nslot = n_batch > L ? 2 : 1;
        }
        // balanced groups: ⌈n_batch / L⌉ groups of (nearly) equal size
        const int64_t ng = (n_batch + L - 1) / L;
        L = (n_batch + ng - 1) / ng;
        nslot = ng > 1 ? 2 : 1;
        // launch columns are int32 in the kernels' arguments
        if (L * n_beta > INT32_MAX) return fail(c, SBR_EARG, "batch: n_beta too large for one learning launch");
        int rc = SBR_OK;
        for (int k = 0; k < nslot && rc == SBR_OK; k++) rc = ensure_learn(c, (size_t)(L * n_beta), cap, k, true);
        if (rc == SBR_OK) {
            P.L = L;
            P.nslot = nslot;
            int64_t E = (SBR_BATCH_EQ_COLS + n_beta - 1) / n_beta;
            P.E = E < 1 ? 1 : (E > L ? L : E);
            return SBR_OK;
        }
        for (int k = 0; k < sbr_ctx::kLearnSlots; k++) free_learn(c, k);
        if (L == 1) return rc;
        // the failed hipMalloc left hipErrorOutOfMemory as the thread's last error: clear it, or
        // the next launch check (hipGetLastError) would report it against a good launch
        (void)hipGetLastError();
        L = (L + 1) / 2;
    }
}

// the learning buffers / results of columns [c0, ...) of a sweep (row views)
sbr::LearnBufs learn_rows(const sbr::LearnBufs& L, size_t c0)
{
    const size_t k = c0 * (size_t)L.cap;
    return {L.t + k,        L.G + k,        L.hr + k,     L.hrI + k,         L.n_knots + c0, L.n_tau + c0,
            L.n_le + c0,    L.status + c0,  L.n_accept + c0, L.n_reject + c0, L.cap, L.lim};
}
sbr::ResultSoA result_rows(const sbr::ResultSoA& r, size_t off)
{
    auto at = [off](auto* p) { return p ? p + off : p; };
    return {at(r.xi), at(r.tau_in_unc), at(r.tau_out_unc), at(r.aw_max), at(r.tol), at(r.status), at(r.iters)};
}

// One sweep.  Every learning column is a serial ODE on one lane, and the launch lasts as long
// as its slowest column (config 3: one column takes 4.4k steps where the median takes 2.9k),
// while the equilibrium stage is a throughput kernel over the whole chip.  Wide sweeps are
// therefore cut into kSweepChunks column chunks, each learned and solved on its own learning
// stream: the equilibria of the chunks that finish learning early run while the slowest
// chunk is still integrating.  Timing records: kind 0 = the learning stage of all chunks
// (fork to the last chunk learned), kind 1 = the equilibrium tail after it.
constexpr int kSweepChunks = sbr_ctx::kLearnStreams;
// pipelined batch: hazard_rate streamed by the learning kernel (no separate hazard launch
// competing with the equilibrium kernel for CU slots); single sweeps keep the hazard kernel
constexpr int kSweepFront = 32;       // the front chunk of a single sweep: 1/32 of the waves (halving only: 4.44 vs 4.25 ms)
constexpr int kReadyLearnCus = 64;    // CUs reserved for the learning waves (8 / 16 / 32 / 64: 13.3 / 9.2 / 3.5 / 3.0 ms of learning)
constexpr int kReadyTileU = 4096;     // u values per equilibrium workgroup (768: three tiles of a config-3 column, 6.7 vs 5.5 ms)
constexpr int kReadySpin = 1 << 24;   // polls (≈ 0.5 µs each) before a waiting workgroup gives up: a bug guard

// the streams with disjoint CU masks and the queue of a readiness sweep
int ensure_ready(sbr_ctx* c, size_t n_beta)
{
    if (c->rs_state == 0) {
        c->rs_state = -1;
        int ncu = 0;
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device);
        if (ncu >= 4 * kReadyLearnCus) {
            std::vector<uint32_t> ml((size_t)(ncu + 31) / 32, 0u), me(ml.size(), 0u);
            for (int i = 0; i < ncu; i++) (i < kReadyLearnCus ? ml : me)[(size_t)i / 32] |= 1u << (i % 32);
            if (hipExtStreamCreateWithCUMask(&c->rs_learn, (uint32_t)ml.size(), ml.data()) == hipSuccess &&
                hipExtStreamCreateWithCUMask(&c->rs_eq, (uint32_t)me.size(), me.data()) == hipSuccess &&
                hipEventCreateWithFlags(&c->ev_rin, kSyncEventFlags) == hipSuccess &&
                hipEventCreateWithFlags(&c->ev_rq, kSyncEventFlags) == hipSuccess &&
                hipEventCreateWithFlags(&c->ev_rl, kSyncEventFlags) == hipSuccess &&
                hipEventCreateWithFlags(&c->ev_re, kSyncEventFlags) == hipSuccess)
                c->rs_state = 1;
        }
    }
    if (c->rs_state != 1) return SBR_EDEVICE;
    const size_t need = 4 + 2 * n_beta;
    if (need > c->rq_cap) {
        if (c->rq) (void)hipFree(c->rq);
        c->rq = nullptr;
        c->rq_cap = 0;
        HIP_TRY(c, hipMalloc(&c->rq, need * 4), SBR_ENOMEM);
        c->rq_cap = need;
    }
    return SBR_OK;
}

// One sweep, readiness schedule (SBR_FLAG_READY_SWEEP): the learning kernel publishes every
// column the moment its lane has solved it (release), and one equilibrium workgroup per
// (column, u-tile) — in publication order, on the CUs the learning waves do not use — runs
// the column's hazard (tile 0) and equilibria (acquire).  Measured on config 3 it is slower
// than the chunked schedule (5.5 vs 4.3 ms): most columns' learning ends late (≈2.8k steps of
// a ≈4.4k-step maximum), so the equilibria cannot start much earlier, and they lose the
// learning CUs.  Timing records: kind 0 = the learning kernel, kind 1 = the equilibrium
// kernel (concurrent).
int run_baseline_ready(sbr_ctx* c, hipStream_t s, const double* beta, const double* eta, const double* t_end,
                       const double* u, int64_t n_beta, int64_t n_u, double kappa, const sbr_opts& o,
                       sbr::LearnArgs la, const sbr::ResultSoA& out)
{
    const int tiles = (int)((n_u + kReadyTileU - 1) / kReadyTileU);
    int32_t* q = c->rq;
    HIP_TRY(c, hipEventRecord(c->ev_rin, s), SBR_EDEVICE);
    HIP_TRY(c, hipStreamWaitEvent(c->rs_learn, c->ev_rin, 0), SBR_EDEVICE);
    HIP_TRY(c, hipMemsetAsync(q, 0, (4 + 2 * (size_t)n_beta) * 4, c->rs_learn), SBR_EDEVICE);
    HIP_TRY(c, hipEventRecord(c->ev_rq, c->rs_learn), SBR_EDEVICE);
    HIP_TRY(c, hipStreamWaitEvent(c->rs_eq, c->ev_rq, 0), SBR_EDEVICE);
    la.fuse_hazard = 0;
    la.ready_tail = q + 2;
    la.ready_q = q + 4;
    hipEvent_t t0 = tstart(c, c->rs_learn);
    HIP_TRY(c, sbr::launch_learn_logistic(beta, eta, t_end, la, c->LW[0], c->rs_learn), SBR_EDEVICE);
    tend(c, c->rs_learn, 0, t0);
    sbr::EqArgs ea{kappa, (int32_t)n_u, o.bisect_max_iters, c->lds_cap_b, nullptr,
                   (o.flags & SBR_FLAG_EXHAUSTIVE) ? 1 : 0, (o.flags >> 8) & 7};
    sbr::ReadyArgs ra{q, q + 4, q + 4 + n_beta, (int32_t)(n_beta * tiles), tiles, kReadyTileU, kReadySpin};
    hipEvent_t t1 = tstart(c, c->rs_eq);
    HIP_TRY(c, sbr::launch_eq_ready(c->LW[0], beta, eta, t_end, u, la, ea, ra, out, 0, c->rs_eq), SBR_EDEVICE);
    tend(c, c->rs_eq, 1, t1);
    HIP_TRY(c, hipEventRecord(c->ev_rl, c->rs_learn), SBR_EDEVICE);
    HIP_TRY(c, hipEventRecord(c->ev_re, c->rs_eq), SBR_EDEVICE);
    HIP_TRY(c, hipStreamWaitEvent(s, c->ev_rl, 0), SBR_EDEVICE);
    HIP_TRY(c, hipStreamWaitEvent(s, c->ev_re, 0), SBR_EDEVICE);
    // a workgroup that gave up left its tile unwritten: mark the whole sweep on the device, so a
    // *_dev caller sees it in the results (the host-pointer entry point also returns SBR_EDEVICE)
    HIP_TRY(c, sbr::launch_ready_fail(q + 1, out, n_beta * n_u, s), SBR_EDEVICE);
    return SBR_OK;
}

int run_baseline(sbr_ctx* c, hipStream_t s, const double* beta, const double* eta, const double* t_end, double x0,
                 const double* u, int64_t n_beta, int64_t n_u, double p, double kappa, double lambda,
                 const sbr_opts& o, const sbr::ResultSoA& out, double* aw_path)
{
    int rc = ensure_learn(c, (size_t)n_beta, (size_t)o.knot_capacity);
    if (rc) return rc;
    c->last_slot = 0;
    c->last_off = 0;
    sbr::LearnArgs la{x0, o.ode_reltol, o.ode_abstol, p, lambda, o.ode_maxiters, (int32_t)n_beta, 1, 0};
    // per-column readiness on request (SBR_FLAG_READY_SWEEP): see above
    c->rs_used = !aw_path && n_beta >= 64 && (o.flags & SBR_FLAG_READY_SWEEP) &&
                 ensure_ready(c, (size_t)n_beta) == SBR_OK;
    if (c->rs_used) return run_baseline_ready(c, s, beta, eta, t_end, u, n_beta, n_u, kappa, o, la, out);
    if (aw_path || n_beta < 64 * kSweepChunks) {
        hipEvent_t t0 = tstart(c, s);
        HIP_TRY(c, sbr::launch_learn_logistic(beta, eta, t_end, la, c->LW[0], s), SBR_EDEVICE);
        tend(c, s, 0, t0);
        return launch_eq(c, s, c->LW[0], eta, t_end, u, n_beta, n_u, kappa, o, out, aw_path);
    }
    rc = ensure_pipe_streams(c);
    if (rc) return rc;
    // chunk boundaries on whole waves (64 columns), halving towards the front: the last chunk
    // gets half of the columns, the others 1/4, 1/8, ...  The longest learning columns of a
    // β-descending grid (Fig 5: large β, outliers of up to 1.5x the median steps) sit in the
    // front chunks, whose equilibria, last to start, then fill one round of workgroups.
    const int64_t waves = (n_beta + 63) / 64;
    int64_t lo[kSweepChunks + 1];
    lo[0] = 0;
    lo[kSweepChunks] = n_beta;
    for (int k = kSweepChunks - 1; k >= 1; k--) {
        const int64_t wk = waves >> (kSweepChunks - k); // waves before chunk k
        lo[k] = std::min<int64_t>(n_beta, std::max<int64_t>(wk * 64, (int64_t)k * 64));
    }
    // the front chunk is 1/kSweepFront of the waves (the Fig 5 grid's outliers sit in
    // its first wave: 1.25x the steps of the next slowest)
    lo[1] = std::min<int64_t>(lo[2] - 64, std::max<int64_t>(64, (waves / kSweepFront) * 64));
    HIP_TRY(c, hipEventRecord(c->ev_in, s), SBR_EDEVICE);
    hipEvent_t t0 = tstart(c, s);
    c->ck_start = c->timing ? t0 : nullptr;
    c->ck_ev.assign(c->timing ? 2 * kSweepChunks : 0, nullptr);
    for (int k = 0; k < kSweepChunks; k++) {
        hipStream_t ls = c->lstream[k];
        const int64_t c0 = lo[k], nb = lo[k + 1] - lo[k];
        HIP_TRY(c, hipStreamWaitEvent(ls, c->ev_in, 0), SBR_EDEVICE);
        if (nb <= 0) continue;
        sbr::LearnArgs lk = la;
        lk.n_beta = (int32_t)nb;
        const sbr::LearnBufs Lk = learn_rows(c->LW[0], (size_t)c0);
        HIP_TRY(c, sbr::launch_learn_logistic(beta + c0, eta + c0, t_end + c0, lk, Lk, ls), SBR_EDEVICE);
        if (c->timing) {
            c->ck_ev[2 * k] = next_event(c);
            if (c->ck_ev[2 * k]) (void)hipEventRecord(c->ck_ev[2 * k], ls);
        }
        HIP_TRY(c, hipEventRecord(c->ev_learned[k], ls), SBR_EDEVICE);
        sbr::EqArgs ea{kappa, (int32_t)n_u, o.bisect_max_iters, c->lds_cap_b, nullptr,
                       (o.flags & SBR_FLAG_EXHAUSTIVE) ? 1 : 0, (o.flags >> 8) & 7};
        HIP_TRY(c, sbr::launch_equilibrium(Lk, eta + c0, t_end + c0, u, ea, result_rows(out, (size_t)(c0 * n_u)),
                                           (int)nb, ls), SBR_EDEVICE);
        if (c->timing) {
            c->ck_ev[2 * k + 1] = next_event(c);
            if (c->ck_ev[2 * k + 1]) (void)hipEventRecord(c->ck_ev[2 * k + 1], ls);
        }
        HIP_TRY(c, hipEventRecord(c->ev_eq[k], ls), SBR_EDEVICE);
    }
    for (int k = 0; k < kSweepChunks; k++)
        if (lo[k + 1] > lo[k]) HIP_TRY(c, hipStreamWaitEvent(s, c->ev_learned[k], 0), SBR_EDEVICE);
    hipEvent_t t1 = tstart(c, s);
    tend(c, s, 0, t0);
    for (int k = 0; k < kSweepChunks; k++)
        if (lo[k + 1] > lo[k]) HIP_TRY(c, hipStreamWaitEvent(s, c->ev_eq[k], 0), SBR_EDEVICE);
    tend(c, s, 1, t1);
    return SBR_OK;
}

int run_interest(sbr_ctx* c, hipStream_t s, const double* beta, const double* eta, const double* t_end, double x0,
                 const double* u, int64_t n_beta, int64_t n_u, double p, double kappa, double lambda, double r,
                 double delta, const sbr_opts& o, const sbr::ResultSoA& out, int64_t* steps, double* aw_path = nullptr,
                 double* v_path = nullptr, int32_t* v_count = nullptr)
{
    int rc = ensure_learn(c, (size_t)n_beta, (size_t)o.knot_capacity);
    if (rc) return rc;
    c->last_slot = 0;
    c->last_off = 0;
    sbr::LearnArgs la{x0, o.ode_reltol, o.ode_abstol, p, lambda, o.ode_maxiters, (int32_t)n_beta, 1, 0};
    hipEvent_t t0 = tstart(c, s);
    HIP_TRY(c, sbr::launch_learn_logistic(beta, eta, t_end, la, c->LW[0], s), SBR_EDEVICE);
    tend(c, s, 0, t0);
    sbr::EqArgs ea{kappa, (int32_t)n_u, o.bisect_max_iters, c->lds_cap, aw_path,
                   (o.flags & SBR_FLAG_EXHAUSTIVE) ? 1 : 0, (o.flags >> 8) & 7};
    sbr::InterestArgs ia{r, delta, o.ode_reltol, o.ode_abstol, o.ode_maxiters, steps, v_path, v_count};
    t0 = tstart(c, s);
    HIP_TRY(c, sbr::launch_interest(c->LW[0], eta, t_end, u, ea, ia, out, (int)n_beta, s), SBR_EDEVICE);
    tend(c, s, 1, t0);
    return SBR_OK;
}

// EconomicParametersInterest / solve_value_function checks (interest_rate_model.jl:40-50,
// value_function_solver.jl:67-69)
bool interest_valid(double r, double delta) { return r >= 0.0 && delta > 0.0 && r < delta; }

int multi_sweep_social(sbr_ctx* c, const double* beta, const double* eta, double x0, const double* u, int64_t n_beta,
                       int64_t n_u, double p, double kappa, double lambda, const double* cmp_grid, int32_t n_cmp,
                       double tol, int32_t max_iter, const sbr_opts& o, sbr_result_soa* out, int32_t* fp_iters,
                       int64_t* rk_steps);
int multi_sweep_hetero(sbr_ctx* c, int32_t K, const double* betas, const double* dist, const double* eta,
                       const double* t_end, double x0, const double* u, int64_t n_col, int64_t n_u, double p,
                       double kappa, double lambda, const sbr_opts& o, sbr_result_soa* out, double* tau_in,
                       double* tau_out);
int multi_sweep_interest(sbr_ctx* c, const double* beta, const double* eta, const double* t_end, double x0,
                         const double* u, int64_t n_beta, int64_t n_u, double p, double kappa, double lambda, double r_,
                         double delta, const sbr_opts& o, sbr_result_soa* out, int64_t* rk_steps);
int multi_sweep_baseline(sbr_ctx* c, const double* beta, const double* eta, const double* t_end, double x0,
                         const double* u, int64_t n_beta, int64_t n_u, double p, double kappa, double lambda,
                         const sbr_opts& o, sbr_result_soa* out);

}  // namespace

// device-pointer entry points address one GPU's HBM: they need a single-device context
#define SBR_SINGLE_DEVICE(c)                                                                                \
    do {                                                                                                    \
        if ((c) && (c)->multi)                                                                              \
            return fail((c), SBR_EARG, "device-pointer entry points need a single-device context "          \
                                       "(sbr_multi_child)");                                                \
    } while (0)
// per-device diagnostics (timings, learning statistics, social counters) describe one
// device's last sweep: on an n-device context they would report rank 0's shard as if it
// were the grid, so they are refused there — ask the rank's child context instead
#define SBR_PER_DEVICE_DIAG(c)                                                                              \
    do {                                                                                                    \
        if ((c) && (c)->multi)                                                                              \
            return fail((c), SBR_EARG, "per-device diagnostic: call it on sbr_multi_child(ctx, rank)");    \
    } while (0)
// single-point / diagnostic entry points on an n-device context run on its rank 0
#define SBR_ON_RANK0(c, call)                                                                               \
    do {                                                                                                    \
        if ((c) && (c)->multi) {                                                                            \
            sbr_ctx* const c0_ = sbr_multi_child((c), 0);                                                   \
            sbr_ctx* const parent_ = (c);                                                                   \
            sbr_ctx* c = c0_;                                                                               \
            const int rc_ = (call);                                                                         \
            parent_->err = rc_ ? std::string(sbr_last_error(c0_)) : std::string();                          \
            return rc_;                                                                                     \
        }                                                                                                   \
    } while (0)

hipStream_t sbr_ctx_stream(sbr_ctx* c) { return c ? c->stream : nullptr; }

extern "C" {

void sbr_default_opts(sbr_opts* o)
{
    o->ode_reltol = 2.220446049250313e-16;
    o->ode_abstol = 2.220446049250313e-16;
    o->ode_maxiters = SBR_DEFAULT_ODE_MAXITERS;
    o->bisect_max_iters = 100;
    o->early_exit_nan_run = 5;
    o->knot_capacity = kDefaultCap;
    o->hetero_max_iters = 500;
    o->flags = 0;
    o->pad = 0;
    o->xi_guess = __builtin_nan(""); // compute_ξ's default first iterate, the midpoint (solver.jl:309)
}

int sbr_init(int device, sbr_ctx** out)
{
    if (!out) return SBR_EARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return SBR_EDEVICE;
    sbr_ctx* c = new sbr_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork, kSyncEventFlags) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, kSyncEventFlags) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_last, kSyncEventFlags) != hipSuccess) {
        delete c;
        return SBR_EDEVICE;
    }
    int smem = 0;
    (void)hipDeviceGetAttribute(&smem, hipDeviceAttributeMaxSharedMemoryPerBlock, device);
    if (smem <= 0) smem = 65536;
    c->lds_smem = smem;
    // per 64 staged knots: t, G, HR (3·64) + HR block max/min (2) + their prefix/suffix tables (4)
    // + 8-knot G prefix-max/suffix-min (16); 1 KiB slack
    c->lds_cap = (int)(((long)(smem - 1024) * 64) / (8 * (3 * 64 + 6 + 16)));
    // baseline equilibrium kernel: t, G (2·64) + summaries per 64 knots, two workgroups per CU
    c->lds_cap_b = (int)(((long)(smem / 2 - 1024) * 64) / (8 * (2 * 64 + 6 + 16)));
    *out = c;
    return SBR_OK;
}

int sbr_init_multi(int n_gpus, const int* devices, sbr_ctx** out)
{
    if (!out) return SBR_EARG;
    *out = nullptr;
    if (n_gpus <= 0) return SBR_EARG;
    sbr_ctx* c = new sbr_ctx();
    std::vector<sbr_ctx*> kids;
    std::string err;
    const int rc = sbr_multi_impl::create(n_gpus, devices, &c->multi, kids, err);
    if (rc != SBR_OK) {
        delete c;
        return rc;
    }
    c->device = kids[0]->device;
    *out = c;
    return SBR_OK;
}

int sbr_multi_size(const sbr_ctx* c) { return c ? sbr_multi_impl::size(c->multi) : 0; }

sbr_ctx* sbr_multi_child(sbr_ctx* c, int rank)
{
    if (!c) return nullptr;
    if (!c->multi) return rank == 0 ? c : nullptr;
    return sbr_multi_impl::child(c->multi, rank);
}

int sbr_free(sbr_ctx* c)
{
    if (!c) return SBR_OK;
    if (c->multi) {
        sbr_multi_impl::destroy(c->multi);
        delete c;
        return SBR_OK;
    }
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (hipStream_t ls : c->lstream)
        if (ls) (void)hipStreamSynchronize(ls);
    for (int k = 0; k < sbr_ctx::kLearnSlots; k++) free_learn(c, k);
    free_hetero(c);
    free_social(c);
    free_pool(c);
    if (c->so_prof) (void)hipFree(c->so_prof);
    if (c->so_count_host) (void)hipHostFree(c->so_count_host);
    if (c->so_args_dev) (void)hipFree(c->so_args_dev);
    if (c->so_args_host) (void)hipHostFree(c->so_args_host);
    if (c->ev_in) (void)hipEventDestroy(c->ev_in);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->ev_last) (void)hipEventDestroy(c->ev_last);
    for (int k = 0; k < sbr_ctx::kLearnSlots; k++) {
        if (c->ev_learned[k]) (void)hipEventDestroy(c->ev_learned[k]);
        if (c->ev_eq[k]) (void)hipEventDestroy(c->ev_eq[k]);
    }
    for (int k = 0; k < sbr_ctx::kLearnStreams; k++)
        if (c->lstream[k]) (void)hipStreamDestroy(c->lstream[k]);
    for (hipStream_t rs : {c->rs_learn, c->rs_eq})
        if (rs) { (void)hipStreamSynchronize(rs); (void)hipStreamDestroy(rs); }
    for (hipEvent_t e : {c->ev_rin, c->ev_rq, c->ev_rl, c->ev_re})
        if (e) (void)hipEventDestroy(e);
    if (c->rq) (void)hipFree(c->rq);
    if (c->stage) (void)hipFree(c->stage);
    if (c->res_pin) (void)hipHostFree(c->res_pin);
    if (c->kn_dev) (void)hipFree(c->kn_dev);
    if (c->kn_pin) (void)hipHostFree(c->kn_pin);
    if (c->kn_zc) (void)hipHostFree(c->kn_zc);
    if (c->hk_dev) (void)hipFree(c->hk_dev);
    if (c->hk_pin) (void)hipHostFree(c->hk_pin);
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_grid) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_hn) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return SBR_OK;
}

const char* sbr_last_error(const sbr_ctx* c)
{
    // an n-device sweep's failure is copied into c->err by fail(); no fallback to the
    // multi layer's message, which would resurface after a later success
    return c ? c->err.c_str() : "null context";
}

int sbr_sweep_baseline_dev(sbr_ctx* c, void* stream, const double* beta, const double* eta, const double* t_end,
                           double x0, const double* u, int64_t n_beta, int64_t n_u, double p, double kappa,
                           double lambda, const sbr_opts* opts, sbr_result_soa* out)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_SINGLE_DEVICE(c);
    if (!c || !out || !out->xi || !out->tau_in_unc || !out->tau_out_unc || !out->aw_max || !out->tol || !out->status)
        return SBR_EARG;
    if (n_beta <= 0 || n_u <= 0 || n_beta > (1 << 30) || n_u > (1 << 30)) return fail(c, SBR_EARG, "grid size");
    if (!scalars_valid(x0, p, kappa, lambda)) return fail(c, SBR_EARG, "ArgumentError: x0/p/kappa/lambda");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    sbr::ResultSoA r{out->xi, out->tau_in_unc, out->tau_out_unc, out->aw_max, out->tol, out->status, out->iters};
    return fenced(c, stream, true, [&](hipStream_t s) {
        return run_baseline(c, s, beta, eta, t_end, x0, u, n_beta, n_u, p, kappa, lambda, o, r, nullptr);
    });
}

// hetero equilibrium LDS slab (doubles): knot times + per-group HR summaries of one column,
// capped so that SBR_HET_MINW = 2 workgroups share a CU's 160 KB (2 x (79.5 KB + the kernel's
// static LDS)); config 4 with Rosenbrock23 after the switch: n <= 7.9k knots
constexpr int kHetLds = 10176;
static int het_lds(const sbr_ctx* c) { return c->lds_cap * 3 < kHetLds ? c->lds_cap * 3 : kHetLds; }


int sbr_sweep_baseline_batch_dev(sbr_ctx* c, void* stream, int64_t n_batch, const double* beta, const double* eta,
                                 const double* t_end, double x0, const double* u, int64_t n_beta, int64_t n_u,
                                 double p, double kappa, double lambda, const sbr_opts* opts, sbr_result_soa* out)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_SINGLE_DEVICE(c);
    if (!c || !out || !beta || !eta || !t_end || !u) return SBR_EARG;
    if (!out->xi || !out->tau_in_unc || !out->tau_out_unc || !out->aw_max || !out->tol || !out->status) return SBR_EARG;
    if (n_batch <= 0 || n_beta <= 0 || n_u <= 0 || n_beta > (1 << 30) || n_u > (1 << 30))
        return fail(c, SBR_EARG, "grid size");
    if (!scalars_valid(x0, p, kappa, lambda)) return fail(c, SBR_EARG, "ArgumentError: x0/p/kappa/lambda");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    BatchPlan P;
    int rc = batch_alloc(c, n_batch, n_beta, (size_t)o.knot_capacity, P);
    if (rc) return rc;
    rc = ensure_pipe_streams(c);
    if (rc) return rc;
    const int64_t n_group = (n_batch + P.L - 1) / P.L;
    const int64_t n_eq_per_group = (P.L + P.E - 1) / P.E;
    while ((int64_t)c->ev_grid.size() < n_batch) {
        hipEvent_t e = nullptr;
        HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming), SBR_EDEVICE);
        c->ev_grid.push_back(e);
    }
    while ((int64_t)c->ev_hn.size() < n_group * n_eq_per_group) {
        hipEvent_t e = nullptr;
        HIP_TRY(c, hipEventCreateWithFlags(&e, kSyncEventFlags), SBR_EDEVICE);
        c->ev_hn.push_back(e);
    }
    c->n_grid = 0;
    return fenced(c, stream, true, [&](hipStream_t s) -> int {
        const size_t np = (size_t)n_beta * (size_t)n_u;
        // learning on lstream[0] (greatest priority), the hazard normalisations on lstream[1],
        // the equilibrium launches on the caller's stream
        hipStream_t ls = c->lstream[0], hs = c->lstream[1], es = s;
        HIP_TRY(c, hipEventRecord(c->ev_in, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamWaitEvent(ls, c->ev_in, 0), SBR_EDEVICE);
        int64_t k_hn = 0;
        for (int64_t m = 0; m < n_group; m++) {
            const int slot = (int)(m % P.nslot);
            const int64_t g0 = m * P.L, gn = (n_batch - g0) < P.L ? (n_batch - g0) : P.L;
            const sbr::LearnBufs& W = c->LW[slot];
            // the slot's previous readers (the equilibria of group m - nslot) must be done
            if (m >= P.nslot) HIP_TRY(c, hipStreamWaitEvent(ls, c->ev_eq[slot], 0), SBR_EDEVICE);
            // every grid of the group in ONE learning launch (the hazard numerators and running
            // integrals streamed with the knots, normalised by launch_hazard_norm): the launch
            // lasts as long as its slowest column whatever its width, so up to
            // SBR_BATCH_LEARN_WAVES waves learn together.  The first group has the chip to itself:
            // its rows leave through LDS as whole lines (mode 2).  Later groups run beside the
            // equilibrium launches and store directly (no LDS taken from the equilibrium slabs).
            const bool wide = m == 0;
            sbr::LearnArgs la{x0, o.ode_reltol, o.ode_abstol, p, lambda, o.ode_maxiters, (int32_t)(gn * n_beta), 1, 1};
            hipEvent_t t0 = tstart(c, ls);
            // (a narrow first group — under 256 waves, e.g. a strong-scaled shard — stores directly:
            // the staging's flush instructions cost more than the stores' contention there)
            const int lmode = !wide ? 0 : ((gn * n_beta + 63) / 64 >= 256 ? 2 : 1);
            // every grid's first wave dealt first (learn_logistic_kernel: the long columns of a
            // β-descending grid sit there; 20 grids 4.2-4.7 → 3.0-3.2 ms)
            if (lmode && n_beta % 64 == 0 && n_beta >= 128) {
                la.head = 1;
                la.wpg = (int32_t)(n_beta / 64);
            }
            // the staged heads-first launch normalises its tail waves' hazard rows itself; one small
            // hazard_norm_kernel launch takes the head waves' columns (no normalisation launches
            // beside the first equilibrium launch)
            const bool norm_in_learn = lmode == 2 && la.wpg;
            if (norm_in_learn) la.fuse_hazard = 2;
            HIP_TRY(c, sbr::launch_learn_kernel(beta + g0 * n_beta, eta + g0 * n_beta, t_end + g0 * n_beta, la, W, ls,
                                                lmode), SBR_EDEVICE);
            tend(c, ls, 0, t0);
            if (norm_in_learn) {
                sbr::LearnArgs lh = la;
                lh.part = 1;
                HIP_TRY(c, sbr::launch_hazard_norm(lh, W, (int)(gn * 64 * la.head), ls), SBR_EDEVICE);
            }
            HIP_TRY(c, hipEventRecord(c->ev_learned[slot], ls), SBR_EDEVICE);
            if (norm_in_learn) HIP_TRY(c, hipStreamWaitEvent(es, c->ev_learned[slot], 0), SBR_EDEVICE);
            else HIP_TRY(c, hipStreamWaitEvent(hs, c->ev_learned[slot], 0), SBR_EDEVICE);
            // the group's equilibria in launches of E grids (balanced).  Without the learning
            // kernel's own normalisation each launch follows a hazard_norm_kernel launch for its
            // columns on hs, run ahead and overlapped with the previous equilibrium launch — all of
            // them beside the first one, which they slowed from 2.28 to 2.71 ms (20 grids)
            const int64_t ne = (gn + P.E - 1) / P.E, Eg = (gn + ne - 1) / ne;
            // timing (sbr_timing_enable): one span over the group's equilibrium launches, from
            // the first one's start to the last one's end, counted as ne launches — two timing
            // events per launch between back-to-back launches cost ≈1 % of the step
            hipEvent_t te = nullptr;
            for (int64_t e0 = 0; e0 < gn; e0 += Eg) {
                const int64_t en = (gn - e0) < Eg ? (gn - e0) : Eg;
                const sbr::LearnBufs We = learn_rows(W, (size_t)(e0 * n_beta));
                const int64_t gg = g0 + e0;
                if (!norm_in_learn) {
                    HIP_TRY(c, sbr::launch_hazard_norm(la, We, (int)(en * n_beta), hs), SBR_EDEVICE);
                    hipEvent_t eh = c->ev_hn[(size_t)k_hn++];
                    HIP_TRY(c, hipEventRecord(eh, hs), SBR_EDEVICE);
                    HIP_TRY(c, hipStreamWaitEvent(es, eh, 0), SBR_EDEVICE);
                }
                if (e0 == 0) te = tstart(c, es);
                // column i·n_beta + j of the launch is grid g0+e0+i's column j: eta / t_end and
                // every out field are [n_batch × n_beta (× n_u)] contiguous
                sbr::ResultSoA r{out->xi + gg * np, out->tau_in_unc + gg * np, out->tau_out_unc + gg * np,
                                 out->aw_max + gg * np, out->tol + gg * np, out->status + gg * np,
                                 out->iters ? out->iters + gg * np : nullptr};
                rc = launch_eq(c, es, We, eta + gg * n_beta, t_end + gg * n_beta, u, en * n_beta, n_u, kappa, o, r,
                               nullptr, (int)en, false);
                if (rc) return rc;
                for (int64_t i = 0; i < en; i++) HIP_TRY(c, hipEventRecord(c->ev_grid[gg + i], es), SBR_EDEVICE);
                c->n_grid = gg + en;
            }
            tend(c, es, 1, te, (int)ne);
            HIP_TRY(c, hipEventRecord(c->ev_eq[slot], es), SBR_EDEVICE);
            c->last_slot = slot;
            c->last_off = (gn - 1) * n_beta;
        }
        return SBR_OK;
    });
}

int sbr_batch_reserve(sbr_ctx* c, int64_t n_batch, int64_t n_beta, const sbr_opts* opts)
{
    SBR_SINGLE_DEVICE(c);
    if (!c) return SBR_EARG;
    if (n_batch <= 0 || n_beta <= 0 || n_beta > (1 << 30)) return fail(c, SBR_EARG, "grid size");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    const sbr_opts o = resolve(opts);
    // the workspaces are replaced only once nothing enqueued earlier can still read them
    if (c->have_last) HIP_TRY(c, hipEventSynchronize(c->ev_last), SBR_EDEVICE);
    BatchPlan P;
    return batch_alloc(c, n_batch, n_beta, (size_t)o.knot_capacity, P);
}

int sbr_set_batch_workspace(sbr_ctx* c, int64_t bytes)
{
    SBR_SINGLE_DEVICE(c);
    if (!c || bytes < 0) return SBR_EARG;
    c->bt_budget = bytes;
    return SBR_OK;
}

int sbr_batch_wait(sbr_ctx* c, void* stream, int64_t k)
{
    SBR_SINGLE_DEVICE(c);
    if (!c) return SBR_EARG;
    if (k < 0 || k >= c->n_grid) return fail(c, SBR_EARG, "sbr_batch_wait: no such grid in the last batch");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    HIP_TRY(c, hipStreamWaitEvent((hipStream_t)stream, c->ev_grid[k], 0), SBR_EDEVICE);
    return SBR_OK;
}

int sbr_sweep_baseline(sbr_ctx* c, const double* beta, const double* eta, const double* t_end, double x0,
                       const double* u, int64_t n_beta, int64_t n_u, double p, double kappa, double lambda,
                       const sbr_opts* opts, sbr_result_soa* out)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    if (!c || !out || !beta || !eta || !t_end || !u) return SBR_EARG;
    if (n_beta <= 0 || n_u <= 0) return fail(c, SBR_EARG, "grid size");
    if (!scalars_valid(x0, p, kappa, lambda)) return fail(c, SBR_EARG, "ArgumentError: x0/p/kappa/lambda");
    for (int64_t i = 0; i < n_beta; i++)
        if (!(beta[i] > 0.0) || !(t_end[i] > 0.0) || !(eta[i] > 0.0))
            return fail(c, SBR_EARG, "ArgumentError: beta/eta/t_end must be positive");
    for (int64_t j = 0; j < n_u; j++)
        if (!(u[j] >= 0.0)) return fail(c, SBR_EARG, "ArgumentError: u must be non-negative");
    if (c->multi) return multi_sweep_baseline(c, beta, eta, t_end, x0, u, n_beta, n_u, p, kappa, lambda, resolve(opts), out);
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    const size_t np = (size_t)n_beta * (size_t)n_u;
    const size_t in_bytes = (3 * (size_t)n_beta + (size_t)n_u) * 8;
    const size_t out_bytes = np * (5 * 8 + 4 + 4);
    int rc = ensure_stage(c, in_bytes + out_bytes + 256);
    if (rc) return rc;
    char* base = (char*)c->stage;
    double* dbeta = (double*)base;
    double* deta = dbeta + n_beta;
    double* dtend = deta + n_beta;
    double* du = dtend + n_beta;
    double* dres = (double*)(base + ((in_bytes + 255) & ~(size_t)255));
    sbr::ResultSoA r{dres, dres + np, dres + 2 * np, dres + 3 * np, dres + 4 * np, (uint32_t*)(dres + 5 * np),
                     (int32_t*)((uint32_t*)(dres + 5 * np) + np)};
    rc = ensure_res_pin(c, out_bytes);
    if (rc) return rc;
    const auto h0 = std::chrono::steady_clock::now();
    hipEvent_t pe[4] = {};
    return fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        if (c->timing)
            for (hipEvent_t& e : pe) e = next_event(c);
        auto mark = [&](int k) { if (pe[k]) (void)hipEventRecord(pe[k], s); };
        mark(0);
        HIP_TRY(c, hipMemcpyAsync(dbeta, beta, n_beta * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(deta, eta, n_beta * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(dtend, t_end, n_beta * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(du, u, n_u * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        mark(1);
        rc = run_baseline(c, s, dbeta, deta, dtend, x0, du, n_beta, n_u, p, kappa, lambda, o, r, nullptr);
        if (rc) return rc;
        mark(2);
        // the result SoA is one contiguous block on the device: one DMA copy into pinned memory,
        // then the fields into the caller's arrays on several host threads
        int32_t gave_up = 0;
        if (c->rs_used) HIP_TRY(c, hipMemcpyAsync(&gave_up, c->rq + 1, 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        const size_t blk = np * (5 * 8 + 4 + (out->iters ? 4 : 0));
        HIP_TRY(c, hipMemcpyAsync(c->res_pin, dres, blk, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        mark(3);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        if (gave_up) return fail(c, SBR_EDEVICE, "readiness schedule: an equilibrium workgroup timed out");
        const auto h1 = std::chrono::steady_clock::now();
        {
            const char* P = (const char*)c->res_pin;
            std::vector<std::array<size_t, 3>> pieces;
            double* hs[5] = {out->xi, out->tau_in_unc, out->tau_out_unc, out->aw_max, out->tol};
            for (int k = 0; k < 5; k++)
                if (hs[k]) pieces.push_back({(size_t)hs[k], (size_t)(P + (size_t)k * np * 8), np * 8});
            if (out->status) pieces.push_back({(size_t)out->status, (size_t)(P + 5 * np * 8), np * 4});
            if (out->iters) pieces.push_back({(size_t)out->iters, (size_t)(P + 5 * np * 8 + np * 4), np * 4});
            sbr_host::parallel_copy(pieces);
        }
        if (o.early_exit_nan_run > 0 && out->status && out->xi && out->aw_max && out->tol)
            sbr_apply_early_exit(n_beta, n_u, o.early_exit_nan_run, out);
        if (pe[3]) {
            float a = 0.f;
            for (int k = 0; k < 3; k++)
                c->ph_ms[k] = hipEventElapsedTime(&a, pe[k], pe[k + 1]) == hipSuccess ? (double)a : -1.0;
            const auto h2 = std::chrono::steady_clock::now();
            c->ph_ms[3] = std::chrono::duration<double, std::milli>(h2 - h1).count();
            c->ph_ms[4] = std::chrono::duration<double, std::milli>(h2 - h0).count();
        }
        return SBR_OK;
    });
}

int sbr_sweep_interest_dev(sbr_ctx* c, void* stream, const double* beta, const double* eta, const double* t_end,
                           double x0, const double* u, int64_t n_beta, int64_t n_u, double p, double kappa,
                           double lambda, double r, double delta, const sbr_opts* opts, sbr_result_soa* out,
                           int64_t* rk_steps)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_SINGLE_DEVICE(c);
    if (!c || !out || !out->xi || !out->tau_in_unc || !out->tau_out_unc || !out->aw_max || !out->tol || !out->status)
        return SBR_EARG;
    if (n_beta <= 0 || n_u <= 0 || n_beta > (1 << 30) || n_u > (1 << 30)) return fail(c, SBR_EARG, "grid size");
    if (!scalars_valid(x0, p, kappa, lambda)) return fail(c, SBR_EARG, "ArgumentError: x0/p/kappa/lambda");
    if (!interest_valid(r, delta)) return fail(c, SBR_EARG, "ArgumentError: need 0 <= r < delta");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    sbr::ResultSoA rs{out->xi, out->tau_in_unc, out->tau_out_unc, out->aw_max, out->tol, out->status, out->iters};
    return fenced(c, stream, true, [&](hipStream_t s) {
        return run_interest(c, s, beta, eta, t_end, x0, u, n_beta, n_u, p, kappa, lambda, r, delta, o, rs, rk_steps);
    });
}

int sbr_sweep_interest(sbr_ctx* c, const double* beta, const double* eta, const double* t_end, double x0,
                       const double* u, int64_t n_beta, int64_t n_u, double p, double kappa, double lambda, double r,
                       double delta, const sbr_opts* opts, sbr_result_soa* out, int64_t* rk_steps)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    if (!c || !out || !beta || !eta || !t_end || !u) return SBR_EARG;
    if (n_beta <= 0 || n_u <= 0) return fail(c, SBR_EARG, "grid size");
    if (!scalars_valid(x0, p, kappa, lambda)) return fail(c, SBR_EARG, "ArgumentError: x0/p/kappa/lambda");
    if (!interest_valid(r, delta)) return fail(c, SBR_EARG, "ArgumentError: need 0 <= r < delta");
    for (int64_t i = 0; i < n_beta; i++)
        if (!(beta[i] > 0.0) || !(t_end[i] > 0.0) || !(eta[i] > 0.0))
            return fail(c, SBR_EARG, "ArgumentError: beta/eta/t_end must be positive");
    for (int64_t j = 0; j < n_u; j++)
        if (!(u[j] >= 0.0)) return fail(c, SBR_EARG, "ArgumentError: u must be non-negative");
    if (c->multi)
        return multi_sweep_interest(c, beta, eta, t_end, x0, u, n_beta, n_u, p, kappa, lambda, r, delta, resolve(opts),
                                    out, rk_steps);
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    const size_t np = (size_t)n_beta * (size_t)n_u;
    const size_t in_bytes = (3 * (size_t)n_beta + (size_t)n_u) * 8;
    const size_t out_bytes = np * (5 * 8 + 4 + 4 + 8);
    int rc = ensure_stage(c, in_bytes + out_bytes + 256);
    if (rc) return rc;
    char* base = (char*)c->stage;
    double* dbeta = (double*)base;
    double* deta = dbeta + n_beta;
    double* dtend = deta + n_beta;
    double* du = dtend + n_beta;
    double* dres = (double*)(base + ((in_bytes + 255) & ~(size_t)255));
    int64_t* dsteps = (int64_t*)(dres + 5 * np);
    sbr::ResultSoA rs{dres, dres + np, dres + 2 * np, dres + 3 * np, dres + 4 * np, (uint32_t*)(dsteps + np),
                      (int32_t*)((uint32_t*)(dsteps + np) + np)};
    return fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        HIP_TRY(c, hipMemcpyAsync(dbeta, beta, n_beta * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(deta, eta, n_beta * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(dtend, t_end, n_beta * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(du, u, n_u * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        rc = run_interest(c, s, dbeta, deta, dtend, x0, du, n_beta, n_u, p, kappa, lambda, r, delta, o, rs, dsteps);
        if (rc) return rc;
        double* hs[5] = {out->xi, out->tau_in_unc, out->tau_out_unc, out->aw_max, out->tol};
        for (int k = 0; k < 5; k++)
            if (hs[k]) HIP_TRY(c, hipMemcpyAsync(hs[k], dres + k * np, np * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (out->status) HIP_TRY(c, hipMemcpyAsync(out->status, rs.status, np * 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (out->iters) HIP_TRY(c, hipMemcpyAsync(out->iters, rs.iters, np * 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (rk_steps) HIP_TRY(c, hipMemcpyAsync(rk_steps, dsteps, np * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        return SBR_OK;
    });
}

int sbr_interest_point_paths(sbr_ctx* c, double beta, double eta, double t_end, double x0, double u, double p,
                             double kappa, double lambda, double r, double delta, const sbr_opts* opts, double* res,
                             uint32_t* status, double* tau, double* hr, double* V, double* aw_cum, int64_t cap,
                             int64_t* n_tau, int64_t* n_v)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_ON_RANK0(c, sbr_interest_point_paths(c, beta, eta, t_end, x0, u, p, kappa, lambda, r, delta, opts, res, status, tau, hr, V, aw_cum, cap, n_tau, n_v));
    if (!c || !res || !status) return SBR_EARG;
    if (!scalars_valid(x0, p, kappa, lambda) || !(beta > 0) || !(eta > 0) || !(t_end > 0) || !(u >= 0))
        return fail(c, SBR_EARG, "ArgumentError");
    if (!interest_valid(r, delta)) return fail(c, SBR_EARG, "ArgumentError: need 0 <= r < delta");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    const size_t kc = (size_t)o.knot_capacity;
    int rc = ensure_stage(c, 4 * 8 + 5 * 8 + 8 + 8 + 2 * kc * 8 + 512);
    if (rc) return rc;
    double* d = (double*)c->stage;
    double hin[4] = {beta, eta, t_end, u};
    return fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        HIP_TRY(c, hipMemcpyAsync(d, hin, 32, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        double* dres = d + 4;
        uint32_t* dst = (uint32_t*)(dres + 5);
        int32_t* dnv = (int32_t*)(dres + 6);
        double* dpath = dres + 7;
        double* dv = dpath + kc;
        HIP_TRY(c, hipMemsetAsync(dnv, 0, 4, s), SBR_EDEVICE);
        sbr::ResultSoA rs{dres, dres + 1, dres + 2, dres + 3, dres + 4, dst, nullptr};
        rc = run_interest(c, s, d, d + 1, d + 2, x0, d + 3, 1, 1, p, kappa, lambda, r, delta, o, rs, nullptr, dpath,
                          r > 0.0 ? dv : nullptr, dnv);
        if (rc) return rc;
        HIP_TRY(c, hipMemcpyAsync(res, dres, 40, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(status, dst, 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        int32_t nt = 0, nle = 0, nv = 0;
        HIP_TRY(c, hipMemcpyAsync(&nt, c->LW[0].n_tau, 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(&nle, c->LW[0].n_le, 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(&nv, dnv, 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        if (r <= 0.0) nv = 0;
        if (n_tau) *n_tau = nt;
        if (n_v) *n_v = nv;
        if (nt > cap) return fail(c, SBR_EARG, "path capacity too small");
        if (tau) {
            HIP_TRY(c, hipMemcpy(tau, c->LW[0].t, (size_t)nle * 8, hipMemcpyDeviceToHost), SBR_EDEVICE);
            if (nt > nle) tau[nle] = eta;
        }
        if (hr) HIP_TRY(c, hipMemcpy(hr, c->LW[0].hr, (size_t)nt * 8, hipMemcpyDeviceToHost), SBR_EDEVICE);
        if (V && nv > 0) HIP_TRY(c, hipMemcpy(V, dv, (size_t)nv * 8, hipMemcpyDeviceToHost), SBR_EDEVICE);
        if (aw_cum) {
            if (*status & SBR_RUN) HIP_TRY(c, hipMemcpy(aw_cum, dpath, (size_t)nt * 8, hipMemcpyDeviceToHost), SBR_EDEVICE);
            else for (int i = 0; i < nt; i++) aw_cum[i] = NAN;
        }
        return SBR_OK;
    });
}

int sbr_learn_baseline(sbr_ctx* c, const double* beta, const double* eta, const double* t_end, double x0,
                       int64_t n_beta, int32_t stop_after_eta, const sbr_opts* opts, double* t_out, double* G_out,
                       int64_t cap, int32_t* n_knots, uint32_t* status)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_ON_RANK0(c, sbr_learn_baseline(c, beta, eta, t_end, x0, n_beta, stop_after_eta, opts, t_out, G_out, cap, n_knots, status));
    if (!c || !beta || !eta || !t_end || n_beta <= 0 || cap <= 0) return SBR_EARG;
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    if (cap < o.knot_capacity) o.knot_capacity = (int32_t)cap;
    int rc = ensure_learn(c, (size_t)n_beta, (size_t)o.knot_capacity);
    if (rc) return rc;
    rc = ensure_stage(c, 3 * (size_t)n_beta * 8);
    if (rc) return rc;
    double* dbeta = (double*)c->stage;
    double* deta = dbeta + n_beta;
    double* dtend = deta + n_beta;
    return fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        HIP_TRY(c, hipMemcpyAsync(dbeta, beta, n_beta * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(deta, eta, n_beta * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(dtend, t_end, n_beta * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        sbr::LearnArgs la{x0, o.ode_reltol, o.ode_abstol, 0.5, 1.0, o.ode_maxiters, (int32_t)n_beta, stop_after_eta, 0};
        HIP_TRY(c, sbr::launch_learn_logistic(dbeta, deta, dtend, la, c->LW[0], s), SBR_EDEVICE);
        const size_t w = (size_t)o.knot_capacity, ld = (size_t)c->LW[0].cap;
        if (t_out)
            HIP_TRY(c, hipMemcpy2DAsync(t_out, cap * 8, c->LW[0].t, ld * 8, w * 8, n_beta, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (G_out)
            HIP_TRY(c, hipMemcpy2DAsync(G_out, cap * 8, c->LW[0].G, ld * 8, w * 8, n_beta, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (n_knots) HIP_TRY(c, hipMemcpyAsync(n_knots, c->LW[0].n_knots, n_beta * 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (status) HIP_TRY(c, hipMemcpyAsync(status, c->LW[0].status, n_beta * 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        return SBR_OK;
    });
}

int sbr_solve_point_paths(sbr_ctx* c, double beta, double eta, double t_end, double x0, double u, double p,
                          double kappa, double lambda, const sbr_opts* opts, double* res, uint32_t* status,
                          double* tau, double* hr, double* aw_cum, int64_t cap, int64_t* n_tau)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_ON_RANK0(c, sbr_solve_point_paths(c, beta, eta, t_end, x0, u, p, kappa, lambda, opts, res, status, tau, hr, aw_cum, cap, n_tau));
    if (!c || !res || !status) return SBR_EARG;
    if (!scalars_valid(x0, p, kappa, lambda) || !(beta > 0) || !(eta > 0) || !(t_end > 0) || !(u >= 0))
        return fail(c, SBR_EARG, "ArgumentError");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    const size_t kc = (size_t)o.knot_capacity;
    int rc = ensure_stage(c, 4 * 8 + 5 * 8 + 8 + kc * 8 + 256);
    if (rc) return rc;
    double* d = (double*)c->stage;
    double hin[4] = {beta, eta, t_end, u};
    return fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        HIP_TRY(c, hipMemcpyAsync(d, hin, 32, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        double* dres = d + 4;
        uint32_t* dst = (uint32_t*)(dres + 5);
        double* dpath = dres + 6 + 1;
        sbr::ResultSoA r{dres, dres + 1, dres + 2, dres + 3, dres + 4, dst, nullptr};
        rc = run_baseline(c, s, d, d + 1, d + 2, x0, d + 3, 1, 1, p, kappa, lambda, o, r, dpath);
        if (rc) return rc;
        HIP_TRY(c, hipMemcpyAsync(res, dres, 40, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(status, dst, 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        int32_t nt = 0, nle = 0, nk = 0;
        HIP_TRY(c, hipMemcpyAsync(&nt, c->LW[0].n_tau, 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(&nle, c->LW[0].n_le, 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(&nk, c->LW[0].n_knots, 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        if (n_tau) *n_tau = nt;
        if (nt > cap) return fail(c, SBR_EARG, "path capacity too small");
        if (tau) {
            HIP_TRY(c, hipMemcpy(tau, c->LW[0].t, (size_t)nle * 8, hipMemcpyDeviceToHost), SBR_EDEVICE);
            if (nt > nle) tau[nle] = eta;
        }
        if (hr) HIP_TRY(c, hipMemcpy(hr, c->LW[0].hr, (size_t)nt * 8, hipMemcpyDeviceToHost), SBR_EDEVICE);
        if (aw_cum) {
            if (*status & SBR_RUN) HIP_TRY(c, hipMemcpy(aw_cum, dpath, (size_t)nt * 8, hipMemcpyDeviceToHost), SBR_EDEVICE);
            else for (int i = 0; i < nt; i++) aw_cum[i] = NAN;
        }
        (void)nk;
        return SBR_OK;
    });
}

}  // extern "C"

namespace {

// byte offsets of sbr_equilibrium_on_knots' device block (and of its pinned mirror) for ck knots
// and cu u values: [counters | β, η | t, G, pdf (packed by the call's n) | HR | t_end, u | results,
// paths]
struct KnotLayout {
    size_t sc, tg, hr, u, res, bytes;
    KnotLayout(size_t ck, size_t cu)
    {
        sc = 64;
        tg = 128;
        hr = tg + 24 * ck;
        u = hr + 8 * (ck + 8);
        res = u + 8 * (cu + 8);
        bytes = res + 8 * (6 * cu + 3 * (ck + 1)) + 256;
    }
};

int ensure_knots(sbr_ctx* c, size_t n, size_t n_u)
{
    if (n <= c->kn_cap_k && n_u <= c->kn_cap_u) return SBR_OK;
    size_t ck = c->kn_cap_k > 4096 ? c->kn_cap_k : 4096, cu = c->kn_cap_u > 64 ? c->kn_cap_u : 64;
    while (ck < n) ck *= 2;
    while (cu < n_u) cu *= 2;
    // each buffer freed once and nulled (a second hipHostFree of the same pointer leaves a sticky
    // error that the next HIP_TRY reports against an unrelated launch)
    if (c->kn_dev) (void)hipFree(c->kn_dev);
    if (c->kn_pin) (void)hipHostFree(c->kn_pin);
    if (c->kn_zc) (void)hipHostFree(c->kn_zc);
    c->kn_dev = c->kn_pin = nullptr;
    c->kn_zc = c->kn_zc_dev = nullptr;
    c->kn_cap_k = c->kn_cap_u = 0;
    c->kn_valid = false;
    const KnotLayout K(ck, cu);
    HIP_TRY(c, hipMalloc(&c->kn_dev, K.bytes), SBR_ENOMEM);
    HIP_TRY(c, hipHostMalloc(&c->kn_pin, K.bytes), SBR_ENOMEM);
    c->kn_cap_k = ck;
    c->kn_cap_u = cu;
    // [t_end, u, results (8 doubles), AW_cum / AW_OUT / AW_IN (ck + 1 each)]
    const size_t zc = 16 + 3 * (ck + 1);
    HIP_TRY(c, hipHostMalloc(&c->kn_zc, zc * 8, hipHostMallocMapped | hipHostMallocCoherent), SBR_ENOMEM);
    HIP_TRY(c, hipHostGetDevicePointer((void**)&c->kn_zc_dev, c->kn_zc, 0), SBR_EDEVICE);
    c->kn_zc_cap = zc;
    return SBR_OK;
}

// sbr_hetero_equilibrium_on_knots' device block (and pinned mirror) for ck knots, cu u values and
// K <= 8 groups: [counters | βs, dist, η | t, G packed by the call's n | HR, I (K·ck each) |
// t_end, u | results, buffers, AW_total path]
struct HeteroKnotLayout {
    size_t sc, tg, hr, hri, u, res, bytes;
    HeteroKnotLayout(size_t ck, size_t cu)
    {
        sc = 64;
        tg = 256;
        hr = tg + 8 * ck * 9;
        hri = hr + 8 * ck * 8;
        u = hri + 8 * ck * 8;
        res = u + 8 * (cu + 8);
        bytes = res + 8 * (5 * cu + 16 * cu + 17 * ck) + 256; // path mode: AW_total + 2K group rows
    }
};

// path mode's rows (AW_total, then AW_OUT_k and AW_IN_k, each n long) into the caller's
// aw_total [n] and aw_groups [2K][cap]; NaN rows without a run (get_AW_hetero returns nothing)
void copy_hetero_paths(const double* src, bool run, int K, int64_t n, int64_t cap, double* aw_total,
                       double* aw_groups)
{
    for (int r = 0; r <= 2 * K; r++) {
        double* dst = r == 0 ? aw_total : (aw_groups ? aw_groups + (size_t)(r - 1) * cap : nullptr);
        if (!dst) continue;
        if (run) memcpy(dst, src + (size_t)r * n, (size_t)n * 8);
        else for (int64_t i = 0; i < n; i++) dst[i] = NAN;
    }
}

int ensure_hetero_knots(sbr_ctx* c, size_t n, size_t n_u)
{
    if (n <= c->hk_cap_k && n_u <= c->hk_cap_u) return SBR_OK;
    size_t ck = c->hk_cap_k > 8192 ? c->hk_cap_k : 8192, cu = c->hk_cap_u > 64 ? c->hk_cap_u : 64;
    while (ck < n) ck *= 2;
    while (cu < n_u) cu *= 2;
    if (c->hk_dev) (void)hipFree(c->hk_dev);
    if (c->hk_pin) (void)hipHostFree(c->hk_pin);
    c->hk_dev = c->hk_pin = nullptr;
    c->hk_cap_k = c->hk_cap_u = 0;
    c->hk_valid = false;
    const HeteroKnotLayout Lh(ck, cu);
    HIP_TRY(c, hipMalloc(&c->hk_dev, Lh.bytes), SBR_ENOMEM);
    HIP_TRY(c, hipHostMalloc(&c->hk_pin, Lh.bytes), SBR_ENOMEM);
    c->hk_cap_k = ck;
    c->hk_cap_u = cu;
    return SBR_OK;
}

}  // namespace

extern "C" {

int sbr_hetero_equilibrium_on_knots(sbr_ctx* c, int32_t K, const double* t, const double* G, int64_t n,
                                    const double* betas, const double* dist, double eta, double t_end, const double* u,
                                    int64_t n_u, double p, double kappa, double lambda, const sbr_opts* opts,
                                    sbr_result_soa* out, double* tau_in, double* tau_out, double* hr, double* aw_total,
                                    double* aw_groups, int64_t cap, int64_t* n_tau)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_ON_RANK0(c, sbr_hetero_equilibrium_on_knots(c, K, t, G, n, betas, dist, eta, t_end, u, n_u, p, kappa, lambda, opts, out, tau_in, tau_out, hr, aw_total, aw_groups, cap, n_tau));
    if (!c || !t || !G || !betas || !dist || !u || !out) return SBR_EARG;
    if (K != 1 && K != 2 && K != 3 && K != 4 && K != 8) return fail(c, SBR_EARG, "K must be 1, 2, 3, 4 or 8");
    if (n < 1 || n > (1 << 24) || n_u < 1 || n_u > (1 << 24)) return fail(c, SBR_EARG, "knot / u count");
    double dsum = 0.0;
    for (int k = 0; k < K; k++) {
        if (!(dist[k] >= 0.0)) return fail(c, SBR_EARG, "ArgumentError: distribution weights must be non-negative");
        if (!(betas[k] > 0.0)) return fail(c, SBR_EARG, "ArgumentError: all learning rates must be positive");
        dsum = dsum + dist[k];
    }
    if (!(fabs(dsum - 1.0) < 1e-10)) return fail(c, SBR_EARG, "ArgumentError: distribution must sum to 1");
    if (!scalars_valid(0.0, p, kappa, lambda) || !(eta > 0) || !(t_end > 0))
        return fail(c, SBR_EARG, "ArgumentError: eta/t_end/p/kappa/lambda");
    for (int64_t j = 0; j < n_u; j++)
        if (!(u[j] >= 0.0)) return fail(c, SBR_EARG, "ArgumentError: u must be non-negative");
    if (!(t[0] == t[0])) return fail(c, SBR_EARG, "ArgumentError: knots must be sorted");
    for (int64_t i = 0; i + 1 < n; i++)
        if (!(t[i] <= t[i + 1])) return fail(c, SBR_EARG, "ArgumentError: knots must be sorted");
    const bool paths = aw_total || aw_groups;
    if (paths && n_u != 1) return fail(c, SBR_EARG, "the AW paths need n_u == 1");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    const sbr_opts o = resolve(opts);
    int rc = ensure_hetero_knots(c, (size_t)n, (size_t)n_u);
    if (rc) return rc;
    const HeteroKnotLayout Lh(c->hk_cap_k, c->hk_cap_u);
    // the explicit-grid hazard (heterogeneity_solver.jl:255, solver.jl:163-164): τ̄ = knots <= η,
    // then η; pdf(η) is a BoundsError before the first knot or past the last one
    int64_t m = 0;
    while (m < n && t[m] <= eta) m++;
    const bool hz_oob = m == 0 || (m == n && !(n >= 2 && t[n - 1] == eta));
    const int64_t ntau = hz_oob ? 0 : m + 1;
    if ((hr && ntau > cap) || (paths && n > cap)) return fail(c, SBR_EARG, "path capacity too small");
    std::vector<double> key;
    key.reserve(2 * (size_t)K + 5);
    key.push_back((double)K);
    key.insert(key.end(), betas, betas + K);
    key.insert(key.end(), dist, dist + K);
    key.push_back(eta);
    key.push_back(p);
    key.push_back(lambda);
    const bool hit = c->hk_valid && c->hk_n == n && c->hk_K == K && c->hk_key == key &&
                     memcmp(c->hk_t.data(), t, (size_t)n * 8) == 0 &&
                     memcmp(c->hk_G.data(), G, (size_t)n * K * 8) == 0;
    char* D = c->hk_dev;
    char* H = c->hk_pin;
    int32_t* dcnt = (int32_t*)D;
    double* dsc = (double*)(D + Lh.sc); // βs [K], dist [K], η
    double* dtg = (double*)(D + Lh.tg);
    const size_t ck = c->hk_cap_k;
    const sbr::HeteroBufs HB{dtg, dtg + n, (double*)(D + Lh.hr), (double*)(D + Lh.hri), dcnt, dcnt + 1, dcnt + 2,
                             (uint32_t*)(dcnt + 3), dcnt + 4, dcnt + 5, (int32_t)ck, (int32_t)ck};
    double* du = (double*)(D + Lh.u); // [t_end, u...]
    double* dres = (double*)(D + Lh.res);
    const size_t nu = (size_t)n_u;
    // results: xi, aw, tol [n_u] | status, iters [n_u] int32 | tau_in, tau_out [n_u][K] |
    // path mode: AW_total [n], AW_OUT_k [K][n], AW_IN_k [K][n]
    double* dtin = dres + 4 * nu;
    double* dtout = dtin + nu * K;
    double* dpath = dtout + nu * K;
    const size_t res_bytes = (4 * nu + 2 * nu * K + (paths ? (size_t)n * (1 + 2 * K) : 0)) * 8;
    if (!hit) c->hk_valid = false;
    rc = fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        sbr::LearnArgs la{0.0, o.ode_reltol, o.ode_abstol, p, lambda, o.ode_maxiters, 1, 0, 0, nullptr, nullptr};
        if (!hit) {
            memset(H, 0, Lh.tg);
            int32_t* hc = (int32_t*)H;
            hc[0] = (int32_t)n;
            double* hs = (double*)(H + Lh.sc);
            memcpy(hs, betas, (size_t)K * 8);
            memcpy(hs + K, dist, (size_t)K * 8);
            hs[2 * K] = eta;
            memcpy(H + Lh.tg, t, (size_t)n * 8);
            memcpy(H + Lh.tg + (size_t)n * 8, G, (size_t)n * K * 8);
            HIP_TRY(c, hipMemcpyAsync(D, H, Lh.tg + (size_t)n * (K + 1) * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
            HIP_TRY(c, sbr::launch_hetero(K, dsc, dsc + K, dsc + 2 * K, nullptr, nullptr, la, sbr::HeteroEqArgs{},
                                          HB, sbr::ResultSoA{}, nullptr, nullptr, s, 2), SBR_EDEVICE);
            for (int k = 0; k < K && ntau > 0; k++)
                HIP_TRY(c, hipMemcpyAsync(H + Lh.hr + (size_t)k * ck * 8, D + Lh.hr + (size_t)k * ck * 8,
                                          (size_t)ntau * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
            HIP_TRY(c, hipMemcpyAsync(H, D, 32, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        }
        double* hu = (double*)(H + Lh.u);
        hu[0] = t_end;
        memcpy(hu + 1, u, nu * 8);
        HIP_TRY(c, hipMemcpyAsync(du, hu, (nu + 1) * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        sbr::HeteroEqArgs ea{kappa, 1e-12, (int32_t)n_u, o.hetero_max_iters, het_lds(c),
                             (o.flags & SBR_FLAG_EXHAUSTIVE) ? 1 : 0, (o.flags >> 8) & 7, aw_total ? dpath : nullptr};
        const sbr::ResultSoA r{dres, nullptr, nullptr, dres + nu, dres + 2 * nu, (uint32_t*)(dres + 3 * nu),
                               (int32_t*)(dres + 3 * nu) + nu};
        HIP_TRY(c, sbr::launch_hetero(K, dsc, dsc + K, dsc + 2 * K, du, du + 1, la, ea, HB, r, dtin, dtout, s, 1),
                SBR_EDEVICE);
        if (aw_groups)
            HIP_TRY(c, sbr::launch_hetero_aw_groups(K, dtg, dtg + n, dcnt, (int)n, dres, dtin, dtout,
                                                    (const uint32_t*)(dres + 3 * nu), dpath + n, (size_t)n, s),
                    SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(H + Lh.res, D + Lh.res, res_bytes, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        return SBR_OK;
    });
    if (rc) return rc;
    if (!hit) {
        const int32_t* hc = (const int32_t*)H;
        if (hc[1] != (int32_t)ntau) return fail(c, SBR_EDEVICE, "hetero hazard grid length mismatch");
        c->hk_t.assign(t, t + n);
        c->hk_G.assign(G, G + n * K);
        c->hk_hr.assign((size_t)K * ntau, 0.0);
        for (int k = 0; k < K; k++)
            memcpy(c->hk_hr.data() + (size_t)k * ntau, H + Lh.hr + (size_t)k * ck * 8, (size_t)ntau * 8);
        c->hk_key = key;
        c->hk_n = n;
        c->hk_K = K;
        c->hk_ntau = (int32_t)ntau;
        c->hk_valid = true;
    }
    const double* hres = (const double*)(H + Lh.res);
    if (out->xi) memcpy(out->xi, hres, nu * 8);
    if (out->aw_max) memcpy(out->aw_max, hres + nu, nu * 8);
    if (out->tol) memcpy(out->tol, hres + 2 * nu, nu * 8);
    if (out->status) memcpy(out->status, hres + 3 * nu, nu * 4);
    if (out->iters) memcpy(out->iters, (const int32_t*)(hres + 3 * nu) + nu, nu * 4);
    if (tau_in) memcpy(tau_in, hres + 4 * nu, nu * K * 8);
    if (tau_out) memcpy(tau_out, hres + 4 * nu + nu * K, nu * K * 8);
    if (n_tau) *n_tau = ntau;
    if (hr)
        for (int k = 0; k < K; k++) memcpy(hr + (size_t)k * cap, c->hk_hr.data() + (size_t)k * ntau, (size_t)ntau * 8);
    if (paths) {
        const bool run = (((const uint32_t*)(hres + 3 * nu))[0] & SBR_RUN) != 0;
        copy_hetero_paths(hres + 4 * nu + 2 * nu * K, run, K, n, cap, aw_total, aw_groups);
    }
    return SBR_OK;
}

}  // extern "C"

namespace {

// sbr_equilibrium_on_knots (pdf == nullptr: the learning pdf βG(1 − G) of the knots' G) and
// sbr_equilibrium_on_knots_pdf (the caller's pdf values on the same knots)
int on_knots(sbr_ctx* c, const double* t, const double* G, const double* pdf, int64_t n, double beta, double eta,
             double t_end, const double* u, int64_t n_u, double p, double kappa, double lambda, const sbr_opts* opts,
             sbr_result_soa* out, double* tau, double* hr, double* aw_cum, double* aw_out, double* aw_in, int64_t cap,
             int64_t* n_tau)
{
    if (!c || !t || !G || !u || !out) return SBR_EARG;
    if (n < 1 || n > (1 << 26) || n_u < 1 || n_u > (1 << 24)) return fail(c, SBR_EARG, "knot / u count");
    if (!scalars_valid(0.0, p, kappa, lambda) || !(beta > 0) || !(eta > 0) || !(t_end > 0))
        return fail(c, SBR_EARG, "ArgumentError: beta/eta/t_end/p/kappa/lambda");
    for (int64_t j = 0; j < n_u; j++)
        if (!(u[j] >= 0.0)) return fail(c, SBR_EARG, "ArgumentError: u must be non-negative");
    // Interpolations' gridded knots must be sorted (and not NaN)
    if (!(t[0] == t[0])) return fail(c, SBR_EARG, "ArgumentError: knots must be sorted");
    for (int64_t i = 0; i + 1 < n; i++)
        if (!(t[i] <= t[i + 1])) return fail(c, SBR_EARG, "ArgumentError: knots must be sorted");
    const bool want_aw = aw_cum || aw_out || aw_in;
    if (want_aw && n_u != 1) return fail(c, SBR_EARG, "AW paths need n_u == 1");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    const sbr_opts o = resolve(opts);
    int rc = ensure_knots(c, (size_t)n, (size_t)n_u);
    if (rc) return rc;
    const KnotLayout K(c->kn_cap_k, c->kn_cap_u);
    // the hazard grid as solver.jl:155-161 builds it (knots are sorted: the .<= η mask is a
    // prefix), and its BoundsError: pdf(η) outside [t_1, t_n]
    int64_t m = 0;
    while (m < n && t[m] <= eta) m++;
    const bool push = m == 0 || t[m - 1] != eta;
    const bool hz_oob = m < n ? m == 0 : push;
    const int64_t ntau = hz_oob ? 0 : m + (push ? 1 : 0);
    if ((tau || hr || want_aw) && ntau > cap) return fail(c, SBR_EARG, "path capacity too small");
    const double key[4] = {beta, eta, p, lambda};
    const bool hit = c->kn_valid && c->kn_n == n && memcmp(c->kn_key, key, sizeof key) == 0 &&
                     memcmp(c->kn_t.data(), t, (size_t)n * 8) == 0 && memcmp(c->kn_G.data(), G, (size_t)n * 8) == 0 &&
                     (pdf ? c->kn_pdf.size() == (size_t)n && memcmp(c->kn_pdf.data(), pdf, (size_t)n * 8) == 0
                          : c->kn_pdf.empty());
    char* D = c->kn_dev;
    char* H = c->kn_pin;
    int32_t* dcnt = (int32_t*)D; // n_knots, n_tau, n_le, status, n_accept, n_reject
    double* dsc = (double*)(D + K.sc);
    double* dtg = (double*)(D + K.tg);
    const sbr::LearnBufs L{dtg, dtg + n, (double*)(D + K.hr), nullptr, dcnt, dcnt + 1, dcnt + 2,
                           (uint32_t*)(dcnt + 3), dcnt + 4, dcnt + 5, (int32_t)c->kn_cap_k, (int32_t)c->kn_cap_k};
    double* du = (double*)(D + K.u); // [t_end, u_0 .. u_{n_u-1}]
    double* dres = (double*)(D + K.res);
    const size_t res_bytes = (size_t)n_u * 48 + (want_aw ? (size_t)ntau * 24 : 0);
    if (!hit) c->kn_valid = false; // the resident copy is being replaced
    rc = fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        if (!hit) {
            int32_t* hc = (int32_t*)H;
            memset(H, 0, K.tg);
            hc[0] = (int32_t)n;
            hc[2] = (int32_t)m;
            double* hs = (double*)(H + K.sc);
            hs[0] = beta;
            hs[1] = eta;
            memcpy(H + K.tg, t, (size_t)n * 8);
            memcpy(H + K.tg + (size_t)n * 8, G, (size_t)n * 8);
            if (pdf) memcpy(H + K.tg + (size_t)n * 16, pdf, (size_t)n * 8);
            HIP_TRY(c, hipMemcpyAsync(D, H, K.tg + (size_t)n * (pdf ? 24 : 16), hipMemcpyHostToDevice, s), SBR_EDEVICE);
            sbr::LearnArgs la{0.0, o.ode_reltol, o.ode_abstol, p, lambda, o.ode_maxiters, 1, 0, 0, nullptr, nullptr};
            la.pdf = pdf ? dtg + 2 * n : nullptr;
            HIP_TRY(c, sbr::launch_hazard(dsc, dsc + 1, la, L, 1, s), SBR_EDEVICE);
            if (ntau > 0)
                HIP_TRY(c, hipMemcpyAsync(H + K.hr, D + K.hr, (size_t)ntau * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
            HIP_TRY(c, hipMemcpyAsync(H, D, 32, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        }
        const size_t nu = (size_t)n_u;
        if (n_u == 1) {
            // one point: the whole workgroup on it (latency), inputs read from and results written
            // to mapped host memory — one launch, no copies
            double* z = c->kn_zc;
            double* zd = c->kn_zc_dev;
            z[0] = t_end;
            z[1] = u[0];
            const sbr::ResultSoA r{zd + 2, zd + 3, zd + 4, zd + 5, zd + 6, (uint32_t*)(zd + 7), (int32_t*)(zd + 7) + 1};
            double* zp = zd + 16;
            sbr::EqArgs ea{kappa, 1, o.bisect_max_iters, c->lds_cap, want_aw ? zp : nullptr,
                           (o.flags & SBR_FLAG_EXHAUSTIVE) ? 1 : 0, (o.flags >> 8) & 7,
                           want_aw ? zp + ntau : nullptr, want_aw ? zp + 2 * ntau : nullptr, 1, dres};
            if (o.flags & SBR_FLAG_XI_GUESS) ea.xi_guess = o.xi_guess;
            HIP_TRY(c, sbr::launch_point_coop(L, dsc + 1, zd, zd + 1, ea, r, s), SBR_EDEVICE);
        } else {
            double* hu = (double*)(H + K.u);
            hu[0] = t_end;
            memcpy(hu + 1, u, nu * 8);
            HIP_TRY(c, hipMemcpyAsync(du, hu, (nu + 1) * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
            const sbr::ResultSoA r{dres, dres + nu, dres + 2 * nu, dres + 3 * nu, dres + 4 * nu,
                                   (uint32_t*)(dres + 5 * nu), (int32_t*)(dres + 5 * nu) + nu};
            if ((o.flags & SBR_FLAG_XI_GUESS) && o.xi_guess == o.xi_guess) {
                // ξ_guess: the single-point kernel, one workgroup per u, in one launch (its plain
                // first-iterate bisection; the sweep kernel carries no guess path, it would cost the
                // sweeps registers)
                sbr::EqArgs ea{kappa, 1, o.bisect_max_iters, c->lds_cap, nullptr,
                               (o.flags & SBR_FLAG_EXHAUSTIVE) ? 1 : 0, (o.flags >> 8) & 7, nullptr, nullptr, 1};
                ea.xi_guess = o.xi_guess;
                HIP_TRY(c, sbr::launch_point_coop(L, dsc + 1, du, du + 1, ea, r, s, (int)nu), SBR_EDEVICE);
            } else {
                sbr::EqArgs ea{kappa, (int32_t)n_u, o.bisect_max_iters, c->lds_cap_b, nullptr,
                               (o.flags & SBR_FLAG_EXHAUSTIVE) ? 1 : 0, (o.flags >> 8) & 7, nullptr, nullptr, 1};
                HIP_TRY(c, sbr::launch_equilibrium(L, dsc + 1, du, du + 1, ea, r, 1, s, n <= c->lds_cap_b ? 1 : 2),
                        SBR_EDEVICE);
            }
            HIP_TRY(c, hipMemcpyAsync(H + K.res, D + K.res, res_bytes, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        }
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        return SBR_OK;
    });
    if (rc) return rc;
    if (!hit) {
        const int32_t* hc = (const int32_t*)H;
        // the device's hazard grid must be the one sized above (a bug guard)
        if (hc[1] != (int32_t)ntau) return fail(c, SBR_EDEVICE, "hazard grid length mismatch");
        c->kn_t.assign(t, t + n);
        c->kn_G.assign(G, G + n);
        if (pdf) c->kn_pdf.assign(pdf, pdf + n);
        else c->kn_pdf.clear();
        const double* hh = (const double*)(H + K.hr);
        c->kn_hr.assign(hh, hh + ntau);
        memcpy(c->kn_key, key, sizeof key);
        c->kn_n = n;
        c->kn_m = (int32_t)m;
        c->kn_ntau = (int32_t)ntau;
        c->kn_valid = true;
    }
    const size_t nu = (size_t)n_u;
    // n_u == 1: the mapped block [t_end, u, xi, τ̄_IN, τ̄_OUT, AW_max, tol, status | iters, pad, paths]
    const double* hr_ = n_u == 1 ? c->kn_zc + 2 : (const double*)(H + K.res);
    double* hs[5] = {out->xi, out->tau_in_unc, out->tau_out_unc, out->aw_max, out->tol};
    for (int k = 0; k < 5; k++)
        if (hs[k]) memcpy(hs[k], hr_ + k * nu, nu * 8);
    if (out->status) memcpy(out->status, hr_ + 5 * nu, nu * 4);
    if (out->iters) memcpy(out->iters, (const int32_t*)(hr_ + 5 * nu) + nu, nu * 4);
    if (n_tau) *n_tau = ntau;
    if (tau) {
        memcpy(tau, t, (size_t)m * 8);
        if (ntau > m) tau[m] = eta;
    }
    if (hr) memcpy(hr, c->kn_hr.data(), (size_t)ntau * 8);
    if (want_aw) { // n_u == 1
        const bool run = (((const uint32_t*)(hr_ + 5))[0] & SBR_RUN) != 0;
        const double* hp = c->kn_zc + 16;
        double* dst[3] = {aw_cum, aw_out, aw_in};
        for (int k = 0; k < 3; k++) {
            if (!dst[k]) continue;
            if (run) memcpy(dst[k], hp + k * ntau, (size_t)ntau * 8);
            else for (int64_t i = 0; i < ntau; i++) dst[k][i] = NAN;
        }
    }
    return SBR_OK;
}

}  // namespace

extern "C" {

int sbr_equilibrium_on_knots(sbr_ctx* c, const double* t, const double* G, int64_t n, double beta, double eta,
                             double t_end, const double* u, int64_t n_u, double p, double kappa, double lambda,
                             const sbr_opts* opts, sbr_result_soa* out, double* tau, double* hr, double* aw_cum,
                             double* aw_out, double* aw_in, int64_t cap, int64_t* n_tau)
{
    SBR_ON_RANK0(c, sbr_equilibrium_on_knots(c, t, G, n, beta, eta, t_end, u, n_u, p, kappa, lambda, opts, out, tau, hr, aw_cum, aw_out, aw_in, cap, n_tau));
    return on_knots(c, t, G, nullptr, n, beta, eta, t_end, u, n_u, p, kappa, lambda, opts, out, tau, hr, aw_cum,
                    aw_out, aw_in, cap, n_tau);
}

int sbr_equilibrium_on_knots_pdf(sbr_ctx* c, const double* t, const double* G, const double* pdf, int64_t n,
                                 double eta, double t_end, const double* u, int64_t n_u, double p, double kappa,
                                 double lambda, const sbr_opts* opts, sbr_result_soa* out, double* tau, double* hr,
                                 double* aw_cum, double* aw_out, double* aw_in, int64_t cap, int64_t* n_tau)
{
    SBR_ON_RANK0(c, sbr_equilibrium_on_knots_pdf(c, t, G, pdf, n, eta, t_end, u, n_u, p, kappa, lambda, opts, out, tau, hr, aw_cum, aw_out, aw_in, cap, n_tau));
    if (!pdf) return c ? fail(c, SBR_EARG, "pdf values missing") : SBR_EARG;
    // β only forms the default pdf; 1.0 passes the argument check and keys nothing else
    return on_knots(c, t, G, pdf, n, 1.0, eta, t_end, u, n_u, p, kappa, lambda, opts, out, tau, hr, aw_cum,
                    aw_out, aw_in, cap, n_tau);
}

int sbr_chunk_timeline(sbr_ctx* c, void* stream, int32_t* n_chunks, double* ms)
{
    SBR_PER_DEVICE_DIAG(c);
    if (!c || !n_chunks) return SBR_EARG;
    *n_chunks = 0;
    if (!c->ck_start || c->ck_ev.empty()) return SBR_OK;
    HIP_TRY(c, hipStreamSynchronize((hipStream_t)stream), SBR_EDEVICE);
    for (hipStream_t ls : c->lstream)
        if (ls) HIP_TRY(c, hipStreamSynchronize(ls), SBR_EDEVICE);
    const int nk = (int)c->ck_ev.size() / 2;
    for (int k = 0; k < nk; k++)
        for (int e = 0; e < 2; e++) {
            float a = -1.f;
            hipEvent_t ev = c->ck_ev[2 * k + e];
            if (ev && hipEventElapsedTime(&a, c->ck_start, ev) != hipSuccess) a = -1.f;
            if (ms) ms[2 * k + e] = ev ? (double)a : -1.0;
        }
    *n_chunks = nk;
    return SBR_OK;
}

int sbr_host_phases(sbr_ctx* c, double* ms5)
{
    if (!c || !ms5) return SBR_EARG;
    const double* ph = c->multi ? sbr_multi_impl::phases(c->multi) : c->ph_ms;
    for (int k = 0; k < 5; k++) ms5[k] = ph[k];
    return SBR_OK;
}

int sbr_last_schedule(sbr_ctx* c, int32_t* schedule)
{
    SBR_PER_DEVICE_DIAG(c);
    if (!c || !schedule) return SBR_EARG;
    *schedule = c->rs_used ? 1 : 0;
    return SBR_OK;
}

int sbr_timing_enable(sbr_ctx* c, int on)
{
    SBR_PER_DEVICE_DIAG(c);
    if (!c) return SBR_EARG;
    c->timing = on != 0;
    c->ev_used = 0;
    c->trec.clear();
    return SBR_OK;
}

int sbr_timing_read(sbr_ctx* c, void* stream, double* learn_ms, double* eq_ms, int32_t* n_calls)
{
    SBR_PER_DEVICE_DIAG(c);
    if (!c) return SBR_EARG;
    hipStream_t s = (hipStream_t)stream; // NULL = HIP null stream
    HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
    HIP_TRY(c, hipStreamSynchronize(c->stream), SBR_EDEVICE); // host-pointer sweeps time on it
    double a = 0.0, b = 0.0;
    int32_t n = 0;
    for (hipStream_t ls : c->lstream)
        if (ls) HIP_TRY(c, hipStreamSynchronize(ls), SBR_EDEVICE);
    for (hipStream_t rs : {c->rs_learn, c->rs_eq})
        if (rs) HIP_TRY(c, hipStreamSynchronize(rs), SBR_EDEVICE);
    for (const auto& r : c->trec) {
        float t = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&t, r.a, r.b), SBR_EDEVICE);
        if (r.kind == 0) a += t;
        else { b += t; n += r.count; }
    }
    if (learn_ms) *learn_ms = a;
    if (eq_ms) *eq_ms = b;
    if (n_calls) *n_calls = n;
    c->ev_used = 0;
    c->trec.clear();
    return SBR_OK;
}

int sbr_learn_stats(sbr_ctx* c, int64_t n_beta, int32_t* n_knots, int32_t* n_tau, int32_t* n_accept,
                    int32_t* n_reject, uint32_t* status)
{
    SBR_PER_DEVICE_DIAG(c);
    if (!c || n_beta <= 0 || (size_t)(n_beta + c->last_off) > c->ws_beta[c->last_slot]) return SBR_EARG;
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    HIP_TRY(c, hipDeviceSynchronize(), SBR_EDEVICE);
    const sbr::LearnBufs& L = c->LW[c->last_slot];
    const int64_t o = c->last_off; // the last grid of a grouped learning slot
    struct { int32_t* h; void* d; } cp[] = {{n_knots, L.n_knots + o}, {n_tau, L.n_tau + o}, {n_accept, L.n_accept + o},
                                           {n_reject, L.n_reject + o}, {(int32_t*)status, L.status + o}};
    for (auto& x : cp)
        if (x.h) HIP_TRY(c, hipMemcpy(x.h, x.d, (size_t)n_beta * 4, hipMemcpyDeviceToHost), SBR_EDEVICE);
    return SBR_OK;
}

int sbr_hetero_learn_stats(sbr_ctx* c, int64_t n_col, int32_t* n_knots, int32_t* n_tau, int32_t* n_accept,
                           int32_t* n_reject, uint32_t* status)
{
    SBR_PER_DEVICE_DIAG(c);
    if (!c || n_col <= 0 || (size_t)n_col > c->hs_col) return SBR_EARG;
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    HIP_TRY(c, hipDeviceSynchronize(), SBR_EDEVICE);
    const sbr::HeteroBufs& H = c->H;
    struct { int32_t* h; void* d; } cp[] = {{n_knots, H.n_knots}, {n_tau, H.n_tau}, {n_accept, H.n_accept},
                                           {n_reject, H.n_reject}, {(int32_t*)status, H.status}};
    for (auto& x : cp)
        if (x.h) HIP_TRY(c, hipMemcpy(x.h, x.d, (size_t)n_col * 4, hipMemcpyDeviceToHost), SBR_EDEVICE);
    return SBR_OK;
}

int sbr_learn_hetero(sbr_ctx* c, int32_t K, const double* betas, const double* dist, const double* t_end, double x0,
                     int64_t n_col, const sbr_opts* opts, double* t_out, double* G_out, int64_t cap, int32_t* n_knots,
                     uint32_t* status)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_ON_RANK0(c, sbr_learn_hetero(c, K, betas, dist, t_end, x0, n_col, opts, t_out, G_out, cap, n_knots, status));
    if (!c || !betas || !dist || !t_end || n_col <= 0 || n_col > (1 << 30) || cap <= 0) return SBR_EARG;
    if (K != 1 && K != 2 && K != 3 && K != 4 && K != 8) return fail(c, SBR_EARG, "K must be 1, 2, 3, 4 or 8");
    // LearningParametersHetero checks (heterogeneity_model.jl:33-41)
    double dsum = 0.0;
    for (int k = 0; k < K; k++) {
        if (!(dist[k] >= 0.0)) return fail(c, SBR_EARG, "ArgumentError: distribution weights must be non-negative");
        dsum = dsum + dist[k];
    }
    if (!(fabs(dsum - 1.0) < 1e-10)) return fail(c, SBR_EARG, "ArgumentError: distribution must sum to 1");
    for (int64_t i = 0; i < n_col * K; i++)
        if (!(betas[i] > 0.0)) return fail(c, SBR_EARG, "ArgumentError: all learning rates must be positive");
    for (int64_t i = 0; i < n_col; i++)
        if (!(t_end[i] > 0.0)) return fail(c, SBR_EARG, "ArgumentError: End time must be greater than start time");
    if (!(x0 >= 0.0)) return fail(c, SBR_EARG, "ArgumentError: Initial condition must be non-negative");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    if (cap < o.knot_capacity) o.knot_capacity = (int32_t)cap;
    int rc = ensure_hetero(c, (size_t)n_col, (size_t)o.knot_capacity, (size_t)K);
    if (rc) return rc;
    rc = ensure_stage(c, ((size_t)n_col * K + K + (size_t)n_col) * 8 + 256);
    if (rc) return rc;
    double* dbeta = (double*)c->stage;
    double* ddist = dbeta + (size_t)n_col * K;
    double* dtend = ddist + K;
    return fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        HIP_TRY(c, hipMemcpyAsync(dbeta, betas, (size_t)n_col * K * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(ddist, dist, (size_t)K * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(dtend, t_end, (size_t)n_col * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        // the knot grid runs to t_end whatever η is (the learning stage of a sweep streams
        // the hazard for η alongside; here η = t_end only sizes that unused stream)
        sbr::LearnArgs la{x0, o.ode_reltol, o.ode_abstol, 0.5, 1.0, o.ode_maxiters, (int32_t)n_col, 0, 0};
        sbr::HeteroEqArgs ea{0.5, 1e-12, 1, o.hetero_max_iters, het_lds(c), 0, 0, nullptr};
        sbr::ResultSoA r{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
        HIP_TRY(c, sbr::launch_hetero(K, dbeta, ddist, dtend, dtend, nullptr, la, ea, c->H, r, nullptr, nullptr, s, 0),
                SBR_EDEVICE);
        const size_t w = (size_t)o.knot_capacity, ld = (size_t)c->H.cap;
        if (t_out)
            HIP_TRY(c, hipMemcpy2DAsync(t_out, (size_t)cap * 8, c->H.t, ld * 8, w * 8, (size_t)n_col, hipMemcpyDeviceToHost, s),
                    SBR_EDEVICE);
        if (G_out)
            HIP_TRY(c, hipMemcpy2DAsync(G_out, (size_t)cap * K * 8, c->H.G, ld * K * 8, w * K * 8, (size_t)n_col,
                                        hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (n_knots) HIP_TRY(c, hipMemcpyAsync(n_knots, c->H.n_knots, (size_t)n_col * 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (status) HIP_TRY(c, hipMemcpyAsync(status, c->H.status, (size_t)n_col * 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        return SBR_OK;
    });
}

int sbr_sweep_hetero_dev(sbr_ctx* c, void* stream, int32_t K, const double* betas, const double* dist,
                         const double* eta, const double* t_end, double x0, const double* u, int64_t n_col,
                         int64_t n_u, double p, double kappa, double lambda, const sbr_opts* opts,
                         sbr_result_soa* out, double* tau_in, double* tau_out)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_SINGLE_DEVICE(c);
    if (!c || !out || !out->xi || !out->aw_max || !out->tol || !out->status) return SBR_EARG;
    if (K != 1 && K != 2 && K != 3 && K != 4 && K != 8) return fail(c, SBR_EARG, "K must be 1, 2, 3, 4 or 8");
    if (n_col <= 0 || n_u <= 0 || n_col > (1 << 30) || n_u > (1 << 30)) return fail(c, SBR_EARG, "grid size");
    if (!scalars_valid(x0, p, kappa, lambda)) return fail(c, SBR_EARG, "ArgumentError: x0/p/kappa/lambda");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    int rc = ensure_hetero(c, (size_t)n_col, (size_t)o.knot_capacity, (size_t)K);
    if (rc) return rc;
    return fenced(c, stream, true, [&](hipStream_t s) -> int {
        sbr::LearnArgs la{x0, o.ode_reltol, o.ode_abstol, p, lambda, o.ode_maxiters, (int32_t)n_col, 0, 0};
        sbr::HeteroEqArgs ea{kappa, 1e-12, (int32_t)n_u, o.hetero_max_iters, het_lds(c),
                             (o.flags & SBR_FLAG_EXHAUSTIVE) ? 1 : 0, (o.flags >> 8) & 7, c->het_aw_path};
        sbr::ResultSoA r{out->xi, nullptr, nullptr, out->aw_max, out->tol, out->status, out->iters};
        hipEvent_t t0 = tstart(c, s);
        HIP_TRY(c, sbr::launch_hetero(K, betas, dist, eta, t_end, u, la, ea, c->H, r, tau_in, tau_out, s, 0), SBR_EDEVICE);
        tend(c, s, 0, t0);
        t0 = tstart(c, s);
        HIP_TRY(c, sbr::launch_hetero(K, betas, dist, eta, t_end, u, la, ea, c->H, r, tau_in, tau_out, s, 1), SBR_EDEVICE);
        tend(c, s, 1, t0);
        return SBR_OK;
    });
}

int sbr_sweep_hetero_batch_dev(sbr_ctx* c, void* stream, int64_t n_batch, int32_t K, const double* betas,
                               const double* dist, const double* eta, const double* t_end, double x0, const double* u,
                               int64_t n_col, int64_t n_u, double p, double kappa, double lambda, const sbr_opts* opts,
                               sbr_result_soa* out, double* tau_in, double* tau_out)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_SINGLE_DEVICE(c);
    if (!c || !out || !out->xi || !out->aw_max || !out->tol || !out->status || !betas || !dist || !eta || !t_end || !u)
        return SBR_EARG;
    if (K != 1 && K != 2 && K != 3 && K != 4 && K != 8) return fail(c, SBR_EARG, "K must be 1, 2, 3, 4 or 8");
    if (n_batch <= 0 || n_col <= 0 || n_u <= 0 || n_col > (1 << 30) || n_u > (1 << 30))
        return fail(c, SBR_EARG, "grid size");
    if (!scalars_valid(x0, p, kappa, lambda)) return fail(c, SBR_EARG, "ArgumentError: x0/p/kappa/lambda");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    const size_t cap = (size_t)o.knot_capacity;
    int rc = ensure_hetero(c, (size_t)n_col, cap, (size_t)K);
    if (!rc && n_batch > 1) rc = ensure_hetero_bufs(c, c->H2, c->hs2_col, c->hs2_cap, c->hs2_K, (size_t)n_col, cap, (size_t)K);
    if (!rc) rc = ensure_pipe_streams(c);
    if (rc) return rc;
    return fenced(c, stream, true, [&](hipStream_t s) -> int {
        sbr::LearnArgs la{x0, o.ode_reltol, o.ode_abstol, p, lambda, o.ode_maxiters, (int32_t)n_col, 0, 0};
        sbr::HeteroEqArgs ea{kappa, 1e-12, (int32_t)n_u, o.hetero_max_iters, het_lds(c),
                             (o.flags & SBR_FLAG_EXHAUSTIVE) ? 1 : 0, (o.flags >> 8) & 7, nullptr};
        const size_t np = (size_t)n_col * (size_t)n_u;
        HIP_TRY(c, hipEventRecord(c->ev_in, s), SBR_EDEVICE);
        for (int k = 0; k < 2; k++) HIP_TRY(c, hipStreamWaitEvent(c->lstream[k], c->ev_in, 0), SBR_EDEVICE);
        for (int64_t k = 0; k < n_batch; k++) {
            const int slot = (int)(k & 1);
            hipStream_t ls = c->lstream[slot];
            const sbr::HeteroBufs& H = slot ? c->H2 : c->H;
            const double* bk = betas + k * n_col * K;
            const double* ek = eta + k * n_col;
            const double* tk = t_end + k * n_col;
            // the slot's previous reader (equilibrium of batch k - 2) must be done
            if (k >= 2) HIP_TRY(c, hipStreamWaitEvent(ls, c->ev_eq[slot], 0), SBR_EDEVICE);
            hipEvent_t t0 = tstart(c, ls);
            sbr::ResultSoA r{out->xi + k * np, nullptr, nullptr, out->aw_max + k * np, out->tol + k * np,
                             out->status + k * np, out->iters ? out->iters + k * np : nullptr};
            double* ti = tau_in ? tau_in + k * np * K : nullptr;
            double* to = tau_out ? tau_out + k * np * K : nullptr;
            HIP_TRY(c, sbr::launch_hetero(K, bk, dist, ek, tk, u, la, ea, H, r, ti, to, ls, 0), SBR_EDEVICE);
            tend(c, ls, 0, t0);
            HIP_TRY(c, hipEventRecord(c->ev_learned[slot], ls), SBR_EDEVICE);
            HIP_TRY(c, hipStreamWaitEvent(s, c->ev_learned[slot], 0), SBR_EDEVICE);
            t0 = tstart(c, s);
            HIP_TRY(c, sbr::launch_hetero(K, bk, dist, ek, tk, u, la, ea, H, r, ti, to, s, 1), SBR_EDEVICE);
            tend(c, s, 1, t0);
            HIP_TRY(c, hipEventRecord(c->ev_eq[slot], s), SBR_EDEVICE);
        }
        return SBR_OK;
    });
}

int sbr_hetero_point_paths(sbr_ctx* c, int32_t K, const double* betas, const double* dist, double eta, double t_end,
                           double x0, double u, double p, double kappa, double lambda, const sbr_opts* opts,
                           double* res, uint32_t* status, double* tau_in, double* tau_out, double* t, double* G,
                           double* aw_total, double* aw_groups, int64_t cap, int64_t* n_knots)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_ON_RANK0(c, sbr_hetero_point_paths(c, K, betas, dist, eta, t_end, x0, u, p, kappa, lambda, opts, res, status, tau_in, tau_out, t, G, aw_total, aw_groups, cap, n_knots));
    if (!c || !res || !status || !betas || !dist) return SBR_EARG;
    if (K != 1 && K != 2 && K != 3 && K != 4 && K != 8) return fail(c, SBR_EARG, "K must be 1, 2, 3, 4 or 8");
    double dsum = 0.0;
    for (int k = 0; k < K; k++) {
        if (!(dist[k] >= 0.0)) return fail(c, SBR_EARG, "ArgumentError: distribution weights must be non-negative");
        if (!(betas[k] > 0.0)) return fail(c, SBR_EARG, "ArgumentError: all learning rates must be positive");
        dsum = dsum + dist[k];
    }
    if (!(fabs(dsum - 1.0) < 1e-10)) return fail(c, SBR_EARG, "ArgumentError: distribution must sum to 1");
    if (!scalars_valid(x0, p, kappa, lambda) || !(eta > 0) || !(t_end > 0) || !(u >= 0))
        return fail(c, SBR_EARG, "ArgumentError");
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    const size_t kc = (size_t)o.knot_capacity;
    int rc = ensure_stage(c, (2 * (size_t)K + 3 + 4 + 2 * (size_t)K + (1 + 2 * (size_t)K) * kc) * 8 + 512);
    if (rc) return rc;
    double* d = (double*)c->stage;
    double *dbeta = d, *ddist = d + K, *deta = d + 2 * K, *dtend = deta + 1, *du = dtend + 1;
    double* dres = du + 1; // xi, aw, tol
    uint32_t* dst = (uint32_t*)(dres + 3);
    double* dtin = dres + 4;
    double* dtout = dtin + K;
    double* dpath = dtout + K;
    return fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        const double hin[3] = {eta, t_end, u};
        HIP_TRY(c, hipMemcpyAsync(dbeta, betas, (size_t)K * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(ddist, dist, (size_t)K * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(deta, hin, 24, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        sbr_result_soa r{dres, nullptr, nullptr, dres + 1, dres + 2, dst, nullptr};
        c->het_aw_path = dpath;
        rc = sbr_sweep_hetero_dev(c, s, K, dbeta, ddist, deta, dtend, x0, du, 1, 1, p, kappa, lambda, &o, &r, dtin, dtout);
        c->het_aw_path = nullptr;
        if (rc) return rc;
        double* dgrp = dpath + kc; // AW_OUT_k / AW_IN_k rows of stride kc
        if (aw_groups)
            HIP_TRY(c, sbr::launch_hetero_aw_groups(K, c->H.t, c->H.G, c->H.n_knots, (int)kc, dres, dtin, dtout, dst,
                                                    dgrp, kc, s), SBR_EDEVICE);
        int32_t n = 0;
        HIP_TRY(c, hipMemcpyAsync(res, dres, 24, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(status, dst, 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (tau_in) HIP_TRY(c, hipMemcpyAsync(tau_in, dtin, (size_t)K * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (tau_out) HIP_TRY(c, hipMemcpyAsync(tau_out, dtout, (size_t)K * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(&n, c->H.n_knots, 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        if (n_knots) *n_knots = n;
        if (n > cap) return fail(c, SBR_EARG, "path capacity too small");
        if (t) HIP_TRY(c, hipMemcpy(t, c->H.t, (size_t)n * 8, hipMemcpyDeviceToHost), SBR_EDEVICE);
        if (G) HIP_TRY(c, hipMemcpy(G, c->H.G, (size_t)n * K * 8, hipMemcpyDeviceToHost), SBR_EDEVICE);
        if (aw_total || aw_groups) {
            const bool run = (*status & SBR_RUN) != 0;
            std::vector<double> h(run ? (size_t)n * (1 + 2 * K) : 0);
            for (int r = 0; run && r <= 2 * K; r++)
                HIP_TRY(c, hipMemcpy(h.data() + (size_t)r * n, r == 0 ? dpath : dgrp + (size_t)(r - 1) * kc,
                                     (size_t)n * 8, hipMemcpyDeviceToHost), SBR_EDEVICE);
            copy_hetero_paths(h.data(), run, K, n, cap, aw_total, aw_groups);
        }
        return SBR_OK;
    });
}

int sbr_sweep_hetero(sbr_ctx* c, int32_t K, const double* betas, const double* dist, const double* eta,
                     const double* t_end, double x0, const double* u, int64_t n_col, int64_t n_u, double p,
                     double kappa, double lambda, const sbr_opts* opts, sbr_result_soa* out, double* tau_in,
                     double* tau_out)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    if (!c || !out || !betas || !dist || !eta || !t_end || !u || K <= 0) return SBR_EARG;
    if (n_col <= 0 || n_u <= 0) return fail(c, SBR_EARG, "grid size");
    // LearningParametersHetero checks (heterogeneity_model.jl:33-41)
    double dsum = 0.0;
    for (int k = 0; k < K; k++) {
        if (!(dist[k] >= 0.0)) return fail(c, SBR_EARG, "ArgumentError: distribution weights must be non-negative");
        dsum = dsum + dist[k];
    }
    if (!(fabs(dsum - 1.0) < 1e-10)) return fail(c, SBR_EARG, "ArgumentError: distribution must sum to 1");
    for (int64_t i = 0; i < n_col * K; i++)
        if (!(betas[i] > 0.0)) return fail(c, SBR_EARG, "ArgumentError: all learning rates must be positive");
    for (int64_t i = 0; i < n_col; i++)
        if (!(eta[i] > 0.0) || !(t_end[i] > 0.0)) return fail(c, SBR_EARG, "ArgumentError: eta/t_end");
    for (int64_t j = 0; j < n_u; j++)
        if (!(u[j] >= 0.0)) return fail(c, SBR_EARG, "ArgumentError: u must be non-negative");
    if (c->multi) {
        if (K != 1 && K != 2 && K != 3 && K != 4 && K != 8) return fail(c, SBR_EARG, "K must be 1, 2, 3, 4 or 8");
        return multi_sweep_hetero(c, K, betas, dist, eta, t_end, x0, u, n_col, n_u, p, kappa, lambda, resolve(opts),
                                  out, tau_in, tau_out);
    }
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    const size_t np = (size_t)n_col * (size_t)n_u;
    const size_t in_d = (size_t)n_col * K + K + 2 * (size_t)n_col + (size_t)n_u;
    const size_t out_d = np * 3 + np + 2 * np * K; // xi, aw, tol | status+iters | tin, tout
    int rc = ensure_stage(c, (in_d + out_d) * 8 + 512);
    if (rc) return rc;
    double* d = (double*)c->stage;
    double *dbeta = d, *ddist = dbeta + (size_t)n_col * K, *deta = ddist + K, *dtend = deta + n_col,
           *du = dtend + n_col;
    double* dres = du + n_u;
    double *dxi = dres, *daw = dxi + np, *dtol = daw + np;
    uint32_t* dst = (uint32_t*)(dtol + np);
    int32_t* dit = (int32_t*)(dst + np);
    double* dtin = (double*)(dit + np);
    double* dtout = dtin + np * K;
    return fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        HIP_TRY(c, hipMemcpyAsync(dbeta, betas, (size_t)n_col * K * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(ddist, dist, (size_t)K * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(deta, eta, (size_t)n_col * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(dtend, t_end, (size_t)n_col * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(du, u, (size_t)n_u * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        sbr_result_soa r{dxi, nullptr, nullptr, daw, dtol, dst, dit};
        rc = sbr_sweep_hetero_dev(c, s, K, dbeta, ddist, deta, dtend, x0, du, n_col, n_u, p, kappa, lambda, opts, &r,
                                  tau_in ? dtin : nullptr, tau_out ? dtout : nullptr);
        if (rc) return rc;
        if (out->xi) HIP_TRY(c, hipMemcpyAsync(out->xi, dxi, np * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (out->aw_max) HIP_TRY(c, hipMemcpyAsync(out->aw_max, daw, np * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (out->tol) HIP_TRY(c, hipMemcpyAsync(out->tol, dtol, np * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (out->status) HIP_TRY(c, hipMemcpyAsync(out->status, dst, np * 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (out->iters) HIP_TRY(c, hipMemcpyAsync(out->iters, dit, np * 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (tau_in) HIP_TRY(c, hipMemcpyAsync(tau_in, dtin, np * K * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        if (tau_out) HIP_TRY(c, hipMemcpyAsync(tau_out, dtout, np * K * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        return SBR_OK;
    });
}

int sbr_social_prof_read(sbr_ctx* c, int64_t* out8)
{
    SBR_PER_DEVICE_DIAG(c);
    if (!c || !out8) return SBR_EARG;
    for (int k = 0; k < 8; k++) out8[k] = k < (int)c->so_prof_acc.size() ? c->so_prof_acc[k] : 0;
    return SBR_OK;
}

int sbr_social_overflow_stats(sbr_ctx* c, int64_t* promoted, int64_t* rerun)
{
    SBR_PER_DEVICE_DIAG(c);
    if (!c) return SBR_EARG;
    if (promoted) *promoted = c->so_promoted;
    if (rerun) *rerun = c->so_rerun;
    return SBR_OK;
}

int sbr_set_social_workspace(sbr_ctx* c, int64_t bytes)
{
    if (!c || bytes < 0) return SBR_EARG;
    for (int r = 0; c->multi && r < sbr_multi_size(c); r++) (void)sbr_set_social_workspace(sbr_multi_child(c, r), bytes);
    c->so_budget = bytes;
    return SBR_OK;
}

}  // extern "C"

namespace {
constexpr int kSocialDefaultCap = 98304;  // ≈1.4× the typical longest iterate on config 5 (≈70k knots)
constexpr int kSocialMaxCap = 1 << 22;    // overflow retries grow 4× per pass up to this
constexpr int64_t kPoolSlots = 256;       // promotion pool slots (points that outgrow the capacity)
constexpr int kSocialInner = 16; // fixed-point iterates per launch (compaction in between)
constexpr int kSocialBulk = 2;   // launches of kSocialInner iterates before the shorter ones
constexpr int kSocialInner2 = 8; // iterates per launch after the bulk launches

int social_checks(sbr_ctx* c, const double* beta, const double* eta, const double* u, int64_t n_beta, int64_t n_u,
                  double x0, double p, double kappa, double lambda, const double* cmp, int32_t n_cmp, double tol,
                  int32_t max_iter, sbr_result_soa* out)
{
    if (!c || !out || !beta || !eta || !u || !cmp) return SBR_EARG;
    if (!out->xi || !out->tau_in_unc || !out->tau_out_unc || !out->aw_max || !out->tol || !out->status)
        return fail(c, SBR_EARG, "result arrays");
    if (n_beta <= 0 || n_u <= 0 || n_beta * n_u > (int64_t(1) << 40)) return fail(c, SBR_EARG, "grid size");
    if (n_cmp < 1 || max_iter < 1 || !(tol > 0.0)) return fail(c, SBR_EARG, "n_cmp / max_iter / tol");
    if (!scalars_valid(x0, p, kappa, lambda)) return fail(c, SBR_EARG, "ArgumentError: x0/p/kappa/lambda");
    return SBR_OK;
}

// one pass of the whole fixed point over points [0, n_total) (list == nullptr)
// or over the global point indices list[0 .. n_total), chunked by workspace
// size; poll > 0 reads the live counts after every launch and stops early.
// Points whose iterate outgrows `cap` are promoted into the pool (16× the
// capacity) and redo that iterate from the pool blocks of the same or the next launch.
int run_social_pass(sbr_ctx* c, hipStream_t s, const double* beta, const double* eta, double x0, const double* u,
                    int64_t n_u, double p, double kappa, double lambda, const double* cmp, int32_t n_cmp, double tol,
                    int32_t max_iter, const sbr_opts& o, sbr_result_soa* out, int32_t* fp_iters, int64_t* rk_steps,
                    int poll, size_t cap, size_t pcap, const int64_t* list, int64_t n_total)
{
    const size_t per_pt = 5 * cap * 8 + (size_t)n_cmp * 8 + 64;
    const size_t per_slot = 5 * pcap * 8 + (size_t)n_cmp * 8 + 64;
    int64_t budget = c->so_budget, pbudget = 0;
    {
        size_t fr = 0, tot = 0;
        HIP_TRY(c, hipMemGetInfo(&fr, &tot), SBR_EDEVICE);
        const double avail = (double)fr + (double)c->so_pts * (5 * c->so_cap * 8 + c->so_cmp * 8 + 64) +
                             (double)c->pl_slots * (5 * c->pl_cap * 8 + c->pl_cmp * 8 + 64);
        if (budget <= 0) budget = (int64_t)(avail * 0.6);
        pbudget = (int64_t)(avail * 0.15);
    }
    int64_t chunk = budget / (int64_t)per_pt;
    if (chunk < 64 && !list) return fail(c, SBR_ENOMEM, "social workspace budget below 64 points");
    if (chunk < 1) chunk = 1; // overflow retries: at least one point at a time
    if (chunk > (1 << 30)) chunk = 1 << 30;
    if (chunk >= n_total) chunk = n_total;
    else if (chunk >= 64) chunk &= ~(int64_t)63; // whole wave groups
    int rc = ensure_social(c, (size_t)chunk, cap, (size_t)n_cmp);
    if (rc) return rc;
    // pool: up to kPoolSlots slots (whole wave groups) within its budget
    int64_t nslots = pcap > cap ? pbudget / (int64_t)per_slot : 0;
    if (nslots > kPoolSlots) nslots = kPoolSlots;
    if (nslots > chunk) nslots = chunk;
    if (nslots >= 64) nslots &= ~(int64_t)63;
    if (nslots > 0) {
        rc = ensure_pool(c, (size_t)nslots, pcap, (size_t)n_cmp);
        if (rc) return rc;
    }
    const bool prof = (o.flags & SBR_FLAG_DIAG_SOCIAL_PROF) != 0;
    if (prof && c->so_prof_pts < (size_t)chunk) {
        if (c->so_prof) (void)hipFree(c->so_prof);
        c->so_prof = nullptr;
        c->so_prof_pts = 0;
        HIP_TRY(c, hipMalloc(&c->so_prof, (size_t)chunk * 64), SBR_ENOMEM);
        c->so_prof_pts = (size_t)chunk;
    }
    for (int64_t pt0 = 0; pt0 < n_total; pt0 += chunk) {
        const int32_t npts = (int32_t)((n_total - pt0) < chunk ? (n_total - pt0) : chunk);
        sbr::SocialArgs a{};
        a.beta = beta; a.eta = eta; a.u = u; a.cmp = cmp;
        a.pt0 = list ? 0 : pt0; a.pts = list ? list + pt0 : nullptr;
        a.n_pts = npts; a.n_u = (int32_t)n_u; a.n_cmp = n_cmp;
        a.max_iter = max_iter; a.bisect_max_iters = o.bisect_max_iters; a.cap = (int32_t)cap;
        a.maxiters = o.ode_maxiters;
        a.x0 = x0; a.p = p; a.kappa = kappa; a.lam = lambda; a.tol = tol; a.rtol = o.ode_reltol; a.atol = o.ode_abstol;
        a.ws = c->so_ws; a.cmpo = c->so_cmpo; a.n_old = c->so_n_old; a.slots = c->so_slots; a.xi_new = c->so_xi;
        a.bits = c->so_bits; a.steps = c->so_steps; a.live = c->so_live; a.work = c->so_work[0];
        a.count = c->so_count;
        a.out = sbr::ResultSoA{out->xi, out->tau_in_unc, out->tau_out_unc, out->aw_max, out->tol, out->status,
                               out->iters};
        a.fp_iters = fp_iters;
        a.steps_out = rk_steps;
        a.prof = prof ? c->so_prof : nullptr;
        a.path_t = c->so_path_t; a.path_G = c->so_path_G; a.path_aw = c->so_path_aw; a.path_n = c->so_path_n;
        a.path_cap = c->so_path_cap;
        a.pool = sbr::SocialPool{};
        sbr::SocialArgs b{}; // the pool's own arguments (n_pts = 0: no pool blocks)
        if (nslots > 0) {
            a.pool = sbr::SocialPool{c->pl_ws,    (int32_t)pcap, (int32_t)nslots, c->so_count + 2, c->so_count + 3,
                                     c->pl_pts,   c->pl_n_old,   c->pl_perm,      c->pl_xi,        c->pl_bits,
                                     c->pl_steps, c->pl_live,    c->pl_it,        c->pl_ready};
            b = a;
            b.pt0 = 0; b.pts = c->pl_pts; b.n_pts = (int32_t)nslots; b.cap = (int32_t)pcap;
            b.ws = c->pl_ws; b.cmpo = c->pl_cmpo; b.n_old = c->pl_n_old; b.slots = c->pl_perm; b.xi_new = c->pl_xi;
            b.bits = c->pl_bits; b.steps = c->pl_steps; b.live = c->pl_live; b.work = nullptr; b.count = nullptr;
            b.prof = nullptr;
            b.pool = sbr::SocialPool{};
            b.it_cur = c->pl_it; b.ready = c->pl_ready; b.n_live = c->so_count + 3;
            HIP_TRY(c, hipMemsetAsync(c->pl_ready, 0, (size_t)nslots * 4, s), SBR_EDEVICE);
        }
        HIP_TRY(c, hipMemsetAsync(c->so_count + 2, 0, 2 * 4, s), SBR_EDEVICE); // pool allocator + live
        // (the staging buffer is reused by the next chunk only after this one's final sync)
        c->so_args_host[0] = a;
        c->so_args_host[1] = b;
        HIP_TRY(c, hipMemcpyAsync(c->so_args_dev, c->so_args_host, 2 * sizeof(sbr::SocialArgs),
                                  hipMemcpyHostToDevice, s),
                SBR_EDEVICE);
        if (prof) HIP_TRY(c, hipMemsetAsync(c->so_prof, 0, (size_t)npts * 64, s), SBR_EDEVICE);
        hipEvent_t t0 = tstart(c, s);
        HIP_TRY(c, sbr::launch_social_init(a, s), SBR_EDEVICE);
        tend(c, s, 0, t0);
        t0 = tstart(c, s);
        // kSocialInner iterates per launch; a point promoted during a launch redoes that
        // iterate in the same or the next launch: one launch past max_iter drains the pool
        // The first kSocialBulk launches run kSocialInner iterates each (the bulk: most points
        // converge around iterate 35); later launches run kSocialInner2, so the survivors are
        // re-spread over the waves (fewer points per wave, then one: the whole-wave mode) sooner.
        std::vector<int> inner;
        for (int done = 0, q = 0; done < max_iter; q++) {
            const int m = q < kSocialBulk ? kSocialInner : kSocialInner2;
            inner.push_back(m);
            done += m;
        }
        const int n_launch = (int)inner.size();
        static const bool trace = getenv("SBR_SOCIAL_TRACE") != nullptr;
        const auto tr0 = std::chrono::steady_clock::now();
        int q = 0, it = 1;
        for (; q < n_launch; it += inner[q], q++) {
            const int k = q & 1;
            HIP_TRY(c, sbr::launch_social_iter(a, b, c->so_args_dev, it, inner[q], c->so_work[k],
                                               c->so_count + k, c->so_work[k ^ 1], c->so_count + (k ^ 1), s),
                    SBR_EDEVICE);
            if ((poll > 0 || trace) && q + 1 < n_launch) {
                HIP_TRY(c, hipMemcpyAsync(c->so_count_host, c->so_count, 4 * 4, hipMemcpyDeviceToHost, s),
                        SBR_EDEVICE);
                HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
                if (trace) // diagnostics: the fixed point's timeline (live points after each launch)
                    fprintf(stderr, "sbr_social_trace launch=%d t=%.3f live=%d pool_used=%d pool_live=%d\n", q,
                                 std::chrono::duration<double>(std::chrono::steady_clock::now() - tr0).count(),
                                 c->so_count_host[k ^ 1], c->so_count_host[2], c->so_count_host[3]);
                if (poll > 0 && c->so_count_host[k ^ 1] == 0 && c->so_count_host[3] == 0) { q++; break; }
            }
        }
        // Pool drain.  A point promoted during a launch restarts at its promotion iterate in the
        // next launch, so it can trail the main worklist by up to one launch's iterates (16) and
        // still be live once the main list has reached max_iter: drain launches of kSocialInner
        // iterates run until the pool has no live point (bounded: each advances every pool point
        // by kSocialInner iterates towards max_iter).
        for (int d = 0; nslots > 0 && d <= max_iter / kSocialInner + 1; d++, it += kSocialInner, q++) {
            HIP_TRY(c, hipMemcpyAsync(c->so_count_host, c->so_count, 4 * 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
            HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
            if (c->so_count_host[3] == 0) break;
            const int k = q & 1;
            HIP_TRY(c, sbr::launch_social_iter(a, b, c->so_args_dev, it, kSocialInner, c->so_work[k],
                                               c->so_count + k, c->so_work[k ^ 1], c->so_count + (k ^ 1), s),
                    SBR_EDEVICE);
            if (trace)
                fprintf(stderr, "sbr_social_trace drain=%d pool_live_before=%d\n", d, c->so_count_host[3]);
        }
        tend(c, s, 1, t0);
        // promotions of this chunk (diagnostics), the pool's live count, and the sync that frees
        // the argument staging
        HIP_TRY(c, hipMemcpyAsync(c->so_count_host + 2, c->so_count + 2, 2 * 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        // the drain is bounded by max_iter; a pool point still live past it would leave its results
        // unwritten — never returned as if solved
        if (nslots > 0 && c->so_count_host[3] != 0)
            return fail(c, SBR_EDEVICE, "social sweep: promoted points still live after the pool drain");
        if (nslots > 0) {
            const int64_t used = c->so_count_host[2];
            c->so_promoted += used < nslots ? used : nslots;
        }
        if (prof) {
            std::vector<int64_t> h((size_t)npts * 8);
            HIP_TRY(c, hipMemcpyAsync(h.data(), c->so_prof, h.size() * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
            HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
            for (size_t i = 0; i < h.size(); i++) c->so_prof_acc[i & 7] += h[i];
        }
    }
    return SBR_OK;
}

size_t pool_cap(size_t cap) { return cap * 16 < (size_t)kSocialMaxCap ? cap * 16 : (size_t)kSocialMaxCap; }

// Every point at the default knot capacity with a 16× promotion pool, then the
// (rare) points that outgrew the pool or found it full, from scratch, at 4× the
// pool capacity, up to kSocialMaxCap: the results are those of an unbounded
// grid.  Finding them synchronises `s` once.
int run_social(sbr_ctx* c, hipStream_t s, const double* beta, const double* eta, double x0, const double* u,
               int64_t n_beta, int64_t n_u, double p, double kappa, double lambda, const double* cmp, int32_t n_cmp,
               double tol, int32_t max_iter, const sbr_opts& o, sbr_result_soa* out, int32_t* fp_iters,
               int64_t* rk_steps, int poll)
{
    const int64_t n_total = n_beta * n_u;
    size_t cap = o.pad > 0 ? (size_t)o.pad : (size_t)kSocialDefaultCap;
    cap = (cap + 15) & ~(size_t)15; // 16-knot lines of the wave-blocked layout
    if (cap > (size_t)kSocialMaxCap) cap = (size_t)kSocialMaxCap;
    c->so_prof_acc.assign(8, 0);
    c->so_promoted = c->so_rerun = 0;
    int rc = run_social_pass(c, s, beta, eta, x0, u, n_u, p, kappa, lambda, cmp, n_cmp, tol, max_iter, o, out,
                             fp_iters, rk_steps, poll, cap, pool_cap(cap), nullptr, n_total);
    if (rc) return rc;
    std::vector<uint32_t> st((size_t)n_total);
    int64_t* dlist = nullptr;
    size_t reached = pool_cap(cap);
    while (reached < (size_t)kSocialMaxCap) {
        HIP_TRY(c, hipMemcpyAsync(st.data(), out->status, (size_t)n_total * 4, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        std::vector<int64_t> idx;
        for (int64_t g = 0; g < n_total; g++)
            if (st[(size_t)g] & SBR_KNOT_OVERFLOW) idx.push_back(g);
        if (idx.empty()) break;
        c->so_rerun += (int64_t)idx.size();
        cap = reached * 4 < (size_t)kSocialMaxCap ? reached * 4 : (size_t)kSocialMaxCap;
        reached = cap;
        if (dlist) (void)hipFree(dlist);
        dlist = nullptr;
        HIP_TRY(c, hipMalloc(&dlist, idx.size() * 8), SBR_ENOMEM);
        hipError_t e = hipMemcpyAsync(dlist, idx.data(), idx.size() * 8, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) { (void)hipFree(dlist); return fail(c, SBR_EDEVICE, "overflow list", e); }
        rc = run_social_pass(c, s, beta, eta, x0, u, n_u, p, kappa, lambda, cmp, n_cmp, tol, max_iter, o, out,
                             fp_iters, rk_steps, poll, cap, cap, dlist, (int64_t)idx.size());
        if (rc) { (void)hipFree(dlist); return rc; }
    }
    if (dlist) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(dlist);
    }
    return SBR_OK;
}
}  // namespace

extern "C" {

int sbr_sweep_social_dev(sbr_ctx* c, void* stream, const double* beta, const double* eta, double x0, const double* u,
                         int64_t n_beta, int64_t n_u, double p, double kappa, double lambda, const double* cmp_grid,
                         int32_t n_cmp, double tol, int32_t max_iter, const sbr_opts* opts, sbr_result_soa* out,
                         int32_t* fp_iters, int64_t* rk_steps)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_SINGLE_DEVICE(c);
    int rc = social_checks(c, beta, eta, u, n_beta, n_u, x0, p, kappa, lambda, cmp_grid, n_cmp, tol, max_iter, out);
    if (rc) return rc;
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    return fenced(c, stream, true, [&](hipStream_t s) {
        return run_social(c, s, beta, eta, x0, u, n_beta, n_u, p, kappa, lambda, cmp_grid, n_cmp, tol, max_iter, o,
                          out, fp_iters, rk_steps, 0);
    });
}

int sbr_social_point_paths(sbr_ctx* c, double beta, double eta, double x0, double u, double p, double kappa,
                           double lambda, const double* cmp_grid, int32_t n_cmp, double tol, int32_t max_iter,
                           const sbr_opts* opts, double* res, uint32_t* status, int32_t* fp_iters, double* t,
                           double* G, double* aw_old, int64_t cap, int64_t* n_knots)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    SBR_ON_RANK0(c, sbr_social_point_paths(c, beta, eta, x0, u, p, kappa, lambda, cmp_grid, n_cmp, tol, max_iter, opts, res, status, fp_iters, t, G, aw_old, cap, n_knots));
    if (!c || !res || !status || !t || !G || cap <= 0 || cap > (int64_t(1) << 30)) return SBR_EARG;
    double* d = nullptr;
    const size_t kc = (size_t)cap;
    HIP_TRY(c, hipMalloc(&d, (3 * kc + 8) * 8), SBR_ENOMEM);
    c->so_path_t = d;
    c->so_path_G = d + kc;
    c->so_path_aw = aw_old ? d + 2 * kc : nullptr;
    c->so_path_n = (int32_t*)(d + 3 * kc);
    c->so_path_cap = (int32_t)cap;
    hipError_t e = hipMemset(c->so_path_n, 0, 4);
    double xi, tin, tout, aw, tl;
    int64_t steps = 0;
    sbr_result_soa out{&xi, &tin, &tout, &aw, &tl, status, nullptr};
    int rc = e == hipSuccess ? sbr_sweep_social(c, &beta, &eta, x0, &u, 1, 1, p, kappa, lambda, cmp_grid, n_cmp, tol,
                                                max_iter, opts, &out, fp_iters, &steps)
                             : fail(c, SBR_EDEVICE, "hipMemset", e);
    c->so_path_t = c->so_path_G = c->so_path_aw = nullptr;
    c->so_path_n = nullptr;
    c->so_path_cap = 0;
    int32_t n = 0;
    if (rc == SBR_OK) {
        e = hipMemcpy(&n, d + 3 * kc, 4, hipMemcpyDeviceToHost);
        const int64_t m = n < 0 ? 0 : n;
        if (e == hipSuccess && m > 0) e = hipMemcpy(t, d, (size_t)m * 8, hipMemcpyDeviceToHost);
        if (e == hipSuccess && m > 0) e = hipMemcpy(G, d + kc, (size_t)m * 8, hipMemcpyDeviceToHost);
        if (e == hipSuccess && m > 0 && aw_old) e = hipMemcpy(aw_old, d + 2 * kc, (size_t)m * 8, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = fail(c, SBR_EDEVICE, "social path copy", e);
    }
    (void)hipFree(d);
    if (rc) return rc;
    res[0] = xi; res[1] = tin; res[2] = tout; res[3] = aw; res[4] = tl;
    if (n_knots) *n_knots = n < 0 ? -n : n;
    if (n < 0) return fail(c, SBR_EARG, "path capacity too small");
    return SBR_OK;
}

int sbr_sweep_social(sbr_ctx* c, const double* beta, const double* eta, double x0, const double* u, int64_t n_beta,
                     int64_t n_u, double p, double kappa, double lambda, const double* cmp_grid, int32_t n_cmp,
                     double tol, int32_t max_iter, const sbr_opts* opts, sbr_result_soa* out, int32_t* fp_iters,
                     int64_t* rk_steps)
{
    if (guess_set(opts)) return fail(c, SBR_EARG, "xi_guess: only sbr_equilibrium_on_knots takes a first iterate");
    int rc = social_checks(c, beta, eta, u, n_beta, n_u, x0, p, kappa, lambda, cmp_grid, n_cmp, tol, max_iter, out);
    if (rc) return rc;
    for (int64_t i = 0; i < n_beta; i++)
        if (!(beta[i] > 0.0) || !(eta[i] > 0.0)) return fail(c, SBR_EARG, "ArgumentError: beta/eta must be positive");
    for (int64_t j = 0; j < n_u; j++)
        if (!(u[j] >= 0.0)) return fail(c, SBR_EARG, "ArgumentError: u must be non-negative");
    if (c->multi)
        return multi_sweep_social(c, beta, eta, x0, u, n_beta, n_u, p, kappa, lambda, cmp_grid, n_cmp, tol, max_iter,
                                  resolve(opts), out, fp_iters, rk_steps);
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    sbr_opts o = resolve(opts);
    const size_t np = (size_t)(n_beta * n_u);
    const size_t in_d = 2 * (size_t)n_beta + (size_t)n_u + (size_t)n_beta * n_cmp;
    const size_t out_d = np * 5 + np + np + np; // 5 doubles | status+iters | fp_iters+pad | steps
    rc = ensure_stage(c, (in_d + out_d) * 8 + 1024);
    if (rc) return rc;
    double* d = (double*)c->stage;
    double *dbeta = d, *deta = dbeta + n_beta, *du = deta + n_beta, *dcmp = du + n_u;
    double* dres = dcmp + (size_t)n_beta * n_cmp;
    double *dxi = dres, *dtin = dxi + np, *dtout = dtin + np, *daw = dtout + np, *dtol = daw + np;
    uint32_t* dst = (uint32_t*)(dtol + np);
    int32_t* dit = (int32_t*)(dst + np);
    int32_t* dfp = dit + np;
    int64_t* dsteps = (int64_t*)(dfp + 2 * np);
    return fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        HIP_TRY(c, hipMemcpyAsync(dbeta, beta, (size_t)n_beta * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(deta, eta, (size_t)n_beta * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(du, u, (size_t)n_u * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(dcmp, cmp_grid, (size_t)n_beta * n_cmp * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        sbr_result_soa r{dxi, dtin, dtout, daw, dtol, dst, dit};
        rc = run_social(c, s, dbeta, deta, x0, du, n_beta, n_u, p, kappa, lambda, dcmp, n_cmp, tol, max_iter, o, &r, dfp,
                        dsteps, 8);
        if (rc) return rc;
        struct { void* h; const void* dv; size_t b; } cp[] = {
            {out->xi, dxi, np * 8}, {out->tau_in_unc, dtin, np * 8}, {out->tau_out_unc, dtout, np * 8},
            {out->aw_max, daw, np * 8}, {out->tol, dtol, np * 8}, {out->status, dst, np * 4},
            {out->iters, dit, np * 4}, {fp_iters, dfp, np * 4}, {rk_steps, dsteps, np * 8}};
        for (auto& x : cp)
            if (x.h) HIP_TRY(c, hipMemcpyAsync(x.h, x.dv, x.b, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        return SBR_OK;
    });
}

int sbr_device_info(sbr_ctx* c, int32_t* lds_bytes_per_block, int32_t* lds_knot_capacity, int32_t* cu_count)
{
    SBR_ON_RANK0(c, sbr_device_info(c, lds_bytes_per_block, lds_knot_capacity, cu_count));
    if (!c) return SBR_EARG;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    if (lds_bytes_per_block) *lds_bytes_per_block = c->lds_smem;
    if (lds_knot_capacity) *lds_knot_capacity = c->lds_cap;
    if (cu_count) *cu_count = cus;
    return SBR_OK;
}

void sbr_apply_early_exit(int64_t n_beta, int64_t n_u, int32_t threshold, sbr_result_soa* r)
{
    for (int64_t b = 0; b < n_beta; b++) {
        int32_t cnt = 0;
        for (int64_t j = 0; j < n_u; j++) {
            const int64_t o = b * n_u + j;
            if (cnt >= threshold) {
                r->xi[o] = NAN;
                r->aw_max[o] = NAN;
                r->tol[o] = INFINITY;
                r->status[o] = SBR_SKIPPED_EARLY_EXIT;
                continue;
            }
            if (r->status[o] & SBR_RUN) cnt = 0;
            else cnt++;
        }
    }
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Diagnostics: evaluate the shared deterministic math on the device so tests
// can check host/device bit equality of sbr_exp / sbr_log / sbr_pow_pos.
// ---------------------------------------------------------------------------
namespace {
__global__ void detmath_kernel(const double* x, const double* y, int n, double* e, double* l, double* pw)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    e[i] = sbr_exp(x[i]);
    l[i] = sbr_log(x[i]);
    pw[i] = sbr_pow_pos(x[i], y[i]);
}

__global__ void fastpow_kernel(const double* x, const double* y, int n, double* out)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = sbr_fastpow(x[i], y[i]);
}
}  // namespace

extern "C" int sbr_selftest_fastpow(sbr_ctx* c, const double* x, const double* y, int n, double* out)
{
    SBR_ON_RANK0(c, sbr_selftest_fastpow(c, x, y, n, out));
    if (!c || n <= 0 || !x || !y || !out) return SBR_EARG;
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    int rc = ensure_stage(c, (size_t)n * 3 * 8);
    if (rc) return rc;
    return fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        double* d = (double*)c->stage;
        HIP_TRY(c, hipMemcpyAsync(d, x, n * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(d + n, y, n * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        hipLaunchKernelGGL(fastpow_kernel, dim3((n + 255) / 256), dim3(256), 0, s, d, d + n, n, d + 2 * n);
        HIP_TRY(c, hipGetLastError(), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(out, d + 2 * n, n * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        return SBR_OK;
    });
}

extern "C" int sbr_selftest_detmath(sbr_ctx* c, const double* x, const double* y, int n, double* e, double* l,
                                    double* pw)
{
    SBR_ON_RANK0(c, sbr_selftest_detmath(c, x, y, n, e, l, pw));
    if (!c || n <= 0) return SBR_EARG;
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, SBR_EDEVICE, "hipSetDevice");
    int rc = ensure_stage(c, (size_t)n * 5 * 8);
    if (rc) return rc;
    double* d = (double*)c->stage;
    return fenced(c, nullptr, false, [&](hipStream_t s) -> int {
        HIP_TRY(c, hipMemcpyAsync(d, x, n * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(d + n, y, n * 8, hipMemcpyHostToDevice, s), SBR_EDEVICE);
        hipLaunchKernelGGL(detmath_kernel, dim3((n + 255) / 256), dim3(256), 0, s, d, d + n, n, d + 2 * n, d + 3 * n,
                           d + 4 * n);
        HIP_TRY(c, hipGetLastError(), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(e, d + 2 * n, n * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(l, d + 3 * n, n * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipMemcpyAsync(pw, d + 4 * n, n * 8, hipMemcpyDeviceToHost, s), SBR_EDEVICE);
        HIP_TRY(c, hipStreamSynchronize(s), SBR_EDEVICE);
        return SBR_OK;
    });
}

namespace {

// ---------------------------------------------------------------------------
// n-device contexts: the host-pointer sweeps fan out over the ranks (sbr_multi.hip).
// Inputs of column i go to rank i mod N; each rank runs the single-device *_dev
// entry point on its GPU; the packed results come back over RCCL.
// ---------------------------------------------------------------------------
using sbr_multi_impl::FieldSpec;

// the rank's columns r, r+N, … of a per-column array with `w` values per column
constexpr auto gather_cols = sbr_shard::deal_cols;

int stage_host(void* dev, const std::vector<double>& h)
{
    return hipMemcpy(dev, h.data(), h.size() * 8, hipMemcpyHostToDevice) == hipSuccess ? SBR_OK : SBR_EDEVICE;
}

int multi_sweep_baseline(sbr_ctx* c, const double* beta, const double* eta, const double* t_end, double x0,
                         const double* u, int64_t n_beta, int64_t n_u, double p, double kappa, double lambda,
                         const sbr_opts& o, sbr_result_soa* out)
{
    const int N = sbr_multi_impl::size(c->multi);
    const int64_t cmax = (n_beta + N - 1) / N;
    std::vector<FieldSpec> fs = {{out->xi, 8, 1},  {out->tau_in_unc, 8, 1}, {out->tau_out_unc, 8, 1},
                                 {out->aw_max, 8, 1}, {out->tol, 8, 1},      {out->status, 4, 1},
                                 {out->iters, 4, 1}};
    auto stage = [&](int r, int64_t nc, void* in, hipStream_t) -> int {
        std::vector<double> h(3 * nc + n_u);
        gather_cols(beta, 1, r, N, nc, h.data());
        gather_cols(eta, 1, r, N, nc, h.data() + nc);
        gather_cols(t_end, 1, r, N, nc, h.data() + 2 * nc);
        memcpy(h.data() + 3 * nc, u, (size_t)n_u * 8);
        return stage_host(in, h);
    };
    auto run = [&](int, int64_t nc, sbr_ctx* kid, hipStream_t s, void* in, const std::vector<void*>& f) -> int {
        const double* d = (const double*)in;
        sbr_result_soa ro{(double*)f[0], (double*)f[1], (double*)f[2], (double*)f[3], (double*)f[4],
                          (uint32_t*)f[5], (int32_t*)f[6]};
        return sbr_sweep_baseline_dev(kid, s, d, d + nc, d + 2 * nc, x0, d + 3 * nc, nc, n_u, p, kappa, lambda, &o,
                                      &ro);
    };
    int rc = sbr_multi_impl::run_sharded(c->multi, n_beta, n_u, fs, (size_t)(3 * cmax + n_u) * 8, stage, run, (o.flags & SBR_FLAG_RCCL_GATHER) != 0);
    if (rc) return fail(c, rc, sbr_multi_impl::last_error(c->multi));
    if (o.early_exit_nan_run > 0 && out->status && out->xi && out->aw_max && out->tol)
        sbr_apply_early_exit(n_beta, n_u, o.early_exit_nan_run, out);
    return SBR_OK;
}

int multi_sweep_interest(sbr_ctx* c, const double* beta, const double* eta, const double* t_end, double x0,
                         const double* u, int64_t n_beta, int64_t n_u, double p, double kappa, double lambda, double r_,
                         double delta, const sbr_opts& o, sbr_result_soa* out, int64_t* rk_steps)
{
    const int N = sbr_multi_impl::size(c->multi);
    const int64_t cmax = (n_beta + N - 1) / N;
    std::vector<FieldSpec> fs = {{out->xi, 8, 1},  {out->tau_in_unc, 8, 1}, {out->tau_out_unc, 8, 1},
                                 {out->aw_max, 8, 1}, {out->tol, 8, 1},      {out->status, 4, 1},
                                 {out->iters, 4, 1},  {rk_steps, 8, 1}};
    auto stage = [&](int r, int64_t nc, void* in, hipStream_t) -> int {
        std::vector<double> h(3 * nc + n_u);
        gather_cols(beta, 1, r, N, nc, h.data());
        gather_cols(eta, 1, r, N, nc, h.data() + nc);
        gather_cols(t_end, 1, r, N, nc, h.data() + 2 * nc);
        memcpy(h.data() + 3 * nc, u, (size_t)n_u * 8);
        return stage_host(in, h);
    };
    auto run = [&](int, int64_t nc, sbr_ctx* kid, hipStream_t s, void* in, const std::vector<void*>& f) -> int {
        const double* d = (const double*)in;
        sbr_result_soa ro{(double*)f[0], (double*)f[1], (double*)f[2], (double*)f[3], (double*)f[4],
                          (uint32_t*)f[5], (int32_t*)f[6]};
        return sbr_sweep_interest_dev(kid, s, d, d + nc, d + 2 * nc, x0, d + 3 * nc, nc, n_u, p, kappa, lambda, r_,
                                      delta, &o, &ro, (int64_t*)f[7]);
    };
    int rc = sbr_multi_impl::run_sharded(c->multi, n_beta, n_u, fs, (size_t)(3 * cmax + n_u) * 8, stage, run, (o.flags & SBR_FLAG_RCCL_GATHER) != 0);
    return rc ? fail(c, rc, sbr_multi_impl::last_error(c->multi)) : SBR_OK;
}

int multi_sweep_hetero(sbr_ctx* c, int32_t K, const double* betas, const double* dist, const double* eta,
                       const double* t_end, double x0, const double* u, int64_t n_col, int64_t n_u, double p,
                       double kappa, double lambda, const sbr_opts& o, sbr_result_soa* out, double* tau_in,
                       double* tau_out)
{
    const int N = sbr_multi_impl::size(c->multi);
    const int64_t cmax = (n_col + N - 1) / N;
    std::vector<FieldSpec> fs = {{out->xi, 8, 1},    {out->aw_max, 8, 1}, {out->tol, 8, 1},
                                 {out->status, 4, 1}, {out->iters, 4, 1},  {tau_in, 8, (size_t)K},
                                 {tau_out, 8, (size_t)K}};
    auto stage = [&](int r, int64_t nc, void* in, hipStream_t) -> int {
        std::vector<double> h(nc * K + K + 2 * nc + n_u);
        gather_cols(betas, K, r, N, nc, h.data());
        memcpy(h.data() + nc * K, dist, (size_t)K * 8);
        gather_cols(eta, 1, r, N, nc, h.data() + nc * K + K);
        gather_cols(t_end, 1, r, N, nc, h.data() + nc * K + K + nc);
        memcpy(h.data() + nc * K + K + 2 * nc, u, (size_t)n_u * 8);
        return stage_host(in, h);
    };
    auto run = [&](int, int64_t nc, sbr_ctx* kid, hipStream_t s, void* in, const std::vector<void*>& f) -> int {
        const double* d = (const double*)in;
        const double *db = d, *dd = d + nc * K, *de = dd + K, *dt = de + nc, *du = dt + nc;
        sbr_result_soa ro{(double*)f[0], nullptr, nullptr, (double*)f[1], (double*)f[2], (uint32_t*)f[3],
                          (int32_t*)f[4]};
        return sbr_sweep_hetero_dev(kid, s, K, db, dd, de, dt, x0, du, nc, n_u, p, kappa, lambda, &o, &ro,
                                    (double*)f[5], (double*)f[6]);
    };
    int rc = sbr_multi_impl::run_sharded(c->multi, n_col, n_u, fs, (size_t)(cmax * K + K + 2 * cmax + n_u) * 8,
                                         stage, run, (o.flags & SBR_FLAG_RCCL_GATHER) != 0);
    return rc ? fail(c, rc, sbr_multi_impl::last_error(c->multi)) : SBR_OK;
}

int multi_sweep_social(sbr_ctx* c, const double* beta, const double* eta, double x0, const double* u, int64_t n_beta,
                       int64_t n_u, double p, double kappa, double lambda, const double* cmp_grid, int32_t n_cmp,
                       double tol, int32_t max_iter, const sbr_opts& o, sbr_result_soa* out, int32_t* fp_iters,
                       int64_t* rk_steps)
{
    const int N = sbr_multi_impl::size(c->multi);
    const int64_t cmax = (n_beta + N - 1) / N;
    std::vector<FieldSpec> fs = {{out->xi, 8, 1},  {out->tau_in_unc, 8, 1}, {out->tau_out_unc, 8, 1},
                                 {out->aw_max, 8, 1}, {out->tol, 8, 1},      {out->status, 4, 1},
                                 {out->iters, 4, 1},  {fp_iters, 4, 1},      {rk_steps, 8, 1}};
    auto stage = [&](int r, int64_t nc, void* in, hipStream_t) -> int {
        std::vector<double> h(2 * nc + n_u + nc * n_cmp);
        gather_cols(beta, 1, r, N, nc, h.data());
        gather_cols(eta, 1, r, N, nc, h.data() + nc);
        memcpy(h.data() + 2 * nc, u, (size_t)n_u * 8);
        gather_cols(cmp_grid, n_cmp, r, N, nc, h.data() + 2 * nc + n_u);
        return stage_host(in, h);
    };
    auto run = [&](int, int64_t nc, sbr_ctx* kid, hipStream_t s, void* in, const std::vector<void*>& f) -> int {
        const double* d = (const double*)in;
        sbr_result_soa ro{(double*)f[0], (double*)f[1], (double*)f[2], (double*)f[3], (double*)f[4],
                          (uint32_t*)f[5], (int32_t*)f[6]};
        return sbr_sweep_social_dev(kid, s, d, d + nc, x0, d + 2 * nc, nc, n_u, p, kappa, lambda, d + 2 * nc + n_u,
                                    n_cmp, tol, max_iter, &o, &ro, (int32_t*)f[7], (int64_t*)f[8]);
    };
    int rc = sbr_multi_impl::run_sharded(c->multi, n_beta, n_u, fs, (size_t)(2 * cmax + n_u + cmax * n_cmp) * 8,
                                         stage, run, (o.flags & SBR_FLAG_RCCL_GATHER) != 0);
    return rc ? fail(c, rc, sbr_multi_impl::last_error(c->multi)) : SBR_OK;
}
}  // namespace
