// The pipelined batch's first learning launch (20 config-3 grids = 640 waves of 64 columns,
// β = 1/range(1e-4, 1, 2048) per grid) lasts as long as its slowest wave: the wave holding
// column 22 (4.45k Tsit5 steps against a 2.9k median).  Does isolating every grid's first
// wave(s) — the large-β head of a β-descending grid, where the long columns sit — on CUs of
// their own (CU-masked streams) shorten the launch?  Columns integrate ode_scalar (csrc/sbr_ode.h)
// and store (t, G) at every attempted step like learn_logistic_kernel (row per column, padded
// stride).  Prints the launch span for each layout, and per-wave end times of the one-launch
// layout (head waves vs the rest).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -o tools/ubench_fill tools/ubench_fill.hip
#include "../replication-social-bank-runs_amd/csrc/sbr_ode.h"
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdio>
#include <vector>
#include <cstdlib>
#include <unistd.h>

using namespace sbr;

constexpr int CAP = 8192, LD = CAP + 16, NB = 2048, WPG = NB / 64;

struct StoreSink {
    double *T, *G;
    int n = 0;
    __device__ bool push(bool acc, double t, double x)
    {
        const bool room = n < CAP - 1;
        if (room) { T[n] = t; G[n] = x; }
        n += (acc & room) ? 1 : 0;
        return true;
    }
    __device__ bool start(double t, double x) { return push(true, t, x); }
    __device__ bool step(bool acc, double, double tn, double, double, double y1, const StepK&, bool)
    {
        return push(acc, tn, y1);
    }
};

__device__ long long g_end[4096];
__device__ unsigned g_hw[4096][2]; // HW_ID, XCC_ID of each wave
__device__ long long g_t0;

// part 0: every wave; part 1: waves w % WPG < H of each grid; part 2: the others
// part 3: one launch, the nh head waves first (blocks [0, nh)), then the others
__global__ __launch_bounds__(64) void learn(const double* beta, double* T, double* G, int part, int H, int nh = 0)
{
    extern __shared__ double blocker[]; // a head launch may reserve LDS to keep other waves off its CU
    if (threadIdx.x == 0 && part == 1 && nh < 0) blocker[0] = 0.0;
    int w = blockIdx.x;
    if (part == 3) {
        if (w < nh) part = 1;
        else { part = 2; w -= nh; }
    }
    if (part == 1) w = (w / H) * WPG + w % H;
    else if (part == 2) w = (w / (WPG - H)) * WPG + H + w % (WPG - H);
    const int col = w * 64 + threadIdx.x;
    StoreSink s{T + (size_t)col * LD, G + (size_t)col * LD};
    LogisticSys f{beta[col % NB]};
    OdeOut o;
    ode_scalar(f, s, 30.0, 1e-4, DBL_EPS, DBL_EPS, 1000000, o);
    if (threadIdx.x == 0) {
        g_end[w] = __builtin_amdgcn_s_memrealtime();
        g_hw[w][0] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));  // HW_ID
        g_hw[w][1] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11)); // XCC_ID
    }
}

__global__ void stamp() { g_t0 = __builtin_amdgcn_s_memrealtime(); }

int main(int argc, char** argv)
{
    // argv: ngrid, then the head-CU counts to try
    std::vector<int> nh_list;
    const int ngrid = argc > 1 ? atoi(argv[1]) : 20;
    for (int i = 2; i < argc; i++) nh_list.push_back(atoi(argv[i]));
    setvbuf(stdout, nullptr, _IONBF, 0); // every line reaches the log at once
    const int nw = ngrid * WPG;
    if (nw > 4096) return 1;
    std::vector<double> hb(NB);
    for (int i = 0; i < NB; i++) hb[i] = 1.0 / (1e-4 + (1.0 - 1e-4) * i / (NB - 1.0));
    double *db, *T, *G;
    (void)hipMalloc(&db, NB * 8);
    (void)hipMemcpy(db, hb.data(), NB * 8, hipMemcpyHostToDevice);
    (void)hipMalloc(&T, (size_t)nw * 64 * LD * 8);
    (void)hipMalloc(&G, (size_t)nw * 64 * LD * 8);
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    hipStream_t s0;
    (void)hipStreamCreate(&s0);
    hipEvent_t e0, e1, eh, et;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); (void)hipEventCreate(&eh); (void)hipEventCreate(&et);
    auto masked = [&](int lo, int hi) { // a stream on CUs [lo, hi)
        std::vector<uint32_t> m((ncu + 31) / 32, 0u);
        for (int i = lo; i < hi; i++) m[i / 32] |= 1u << (i % 32);
        hipStream_t s;
        (void)hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data());
        return s;
    };
    std::vector<long long> end(nw);
    auto report_ends = [&](const char* name) {
        long long t0 = 0;
        (void)hipMemcpyFromSymbol(&t0, HIP_SYMBOL(g_t0), 8);
        (void)hipMemcpyFromSymbol(end.data(), HIP_SYMBOL(g_end), nw * 8);
        std::vector<double> head, rest;
        for (int w = 0; w < nw; w++) ((w % WPG) == 0 ? head : rest).push_back((end[w] - t0) / 100.0);
        std::sort(head.begin(), head.end());
        std::sort(rest.begin(), rest.end());
        auto q = [](std::vector<double>& v, double f) { return v[(size_t)(f * (v.size() - 1))]; };
        std::vector<unsigned> hw(2 * nw);
        (void)hipMemcpyFromSymbol(hw.data(), HIP_SYMBOL(g_hw), nw * 8);
        std::vector<int> seen;
        int maxper = 0;
        {
            std::vector<int> cnt(1 << 16, 0);
            for (int w = 0; w < nw; w += WPG) {
                const unsigned h = hw[2 * w], x = hw[2 * w + 1] & 0xf;
                const int cu = (int)((x << 8) | (((h >> 13) & 7) << 5) | (((h >> 12) & 1) << 4) | ((h >> 8) & 15));
                if (cnt[cu]++ == 0) seen.push_back(cu);
                maxper = cnt[cu] > maxper ? cnt[cu] : maxper;
            }
        }
        printf("  %s: head waves on %zu distinct CUs (max %d per CU)\n", name, seen.size(), maxper);
        printf("  %s: head waves end %.0f..%.0f us (median %.0f); other waves median %.0f, p90 %.0f, max %.0f us\n", name,
               head.front(), head.back(), q(head, 0.5), q(rest, 0.5), q(rest, 0.9), rest.back());
    };
    printf("CUs %d, %d waves (%d grids x %d)\n", ncu, nw, ngrid, WPG);
    // one launch (the library's wide learning launch)
    for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(e0, s0);
        hipLaunchKernelGGL(stamp, dim3(1), dim3(1), 0, s0);
        hipLaunchKernelGGL(learn, dim3(nw), dim3(64), 0, s0, db, T, G, 0, 0);
        (void)hipEventRecord(e1, s0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("one launch: %.3f ms\n", ms);
        if (rep == 2) report_ends("one launch");
    }
    // one launch, heads first
    for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(e0, s0);
        hipLaunchKernelGGL(stamp, dim3(1), dim3(1), 0, s0);
        hipLaunchKernelGGL(learn, dim3(nw), dim3(64), 0, s0, db, T, G, 3, 1, ngrid);
        (void)hipEventRecord(e1, s0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("one launch, heads first: %.3f ms\n", ms);
        if (rep == 2) report_ends("heads first");
    }
    // heads (H waves per grid) on CUs [0, nh), the rest on [nh, ncu): NH_LIST from argv, one
    // pair of masked streams per configuration, never destroyed (as the library holds them)
    auto masked_ok = [&](int lo, int hi, hipStream_t* s) {
        std::vector<uint32_t> m((ncu + 31) / 32, 0u);
        for (int i = lo; i < hi; i++) m[i / 32] |= 1u << (i % 32);
        const hipError_t e = hipExtStreamCreateWithCUMask(s, (uint32_t)m.size(), m.data());
        printf("  mask [%d, %d): %s\n", lo, hi, hipGetErrorString(e));
        return e == hipSuccess;
    };
    for (int nh : nh_list) {
        const int H = 1;
        hipStream_t sh, st;
        if (!masked_ok(0, nh, &sh) || !masked_ok(nh, ncu, &st)) { printf("mask creation failed\n"); return 1; }
        float best = 1e9f;
        for (int rep = 0; rep < 5; rep++) {
            (void)hipEventRecord(e0, s0);
            (void)hipStreamWaitEvent(sh, e0, 0);
            (void)hipStreamWaitEvent(st, e0, 0);
            hipLaunchKernelGGL(stamp, dim3(1), dim3(1), 0, sh);
            hipLaunchKernelGGL(learn, dim3(ngrid * H), dim3(64), 0, sh, db, T, G, 1, H);
            hipLaunchKernelGGL(learn, dim3(ngrid * (WPG - H)), dim3(64), 0, st, db, T, G, 2, H);
            (void)hipEventRecord(eh, sh);
            (void)hipEventRecord(et, st);
            (void)hipStreamWaitEvent(s0, eh, 0);
            (void)hipStreamWaitEvent(s0, et, 0);
            (void)hipEventRecord(e1, s0);
            // bounded wait: give up (and say so) instead of hanging the box
            int polls = 0;
            while (hipEventQuery(e1) == hipErrorNotReady && polls < 20000) { usleep(100); polls++; }
            if (polls >= 20000) { printf("  TIMEOUT waiting for nh=%d rep %d\n", nh, rep); return 2; }
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            printf("  nh=%d rep %d: %.3f ms\n", nh, rep, ms);
            best = ms < best ? ms : best;
        }
        printf("heads H=%d on %d CUs, rest on %d: %.3f ms\n", H, nh, ncu - nh, best);
        char nm[64];
        snprintf(nm, sizeof nm, "H=%d/%d CUs", H, nh);
        report_ends(nm);
    }
    // heads first on an unmasked stream, rest after on another (no masks)
    if (nh_list.empty()) {
        hipStream_t sh, st;
        (void)hipStreamCreate(&sh);
        (void)hipStreamCreate(&st);
        float best = 1e9f;
        for (int rep = 0; rep < 3; rep++) {
            (void)hipEventRecord(e0, s0);
            (void)hipStreamWaitEvent(sh, e0, 0);
            (void)hipStreamWaitEvent(st, e0, 0);
            hipLaunchKernelGGL(stamp, dim3(1), dim3(1), 0, sh);
            hipLaunchKernelGGL(learn, dim3(ngrid), dim3(64), 0, sh, db, T, G, 1, 1);
            hipLaunchKernelGGL(learn, dim3(ngrid * (WPG - 1)), dim3(64), 0, st, db, T, G, 2, 1);
            (void)hipEventRecord(eh, sh);
            (void)hipEventRecord(et, st);
            (void)hipStreamWaitEvent(s0, eh, 0);
            (void)hipStreamWaitEvent(s0, et, 0);
            (void)hipEventRecord(e1, s0);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        printf("heads then rest, two plain streams: %.3f ms\n", best);
        report_ends("plain streams");
        // the same with the head launch reserving LDS (no tail wave fits beside it)
        for (int kb : {64, 96, 120, 128, 160}) {
            const size_t lds = (size_t)kb * 1024;
            const hipError_t ea = hipFuncSetAttribute((const void*)learn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            best = 1e9f;
            bool ok = ea == hipSuccess;
            for (int rep = 0; ok && rep < 3; rep++) {
                (void)hipEventRecord(e0, s0);
                (void)hipStreamWaitEvent(sh, e0, 0);
                (void)hipStreamWaitEvent(st, e0, 0);
                hipLaunchKernelGGL(stamp, dim3(1), dim3(1), 0, sh);
                hipLaunchKernelGGL(learn, dim3(ngrid), dim3(64), lds, sh, db, T, G, 1, 1, -1);
                ok = hipGetLastError() == hipSuccess;
                hipLaunchKernelGGL(learn, dim3(ngrid * (WPG - 1)), dim3(64), 0, st, db, T, G, 2, 1, 0);
                (void)hipEventRecord(eh, sh);
                (void)hipEventRecord(et, st);
                (void)hipStreamWaitEvent(s0, eh, 0);
                (void)hipStreamWaitEvent(s0, et, 0);
                (void)hipEventRecord(e1, s0);
                int polls = 0;
                while (hipEventQuery(e1) == hipErrorNotReady && polls < 20000) { usleep(100); polls++; }
                if (polls >= 20000) { printf("  TIMEOUT lds %d KiB\n", kb); return 2; }
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            printf("heads (LDS %d KiB) then rest, two plain streams: %s %.3f ms\n", kb, ok ? "ok" : "launch failed", best);
            if (ok) { char nm[64]; snprintf(nm, sizeof nm, "LDS %d KiB", kb); report_ends(nm); }
        }
    }
    return 0;
}
