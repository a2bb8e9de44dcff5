// Why is the learning launch's first wave (β = 1e4 .. 32, the head of β = 1/range(1e-4, 1, 2048))
// ~50 % slower than the others at the same step count?  Runs 64 consecutive columns of that
// grid with S active lanes per wave (64/S waves, one per CU), the scalar ODE loop of
// csrc/sbr_ode.h without stores, and prints each wave's time (s_memtime cycles / realtime):
// if S = 1 (every column alone) is much faster than S = 64, the cost is lane divergence
// inside the wave, and the learning launch should spread the head columns over more waves.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -o tools/ubench_spread tools/ubench_spread.hip
#include "../replication-social-bank-runs_amd/csrc/sbr_ode.h"
#include <cstdio>
#include <vector>

using namespace sbr;

struct CountSink {
    int n = 0;
    __device__ bool start(double, double) { return true; }
    __device__ bool step(bool acc, double, double, double, double, double, const StepK&, bool)
    {
        n += acc ? 1 : 0;
        return true;
    }
};

// wave w (one 64-thread block) runs columns c0 + w·S + l for lanes l < S
__global__ __launch_bounds__(64) void spread(const double* beta, int c0, int S, long long* out)
{
    const int l = threadIdx.x, w = blockIdx.x;
    const bool live = l < S;
    const double B = live ? beta[c0 + w * S + l] : 1.0;
    long long steps = 0;
    const long long a0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if (live) {
        LogisticSys f{B};
        CountSink sink;
        OdeOut o;
        ode_scalar(f, sink, 30.0, 1e-4, DBL_EPS, DBL_EPS, 1000000, o);
        steps = o.naccept + o.nreject;
    }
    const long long a1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (live) out[3 * (c0 + w * S + l) + 2] = steps;
    if (l == 0) { out[3 * (c0 + w * S)] = a1 - a0; out[3 * (c0 + w * S) + 1] = r1 - r0; }
}

int main()
{
    std::vector<double> hb(2048);
    for (int i = 0; i < 2048; i++) hb[i] = 1.0 / (1e-4 + (1.0 - 1e-4) * i / 2047.0);
    double* db;
    long long* dout;
    (void)hipMalloc(&db, 2048 * 8);
    (void)hipMalloc(&dout, 2048 * 3 * 8);
    (void)hipMemcpy(db, hb.data(), 2048 * 8, hipMemcpyHostToDevice);
    std::vector<long long> h(2048 * 3);
    for (int c0 : {0, 64, 256, 1024}) {
        for (int S : {64, 32, 16, 8, 4, 2, 1}) {
            const int nw = 64 / S;
            double mx = 0, mn = 1e30;
            for (int rep = 0; rep < 2; rep++) { // second launch timed (warm)
                hipLaunchKernelGGL(spread, dim3(nw), dim3(64), 0, 0, db, c0, S, dout);
                (void)hipDeviceSynchronize();
            }
            (void)hipMemcpy(h.data(), dout, h.size() * 8, hipMemcpyDeviceToHost);
            long long smax = 0;
            printf("cols %4d..%4d S=%2d:", c0, c0 + 63, S);
            for (int w = 0; w < nw; w++) {
                const int c = c0 + w * S;
                const double us = h[3 * c + 1] / 100.0; // realtime ticks at 100 MHz
                mx = us > mx ? us : mx;
                mn = us < mn ? us : mn;
                for (int l = 0; l < S; l++) smax = h[3 * (c + l) + 2] > smax ? h[3 * (c + l) + 2] : smax;
                if (nw <= 8 || w < 4 || w >= nw - 2) printf(" w%d %.0f", w, us);
                else if (w == 4) printf(" ...");
            }
            printf(" | max %.0f us, min %.0f us, max steps %lld, cycles/step (w0) %.0f\n", mx, mn, smax,
                   (double)h[3 * c0] / (double)h[3 * c0 + 2]);
            fflush(stdout);
        }
    }
    return 0;
}
