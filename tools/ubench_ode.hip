// Phase costs of the scalar learning ODE loop (csrc/sbr_ode.h) for one wave64 alone on
// a SIMD — how learn_logistic_kernel runs.  s_memtime (shader clock) and s_memrealtime
// (100 MHz) bracket each part, so cycles/step and the clock are both reported.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -o tools/ubench_ode tools/ubench_ode.hip
#include "../replication-social-bank-runs_amd/csrc/sbr_ode.h"
#include <cstdio>

using namespace sbr;

struct NullSink {
    int n = 0;
    __device__ bool start(double, double) { return true; }
    __device__ bool step(bool acc, double, double, double, double, double, const StepK&, bool)
    {
        n += acc ? 1 : 0;
        return true;
    }
};

// knot stores as learn_logistic_kernel makes them: one row of `cap` doubles per column
// (stride = column-major rows, the hazard / equilibrium kernels' layout) or knot-major
struct StoreSink {
    double* T;
    double* G;
    size_t stride; // distance between consecutive knots of one column
    int n = 0, cap;
    __device__ bool push(bool acc, double t, double x)
    {
        const bool room = n < cap;
        if (room) { T[(size_t)n * stride] = t; G[(size_t)n * stride] = x; }
        n += (acc & room) ? 1 : 0;
        return true;
    }
    __device__ bool start(double t, double x) { return push(true, t, x); }
    __device__ bool step(bool acc, double, double tn, double, double, double y1, const StepK&, bool)
    {
        return push(acc, tn, y1);
    }
};

// the same stores with the nontemporal hint (streamed past the caches' allocation)
struct NtStoreSink {
    double* T;
    double* G;
    int n = 0, cap;
    __device__ bool push(bool acc, double t, double x)
    {
        const bool room = n < cap;
        if (room) { __builtin_nontemporal_store(t, T + n); __builtin_nontemporal_store(x, G + n); }
        n += (acc & room) ? 1 : 0;
        return true;
    }
    __device__ bool start(double t, double x) { return push(true, t, x); }
    __device__ bool step(bool acc, double, double tn, double, double, double y1, const StepK&, bool)
    {
        return push(acc, tn, y1);
    }
};

#define OPAQUE(x) asm volatile("" : "+v"(x))
constexpr int REPS = 2048;

__device__ double* g_T;
__device__ double* g_G;

template <int PART>
__global__ void part(const double* beta, double* out, long long* cyc, long long* rt, long long* steps)
{
    const double B = PART >= 6 ? beta[blockIdx.x * 64 + threadIdx.x] : beta[threadIdx.x & 63];
    if (PART == 8) { // the full loop without stores on the bench grid's columns (compare with 6 / 9)
        LogisticSys f{B};
        NullSink sink;
        OdeOut o;
        const long long a0 = __builtin_amdgcn_s_memtime();
        ode_scalar(f, sink, 30.0, 1e-4, DBL_EPS, DBL_EPS, 1000000, o);
        const long long a1 = __builtin_amdgcn_s_memtime();
        out[blockIdx.x * blockDim.x + threadIdx.x] = (double)sink.n;
        if (threadIdx.x == 0 && blockIdx.x == 0) { cyc[0] = a1 - a0; rt[0] = 1; steps[0] = o.naccept + o.nreject; }
        return;
    }
    if (PART == 9) { // nontemporal knot stores, row per column
        const int col = blockIdx.x * 64 + threadIdx.x;
        constexpr int cap = 4096;
        NtStoreSink sink{g_T + (size_t)col * cap, g_G + (size_t)col * cap, 0, cap};
        LogisticSys f{B};
        OdeOut o;
        const long long a0 = __builtin_amdgcn_s_memtime();
        ode_scalar(f, sink, 30.0, 1e-4, DBL_EPS, DBL_EPS, 1000000, o);
        const long long a1 = __builtin_amdgcn_s_memtime();
        out[blockIdx.x * blockDim.x + threadIdx.x] = (double)sink.n;
        if (threadIdx.x == 0 && blockIdx.x == 0) { cyc[0] = a1 - a0; rt[0] = 1; steps[0] = o.naccept + o.nreject; }
        return;
    }
    double acc = 0.0;
    long long nsteps = 0;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if (PART == 0) { // the full loop on the config-3 column (T = 30)
        LogisticSys f{B};
        NullSink sink;
        OdeOut o;
        ode_scalar(f, sink, 30.0, 1e-4, DBL_EPS, DBL_EPS, 1000000, o);
        nsteps = o.naccept + o.nreject;
        acc = (double)sink.n;
    } else if (PART == 6 || PART == 7) { // full loop with the knot stores (6: row per column, 7: knot-major)
        const int col = blockIdx.x * 64 + threadIdx.x, ncol = gridDim.x * 64;
        constexpr int cap = 4096;
        StoreSink sink{PART == 6 ? g_T + (size_t)col * cap : g_T + col, PART == 6 ? g_G + (size_t)col * cap : g_G + col,
                       PART == 6 ? (size_t)1 : (size_t)ncol, 0, cap};
        LogisticSys f{B};
        OdeOut o;
        ode_scalar(f, sink, 30.0, 1e-4, DBL_EPS, DBL_EPS, 1000000, o);
        nsteps = o.naccept + o.nreject;
        acc = (double)sink.n;
    } else if (PART == 1) { // Tsit5 stages + error estimate, x chained
        double x = 1e-4 * (1.0 + threadIdx.x * 1e-3), dt = 1e-3, k1 = B * x * (1.0 - x);
        OPAQUE(dt);
        for (int i = 0; i < REPS; i++) {
            double tmp = fma(dt * A21, k1, x);
            const double k2 = (B * tmp) * (1.0 - tmp);
            tmp = fma(dt, fma(A31, k1, A32 * k2), x);
            const double k3 = (B * tmp) * (1.0 - tmp);
            tmp = fma(dt, fma(A41, k1, fma(A42, k2, A43 * k3)), x);
            const double k4 = (B * tmp) * (1.0 - tmp);
            tmp = fma(dt, fma(A51, k1, fma(A52, k2, fma(A53, k3, A54 * k4))), x);
            const double k5 = (B * tmp) * (1.0 - tmp);
            const double tmp6 = fma(dt, fma(A61, k1, fma(A62, k2, fma(A63, k3, fma(A64, k4, A65 * k5)))), x);
            const double k6 = (B * tmp6) * (1.0 - tmp6);
            const double u = fma(dt, fma(A71, k1, fma(A72, k2, fma(A73, k3, fma(A74, k4, fma(A75, k5, A76 * k6))))), x);
            const double k7 = (B * u) * (1.0 - u);
            const double ut =
                dt * fma(BT1, k1, fma(BT2, k2, fma(BT3, k3, fma(BT4, k4, fma(BT5, k5, fma(BT6, k6, BT7 * k7))))));
            const double EEst = fabs(ut / fma(dmax(fabs(x), fabs(u)), DBL_EPS, DBL_EPS));
            acc += EEst;
            x = u;
            k1 = k7;
        }
        nsteps = REPS;
    } else if (PART == 2) { // PI controller pass, chained through dt
        PIControl pc;
        double dt = 1e-3, E = 0.3 + threadIdx.x * 1e-3;
        OPAQUE(E);
        for (int i = 0; i < REPS; i++) {
            bool a;
            dt = pc.next_dt(E * (dt * 1e3), dt, 30.0, 1e-14, a);
        }
        acc = dt;
        nsteps = REPS;
    } else if (PART == 3) { // f64 division chain inside a step-like dependency
        double x = 1.0 + threadIdx.x, y = 3.0;
        OPAQUE(y);
        for (int i = 0; i < REPS; i++) x = fabs(y / fma(x, DBL_EPS, DBL_EPS)) * 1e-16;
        acc = x;
        nsteps = REPS;
    } else if (PART == 4) { // fastlog2 + exp2 (one fastpower)
        float x = 0.5f + threadIdx.x * 1e-3f;
        for (int i = 0; i < REPS; i++) x = sbr_exp2f_jl(0.14f * sbr_fastlog2f(x)) * 0.5f;
        acc = x;
        nsteps = REPS;
    } else if (PART == 5) { // select-based min/max chain (dmin/dmax) x3
        double dt = 1e-3 * (1 + threadIdx.x), a = 30.0, b = 1e-14, c = 29.0;
        OPAQUE(a); OPAQUE(b); OPAQUE(c);
        for (int i = 0; i < REPS; i++) { dt = dmin(a, dt); dt = dmax(dt, b); dt = dmin(dt, c) * 1.0000001; }
        acc = dt;
        nsteps = REPS;
    }
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) { cyc[0] = t1 - t0; rt[0] = r1 - r0; steps[0] = nsteps; }
}

int main()
{
    // parts 0-5: β = 1.00 .. 1.63; parts 6-7: the config-3 (Fig 5) β column grid,
    // β = 1 / range(1e-4, 1, 2048) (every 64 consecutive columns in one wave)
    static double hb[2048];
    for (int i = 0; i < 64; i++) hb[i] = 1.0 + i * 0.01;
    double *db, *dout;
    long long *dc, *dr, *ds;
    (void)hipMalloc(&db, sizeof(hb));
    (void)hipMalloc(&dout, 1 << 20);
    static double hg[2048];
    for (int i = 0; i < 2048; i++) hg[i] = 1.0 / (1e-4 + (1.0 - 1e-4) * i / 2047.0);
    double* dg;
    (void)hipMalloc(&dg, sizeof(hg));
    (void)hipMemcpy(dg, hg, sizeof(hg), hipMemcpyHostToDevice);
    (void)hipMalloc(&dc, 8); (void)hipMalloc(&dr, 8); (void)hipMalloc(&ds, 8);
    (void)hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
    double *dT, *dG;
    (void)hipMalloc(&dT, (size_t)2048 * 4096 * 8);
    (void)hipMalloc(&dG, (size_t)2048 * 4096 * 8);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_T), &dT, sizeof(dT));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_G), &dG, sizeof(dG));
    const char* names[] = {"full ode_scalar loop (per step)", "Tsit5 stages + EEst (per step)",
                           "PI controller pass", "f64 division chain", "fastpower (log2+exp2)", "3 select min/max",
                           "loop + knot stores, row/column", "loop + knot stores, knot-major"};
    auto run = [&](auto kern, int p, int blocks = 1, int threads = 64, int lds = 0) {
        long long c = 0, r = 0, s = 0;
        if (lds) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        for (int rep = 0; rep < 3; rep++) {
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds, 0, p >= 6 ? dg : db, dout, dc, dr, ds);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
            (void)hipMemcpy(&r, dr, 8, hipMemcpyDeviceToHost);
            (void)hipMemcpy(&s, ds, 8, hipMemcpyDeviceToHost);
        }
        printf("%-34s grid %4d x %3d lds %6d: %9.1f cycles  %8.1f ns   (clock %.2f GHz, %lld steps)\n", names[p],
               blocks, threads, lds, (double)c / s, (double)r * 10.0 / s, (double)c / (r * 10.0), s);
    };
    run(part<0>, 0); run(part<1>, 1); run(part<2>, 2); run(part<3>, 3); run(part<4>, 4); run(part<5>, 5);
    run(part<0>, 0, 32); run(part<0>, 0, 2048);
    run(part<6>, 6, 1); run(part<6>, 6, 32); run(part<7>, 7, 1); run(part<7>, 7, 32);
    // every 4th wave of the grid alone: the loop without stores (8), with stores (6), with
    // nontemporal stores (9), on the same 64 columns
    for (int w = 0; w < 32; w += 4) {
        double us[3];
        int k = 0;
        for (auto kern : {part<8>, part<6>, part<9>}) {
            hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, dg + w * 64, dout, dc, dr, ds);
            long long c = 0;
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
            us[k++] = c / 2400.0;
        }
        printf("  wave %2d: no stores %.1f us, stores %.1f us, nontemporal stores %.1f us\n", w, us[0], us[1], us[2]);
    }
    // every wave of the grid: cycles of the slowest one
    for (int w = 0; w < 32; w += 4) {
        hipLaunchKernelGGL(part<6>, dim3(1), dim3(64), 0, 0, dg + w * 64, dout, dc, dr, ds);
        long long c = 0, s = 0;
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&s, ds, 8, hipMemcpyDeviceToHost);
        printf("  wave %2d (beta %.4g..%.4g): %lld steps (lane 0), %.1f us total\n", w, hg[w * 64], hg[w * 64 + 63], s,
               c / 2400.0);
    }
    return 0;
}
