// Latency / issue micro-benchmark for one wave64 on one SIMD of gfx950 (the learning
// kernels run one lone wave per SIMD, so their step time is set by dependent-chain
// latency and single-wave issue cost, not throughput).  Each kernel runs N dependent
// (or K-way independent) operations between two s_memtime reads; prints cycles per op.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_lat tools/ubench_lat.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 4096;

#define OPAQUE(x) asm volatile("" : "+v"(x))

template <int OP>
__global__ void lat(const double* in, double* out, long long* cyc)
{
    double x = in[threadIdx.x], a = in[64 + threadIdx.x], b = in[128 + threadIdx.x];
    double y0 = x * 1.1, y1 = x * 1.2, y2 = x * 1.3;
    float xf = (float)x, af = (float)a, bf = (float)b;
    OPAQUE(x); OPAQUE(a); OPAQUE(b); OPAQUE(y0); OPAQUE(y1); OPAQUE(y2);
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
    for (int i = 0; i < N; i++) {
        if (OP == 0) x = fma(x, a, b);                       // dependent f64 fma
        if (OP == 1) { x = fma(x, a, b); y0 = fma(y0, a, b); y1 = fma(y1, a, b); y2 = fma(y2, a, b); } // 4 chains
        if (OP == 2) xf = __builtin_fmaf(xf, af, bf);         // dependent f32 fma
        if (OP == 3) x = b / x;                               // dependent IEEE f64 division
        if (OP == 4) x = (x < a) ? b : x * a;                 // cmp + mul + 2 cndmask chain
        if (OP == 5) x = __builtin_fmin(x, a) + b;            // v_min_f64 + add
        if (OP == 6) x = __builtin_amdgcn_rcp(x);             // v_rcp_f64
        if (OP == 7) x = (double)(float)x * a;                // cvt pair + mul
        if (OP == 8) x = x * a;                               // dependent f64 mul
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x + y0 + y1 + y2 + (double)xf;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main()
{
    double h[192];
    for (int i = 0; i < 64; i++) { h[i] = 1.0 + i * 1e-3; h[64 + i] = 0.999999; h[128 + i] = 1e-7; }
    double *din, *dout;
    long long* dc;
    hipMalloc(&din, sizeof(h));
    hipMalloc(&dout, 64 * sizeof(double));
    hipMalloc(&dc, sizeof(long long));
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    const char* names[] = {"fma_f64 dependent", "fma_f64 4 chains (per fma)", "fma_f32 dependent",
                           "div_f64 dependent (IEEE seq)", "cmp+mul+cndmask chain", "min_f64+add chain",
                           "rcp_f64 dependent", "cvt f64->f32->f64 + mul", "mul_f64 dependent"};
    auto run = [&](auto kern, int op, double per) {
        long long c = 0;
        for (int rep = 0; rep < 3; rep++) {
            hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, din, dout, dc);
            hipDeviceSynchronize();
            hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
        }
        printf("%-32s %8.2f cycles/op\n", names[op], (double)c / (N * per));
    };
    run(lat<0>, 0, 1); run(lat<1>, 1, 4); run(lat<2>, 2, 1); run(lat<3>, 3, 1); run(lat<4>, 4, 1);
    run(lat<5>, 5, 1); run(lat<6>, 6, 1); run(lat<7>, 7, 1); run(lat<8>, 8, 1);
    return 0;
}
