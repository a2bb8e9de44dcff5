// Dependent-chain latency of FP64 operations on gfx950 (one wave, s_memtime cycles).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../include/sbr_detmath.h"

#define N 4096
__global__ void k_fma(double* out, long long* cyc, double a, double b)
{
    double x = out[threadIdx.x];
    long long c0 = clock64();
#pragma unroll 16
    for (int i = 0; i < N; i++) x = fma(x, a, b);
    long long c1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = c1 - c0;
}
__global__ void k_fma4(double* out, long long* cyc, double a, double b)
{   // 4 independent chains interleaved
    double x0 = out[threadIdx.x], x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    long long c0 = clock64();
#pragma unroll 16
    for (int i = 0; i < N; i++) { x0 = fma(x0, a, b); x1 = fma(x1, a, b); x2 = fma(x2, a, b); x3 = fma(x3, a, b); }
    long long c1 = clock64();
    out[threadIdx.x] = x0 + x1 + x2 + x3;
    if (threadIdx.x == 0) cyc[1] = c1 - c0;
}
__global__ void k_div(double* out, long long* cyc, double a, double b)
{
    double x = out[threadIdx.x] + 1.5;
    long long c0 = clock64();
#pragma unroll 4
    for (int i = 0; i < N / 16; i++) x = a / (x + b);
    long long c1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[2] = c1 - c0;
}
__global__ void k_exp(double* out, long long* cyc, double a, double b)
{
    double x = out[threadIdx.x] * 1e-3;
    long long c0 = clock64();
    for (int i = 0; i < N / 16; i++) x = sbr_exp(x * a) * b;
    long long c1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[3] = c1 - c0;
}
__global__ void k_log(double* out, long long* cyc, double a, double b)
{
    double x = out[threadIdx.x] + 2.0;
    long long c0 = clock64();
    for (int i = 0; i < N / 16; i++) x = sbr_log(x) * a + b;
    long long c1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[4] = c1 - c0;
}
__global__ void k_mul(double* out, long long* cyc, double a, double b)
{
    double x = out[threadIdx.x];
    long long c0 = clock64();
#pragma unroll 16
    for (int i = 0; i < N; i++) x = x * a;
    long long c1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[5] = c1 - c0;
}
__global__ void k_load(double* out, long long* cyc, const int* idx)
{   // dependent pointer chase through an L2-resident table
    int j = threadIdx.x;
    long long c0 = clock64();
    for (int i = 0; i < 256; i++) j = idx[j];
    long long c1 = clock64();
    out[threadIdx.x] = j;
    if (threadIdx.x == 0) cyc[6] = c1 - c0;
}

int main()
{
    double* d; long long* c; int* idx;
    hipMalloc(&d, 64 * 8); hipMalloc(&c, 16 * 8); hipMalloc(&idx, 1 << 20);
    hipMemset(d, 0, 64 * 8);
    int h[1 << 18];
    for (int i = 0; i < (1 << 18); i++) h[i] = (i * 7919 + 13) & ((1 << 18) - 1);
    hipMemcpy(idx, h, sizeof(h), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_fma, 1, 64, 0, 0, d, c, 0.999, 1e-3);
        hipLaunchKernelGGL(k_fma4, 1, 64, 0, 0, d, c, 0.999, 1e-3);
        hipLaunchKernelGGL(k_div, 1, 64, 0, 0, d, c, 1.3, 0.7);
        hipLaunchKernelGGL(k_exp, 1, 64, 0, 0, d, c, 0.3, 1.1);
        hipLaunchKernelGGL(k_log, 1, 64, 0, 0, d, c, 0.9, 1.7);
        hipLaunchKernelGGL(k_mul, 1, 64, 0, 0, d, c, 0.999, 0);
        hipLaunchKernelGGL(k_load, 1, 64, 0, 0, d, c, idx);
        hipDeviceSynchronize();
    }
    long long hc[16];
    hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
    printf("{\"fma_dep_cyc\": %.2f, \"fma_4chains_cyc_per_op\": %.2f, \"div_dep_cyc\": %.1f, \"sbr_exp_cyc\": %.1f, "
           "\"sbr_log_cyc\": %.1f, \"mul_dep_cyc\": %.2f, \"load_chain_cyc\": %.1f}\n",
           hc[0] / (double)N, hc[1] / (4.0 * N), hc[2] / (double)(N / 16), hc[3] / (double)(N / 16),
           hc[4] / (double)(N / 16), hc[5] / (double)N, hc[6] / 256.0);
    return 0;
}
