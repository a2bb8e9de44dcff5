// Checks DPP row_newbcast:j on gfx950: every lane of each 16-lane row receives lane j of its row
// (the broadcast learn_hetero_wave4_kernel uses for its row-per-column couplings), with all
// lanes active and with whole rows masked off.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int J>
__device__ __forceinline__ double rowbc(double v)
{
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x150 + J, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x150 + J, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__global__ void k(double* out)
{
    const int l = threadIdx.x;
    const double v = 1000.0 * (l >> 4) + (l & 15) + 0.5;
    out[l] = rowbc<3>(v);
    double w = -1.0;
    if ((l >> 4) & 1) w = rowbc<5>(v); // rows 1 and 3 only
    out[64 + l] = w;
}
int main()
{
    double* d;
    double h[128];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    for (int l = 0; l < 64; l++) {
        const double e0 = 1000.0 * (l >> 4) + 3 + 0.5;
        const double e1 = ((l >> 4) & 1) ? 1000.0 * (l >> 4) + 5 + 0.5 : -1.0;
        if (h[l] != e0 || h[64 + l] != e1) { bad++; printf("lane %d: %g %g (want %g %g)\n", l, h[l], h[64 + l], e0, e1); }
    }
    printf("row_newbcast %s\n", bad ? "MISMATCH" : "ok");
    return bad ? 1 : 0;
}
