// Phase cycles of hazard_kernel (csrc/sbr_baseline.hip built with SBR_HZ_PROF) after the
// learning kernel on 512 config-3 columns; prints the per-phase mean / max over blocks.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -DSBR_HZ_PROF \
//         -o tools/ubench_hazard tools/ubench_hazard.hip
#include "../replication-social-bank-runs_amd/csrc/sbr_baseline.hip"
#include <cstdio>
#include <vector>

int main()
{
    using namespace sbr;
    const int nb = 512, cap = 65536;
    std::vector<double> hb(nb), he(nb, 15.0), ht(nb, 30.0);
    for (int i = 0; i < nb; i++) hb[i] = 1.0 / (1e-4 + (1.0 - 1e-4) * (i + 512) / 2047.0);
    double *db, *de, *dt;
    (void)hipMalloc(&db, nb * 8); (void)hipMalloc(&de, nb * 8); (void)hipMalloc(&dt, nb * 8);
    (void)hipMemcpy(db, hb.data(), nb * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(de, he.data(), nb * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dt, ht.data(), nb * 8, hipMemcpyHostToDevice);
    LearnBufs L{};
    (void)hipMalloc(&L.t, (size_t)nb * cap * 8); (void)hipMalloc(&L.G, (size_t)nb * cap * 8);
    (void)hipMalloc(&L.hr, (size_t)nb * cap * 8);
    (void)hipMalloc(&L.n_knots, nb * 4); (void)hipMalloc(&L.n_tau, nb * 4); (void)hipMalloc(&L.n_le, nb * 4);
    (void)hipMalloc(&L.status, nb * 4); (void)hipMalloc(&L.n_accept, nb * 4); (void)hipMalloc(&L.n_reject, nb * 4);
    L.cap = cap;
    LearnArgs a{1e-4, DBL_EPS, DBL_EPS, 0.5, 0.01, 1000000, nb, 1, 0};
    for (int rep = 0; rep < 2; rep++) {
        std::vector<long long> z(8192 * 6, 0);
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_hzprof), z.data(), z.size() * 8);
        hipEvent_t e0, e1, e2;
        hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&e2);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(learn_logistic_kernel, dim3(nb / 64), dim3(64), 0, 0, db, de, dt, a, L);
        hipEventRecord(e1, 0);
        hipLaunchKernelGGL(hazard_kernel, dim3(nb), dim3(HZ_BLOCK), 0, 0, db, de, a, L);
        hipEventRecord(e2, 0);
        (void)hipDeviceSynchronize();
        float ml = 0, mh = 0;
        hipEventElapsedTime(&ml, e0, e1); hipEventElapsedTime(&mh, e1, e2);
        (void)hipMemcpyFromSymbol(z.data(), HIP_SYMBOL(g_hzprof), z.size() * 8);
        std::vector<int> ntau(nb);
        (void)hipMemcpy(ntau.data(), L.n_tau, nb * 4, hipMemcpyDeviceToHost);
        printf("learn %.1f us, hazard %.1f us, ntau[0] %d\n", ml * 1e3, mh * 1e3, ntau[0]);
        const char* names[] = {"prologue", "e*g pass", "terms", "serial scan", "park I", "final HR"};
        for (int ph = 0; ph < 6; ph++) {
            double sum = 0, mx = 0;
            for (int b = 0; b < nb; b++) { sum += z[b * 6 + ph]; mx = std::max(mx, (double)z[b * 6 + ph]); }
            printf("  %-12s mean %9.0f cycles  max %9.0f cycles\n", names[ph], sum / nb, mx);
        }
    }
    return 0;
}
