// sbr_scan.h — optimal_buffer's linear scan (src/baseline/solver.jl:218-261)
// answered from per-64-entry block summaries of the hazard path: any/all, the
// first/last index above u, and the first 0→1 / last 1→0 transitions — the same
// indices as the linear scan, with whole uniform blocks skipped.
//   S.hmax[b] = max over the block's non-NaN entries ("some entry > u" ⇔ hmax > u)
//   S.hmin[b] = min with NaN as −∞            ("every entry > u" ⇔ hmin > u)
// Shared by the baseline and heterogeneity equilibrium kernels.
#pragma once

namespace sbr {

// first i >= s with H[i] > u (or -1); whole blocks are skipped on their summary
template <class P, class SU>
__device__ __forceinline__ int first_above(P H, const SU& S, int ntau, int s, double u)
{
    int i = s;
    for (; i < ntau && (i & 63); i++)
        if (H[i] > u) return i;
    for (; i < ntau; i += 64) {
        if (S.hmax[i >> 6] > u) {
            const int e = i + 64 < ntau ? i + 64 : ntau;
            for (; i < e; i++)
                if (H[i] > u) return i;
            return -1;
        }
    }
    return -1;
}

// first i >= s with !(H[i] > u) (or -1)
template <class P, class SU>
__device__ __forceinline__ int first_not_above(P H, const SU& S, int ntau, int s, double u)
{
    int i = s;
    for (; i < ntau && (i & 63); i++)
        if (!(H[i] > u)) return i;
    for (; i < ntau; i += 64) {
        if (!(S.hmin[i >> 6] > u)) {
            const int e = i + 64 < ntau ? i + 64 : ntau;
            for (; i < e; i++)
                if (!(H[i] > u)) return i;
            return -1;
        }
    }
    return -1;
}

// last i <= e with H[i] > u (or -1)
template <class P, class SU>
__device__ __forceinline__ int last_above(P H, const SU& S, int e, double u)
{
    if (e < 0) return -1;
    const int b0 = e >> 6;
    for (int i = e; i >= (b0 << 6); i--)
        if (H[i] > u) return i;
    for (int b = b0 - 1; b >= 0; b--) {
        if (S.hmax[b] > u) {
            for (int i = (b << 6) + 63; i >= (b << 6); i--)
                if (H[i] > u) return i;
            return -1;
        }
    }
    return -1;
}

// last i <= e with !(H[i] > u) (or -1)
template <class P, class SU>
__device__ __forceinline__ int last_not_above(P H, const SU& S, int e, double u)
{
    if (e < 0) return -1;
    const int b0 = e >> 6;
    for (int i = e; i >= (b0 << 6); i--)
        if (!(H[i] > u)) return i;
    for (int b = b0 - 1; b >= 0; b--) {
        if (!(S.hmin[b] > u)) {
            for (int i = (b << 6) + 63; i >= (b << 6); i--)
                if (!(H[i] > u)) return i;
            return -1;
        }
    }
    return -1;
}

// The linear scan of optimal_buffer (solver.jl:218-261) answered with block
// summaries: any/all, first/last index above u, first 0→1 and last 1→0 pair.
template <class P, class SU>
__device__ __forceinline__ void buffer_scan_blocked(P H, const SU& S, int ntau, double u, bool& any, bool& all,
                                                    int& fa, int& la, int& cin, int& cout)
{
    fa = first_above(H, S, ntau, 0, u);
    any = fa >= 0;
    const int fb = first_not_above(H, S, ntau, 0, u);
    all = fb < 0;
    la = any ? last_above(H, S, ntau - 1, u) : -1;
    cin = -1;
    cout = -1;
    if (!any || all) return;
    if (fa > 0) {
        cin = fa - 1; // H[0..fa) not above, H[fa] above
    } else {
        const int k = first_above(H, S, ntau, fb, u); // first above after the first drop
        cin = k >= 0 ? k - 1 : -1;
    }
    if (la < ntau - 1) {
        cout = la; // everything after la is not above
    } else {
        const int lb = last_not_above(H, S, ntau - 1, u);
        cout = last_above(H, S, lb, u);
    }
}


}  // namespace sbr
