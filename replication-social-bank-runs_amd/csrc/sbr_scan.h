// sbr_scan.h — optimal_buffer's linear scan (src/baseline/solver.jl:218-261)
// answered from per-64-entry block summaries of the hazard path: any/all, the
// first/last index above u, and the first 0→1 / last 1→0 transitions — the same
// indices as the linear scan, with whole uniform blocks skipped.
//   S.hmax[b] = max over the block's non-NaN entries ("some entry > u" ⇔ hmax > u)
//   S.hmin[b] = min with NaN as −∞            ("every entry > u" ⇔ hmin > u)
// Shared by the baseline and heterogeneity equilibrium kernels.
#pragma once

namespace sbr {

// Inside a block the entries are read 8 at a time (independent loads issued together, then
// tested in order), so finding the index costs ≤ 8 dependent round trips to L2 instead of ≤ 64.
#ifndef SBR_SCAN_CHUNK
#define SBR_SCAN_CHUNK 8
#endif
constexpr int kScanChunk = SBR_SCAN_CHUNK;

// first i in [i, e) with (H[i] > u) == ABOVE, or -1
template <bool ABOVE, class P>
__device__ __forceinline__ int scan_fwd(P H, int i, int e, double u)
{
    for (; i < e; i += kScanChunk) {
        double h[kScanChunk];
#pragma unroll
        for (int k = 0; k < kScanChunk; k++) h[k] = i + k < e ? H[i + k] : 0.0;
#pragma unroll
        for (int k = 0; k < kScanChunk; k++)
            if (i + k < e && (h[k] > u) == ABOVE) return i + k;
    }
    return -1;
}

// last i in [s, e] with (H[i] > u) == ABOVE, or -1
template <bool ABOVE, class P>
__device__ __forceinline__ int scan_bwd(P H, int s, int e, double u)
{
    for (; e >= s; e -= kScanChunk) {
        double h[kScanChunk];
#pragma unroll
        for (int k = 0; k < kScanChunk; k++) h[k] = e - k >= s ? H[e - k] : 0.0;
#pragma unroll
        for (int k = 0; k < kScanChunk; k++)
            if (e - k >= s && (h[k] > u) == ABOVE) return e - k;
    }
    return -1;
}

// first i >= s with (H[i] > u) == ABOVE (or -1); whole blocks are skipped on their summary:
// some entry > u ⇔ hmax > u, every entry > u ⇔ hmin > u
template <bool ABOVE, class P, class SU>
__device__ __forceinline__ int first_where(P H, const SU& S, int ntau, int s, double u)
{
    int i = s;
    if (i & 63) {
        const int e = ((i | 63) + 1) < ntau ? ((i | 63) + 1) : ntau;
        const int r = scan_fwd<ABOVE>(H, i, e, u);
        if (r >= 0) return r;
        i = e;
    }
    for (; i < ntau; i += 64) {
        if (ABOVE ? (S.hmax[i >> 6] > u) : !(S.hmin[i >> 6] > u))
            return scan_fwd<ABOVE>(H, i, i + 64 < ntau ? i + 64 : ntau, u);
    }
    return -1;
}

// last i <= e with (H[i] > u) == ABOVE (or -1)
template <bool ABOVE, class P, class SU>
__device__ __forceinline__ int last_where(P H, const SU& S, int e, double u)
{
    if (e < 0) return -1;
    const int b0 = e >> 6;
    const int r = scan_bwd<ABOVE>(H, b0 << 6, e, u);
    if (r >= 0) return r;
    for (int b = b0 - 1; b >= 0; b--) {
        if (ABOVE ? (S.hmax[b] > u) : !(S.hmin[b] > u)) return scan_bwd<ABOVE>(H, b << 6, (b << 6) + 63, u);
    }
    return -1;
}

template <class P, class SU>
__device__ __forceinline__ int first_above(P H, const SU& S, int ntau, int s, double u)
{
    return first_where<true>(H, S, ntau, s, u);
}
template <class P, class SU>
__device__ __forceinline__ int first_not_above(P H, const SU& S, int ntau, int s, double u)
{
    return first_where<false>(H, S, ntau, s, u);
}
template <class P, class SU>
__device__ __forceinline__ int last_above(P H, const SU& S, int e, double u)
{
    return last_where<true>(H, S, e, u);
}
template <class P, class SU>
__device__ __forceinline__ int last_not_above(P H, const SU& S, int e, double u)
{
    return last_where<false>(H, S, e, u);
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
