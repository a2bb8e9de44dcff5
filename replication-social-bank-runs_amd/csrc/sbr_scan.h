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
constexpr int kScanChunk = 8;

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

// Index queries over a monotone block table by binary search with a wave-uniform trip count
// (the table length is the column's): no per-lane loop exits, a few LDS reads per query.
// first b in [0, nb) with key[b] > u for a nondecreasing key (nb when none)
template <class P>
__device__ __forceinline__ int bs_first_gt_inc(P key, int nb, double u)
{
    int lo = -1; // key[lo] <= u (virtual −∞ at −1)
    for (int step = 1 << (31 - __builtin_clz(nb | 1)); step > 0; step >>= 1) {
        const int m = lo + step;
        if (m < nb && !(key[m] > u)) lo = m;
    }
    return lo + 1;
}
// first b with !(key[b] > u) for a nonincreasing key (nb when none)
template <class P>
__device__ __forceinline__ int bs_first_le_dec(P key, int nb, double u)
{
    int lo = -1;
    for (int step = 1 << (31 - __builtin_clz(nb | 1)); step > 0; step >>= 1) {
        const int m = lo + step;
        if (m < nb && key[m] > u) lo = m;
    }
    return lo + 1;
}
// last b with key[b] > u for a nonincreasing key (−1 when none)
template <class P>
__device__ __forceinline__ int bs_last_gt_dec(P key, int nb, double u)
{
    return bs_first_le_dec(key, nb, u) - 1;
}
// last b with !(key[b] > u) for a nondecreasing key (−1 when none)
template <class P>
__device__ __forceinline__ int bs_last_le_inc(P key, int nb, double u)
{
    return bs_first_gt_inc(key, nb, u) - 1;
}

// buffer_scan_blocked with the four scans from index 0 / from the end answered by the prefix /
// suffix tables (hpm = prefix max of hmax, hpn = prefix min of hmin, hsm = suffix max of hmax,
// hsn = suffix min of hmin: "some entry of blocks <= b above u" ⇔ hpm[b] > u, and so on), then
// one in-block scan each; the two scans from an interior start keep the block loop.  The same
// indices as buffer_scan_blocked.
template <class P, class SU, class Q>
__device__ __forceinline__ void buffer_scan_bs(P H, const SU& S, Q hpm, Q hpn, Q hsm, Q hsn, int nb, int ntau,
                                               double u, bool& any, bool& all, int& fa, int& la, int& cin, int& cout)
{
    auto blk_end = [&](int b) { return (b << 6) + 64 < ntau ? (b << 6) + 64 : ntau; };
    const int ba = bs_first_gt_inc(hpm, nb, u);
    fa = ba < nb ? scan_fwd<true>(H, ba << 6, blk_end(ba), u) : -1;
    any = fa >= 0;
    const int bb = bs_first_le_dec(hpn, nb, u);
    const int fb = bb < nb ? scan_fwd<false>(H, bb << 6, blk_end(bb), u) : -1;
    all = fb < 0;
    int lab = any ? bs_last_gt_dec(hsm, nb, u) : -1;
    la = lab >= 0 ? scan_bwd<true>(H, lab << 6, blk_end(lab) - 1, u) : -1;
    cin = -1;
    cout = -1;
    if (!any || all) return;
    if (fa > 0) {
        cin = fa - 1;
    } else {
        const int k = first_above(H, S, ntau, fb, u);
        cin = k >= 0 ? k - 1 : -1;
    }
    if (la < ntau - 1) {
        cout = la;
    } else {
        const int lbb = bs_last_le_inc(hsn, nb, u);
        const int lb = lbb >= 0 ? scan_bwd<false>(H, lbb << 6, blk_end(lbb) - 1, u) : -1;
        cout = last_above(H, S, lb, u);
    }
}

}  // namespace sbr
