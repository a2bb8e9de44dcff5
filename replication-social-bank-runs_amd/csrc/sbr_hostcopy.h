// sbr_hostcopy.h — multi-threaded host copy of result blocks from a pinned landing buffer into
// the caller's (pageable) arrays: shared by the single-device host-pointer sweeps
// (sbr_capi.hip) and the n-device direct transport (sbr_multi.hip).
#pragma once

#include <string.h>

#include <algorithm>
#include <array>
#include <thread>
#include <vector>

namespace sbr_host {

// copy (dst_k, src_k, bytes_k) pieces with up to max_threads host threads in ≈1 MiB slices: the
// caller's result arrays are often fresh pages (first-touch faults), which one thread would take
// serially
inline void parallel_copy(const std::vector<std::array<size_t, 3>>& pieces, size_t max_threads = 8)
{
    constexpr size_t kSlice = 1 << 20;
    std::vector<std::array<size_t, 3>> sl;
    size_t total = 0;
    for (const auto& p : pieces)
        for (size_t o = 0; o < p[2]; o += kSlice) {
            const size_t b = std::min(kSlice, p[2] - o);
            sl.push_back({p[0] + o, p[1] + o, b});
            total += b;
        }
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nt = std::min<size_t>({max_threads, (size_t)hw, (total + (4u << 20) - 1) / (4u << 20)});
    auto work = [&](size_t k0) {
        for (size_t k = k0; k < sl.size(); k += nt) memcpy((void*)sl[k][0], (const void*)sl[k][1], sl[k][2]);
    };
    if (nt <= 1) { work(0); return; }
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; t++) th.emplace_back(work, t);
    work(0);
    for (auto& t : th) t.join();
}

}  // namespace sbr_host
