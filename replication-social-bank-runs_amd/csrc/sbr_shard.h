// sbr_shard.h — the data movement of an n-device sweep, host-only and
// transport-agnostic, so that it runs the same on the GPUs (sbr_multi.hip: RCCL over xGMI,
// hipMemcpy2DAsync) and in a host loopback (sbr_shard_host_run: memcpy), which the CPU
// tests drive at N = 2, 3, 8 against single-device results.
//
//  * deal:    grid column i goes to rank i mod N; rank r holds columns r, r+N, r+2N, …
//             (block row c of rank r is grid column r + c·N);
//  * pack:    a rank's results are one block: field after field, each field u-fastest per
//             column ([c][j][per_pt] elements of esz bytes);
//  * gather:  every rank's block lands in rank 0's gather buffer at block offset off[r]
//             (rank 0 copies its own; ranks ≥ 1 send, rank 0 receives — posted together);
//  * scatter: field f of rank r's block is a (cols[r] × row) matrix copied with pitch N·row
//             into the caller's u-fastest array at row offset r·row — either by each rank
//             from its own block (direct: host destinations, every GPU's own PCIe link, no
//             collective) or by rank 0 from the gathered blocks.
#pragma once

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <vector>

namespace sbr_shard {

// one result array of the caller: n_col·n_u·per_pt elements of esz bytes, u-fastest per
// column (host == nullptr: computed but not returned)
struct Field {
    void* host;
    size_t esz;
    size_t per_pt;
};

struct Plan {
    int N = 1;
    int64_t n_col = 0, n_u = 0;
    std::vector<int64_t> cols; // columns of rank r
    std::vector<int64_t> off;  // first block row of rank r in the gather buffer (off[N] = n_col)
    size_t per_col = 0;        // packed bytes per column over all fields
    size_t block_bytes(int r) const { return (size_t)cols[r] * per_col; }
    size_t gather_bytes() const { return (size_t)n_col * per_col; }
    int64_t max_cols() const { return N > 0 && n_col > 0 ? (n_col + N - 1) / N : 0; }
};

inline Plan make_plan(int N, int64_t n_col, int64_t n_u, const std::vector<Field>& fields)
{
    Plan p;
    p.N = N;
    p.n_col = n_col;
    p.n_u = n_u;
    p.cols.assign((size_t)N, 0);
    p.off.assign((size_t)N + 1, 0);
    for (int r = 0; r < N; r++) p.cols[r] = n_col > r ? (n_col - r + N - 1) / N : 0;
    for (int r = 0; r < N; r++) p.off[r + 1] = p.off[r] + p.cols[r];
    for (const Field& f : fields) p.per_col += (size_t)n_u * f.per_pt * f.esz;
    return p;
}

// grid column of block row c of rank r
inline int64_t global_col(int r, int64_t c, int N) { return r + c * (int64_t)N; }

// the rank's columns of a per-column input array with w values per column, packed
inline void deal_cols(const double* src, int64_t w, int r, int N, int64_t nc, double* dst)
{
    for (int64_t c = 0; c < nc; c++) memcpy(dst + c * w, src + global_col(r, c, N) * w, (size_t)w * 8);
}

// byte offsets of each field inside rank r's block
inline std::vector<size_t> field_offsets(const Plan& p, int r, const std::vector<Field>& fields)
{
    std::vector<size_t> o;
    size_t at = 0;
    for (const Field& f : fields) {
        o.push_back(at);
        at += (size_t)p.cols[r] * p.n_u * f.per_pt * f.esz;
    }
    return o;
}

// Transport of the gather: calls between begin() and end() are posted together (RCCL:
// one group over every rank's communicator), end() launches them, wait() completes them.
struct Transport {
    virtual ~Transport() {}
    virtual int begin() = 0;
    virtual int local_copy(void* dst, const void* src, size_t bytes) = 0; // rank 0's own block
    virtual int recv(int from, void* dst, size_t bytes) = 0;              // on rank 0
    virtual int send(int from, const void* src, size_t bytes) = 0;        // on rank `from`
    virtual int end() = 0;
    virtual int wait() = 0;
};

// gather every rank's block (blocks[r], device or host memory of rank r) into `gathered`
// (rank 0's memory).  Every buffer must exist before this is called: nothing fallible but
// the transport itself runs once a send or receive has been posted.
inline int gather(const Plan& p, Transport& t, const std::vector<const void*>& blocks, void* gathered)
{
    // rank 0's own block first: it can fail without leaving a peer waiting
    int rc = p.cols[0] > 0 ? t.local_copy(gathered, blocks[0], p.block_bytes(0)) : 0;
    if (rc == 0) rc = t.begin();
    if (rc) return rc;
    for (int r = 1; r < p.N && rc == 0; r++) {
        if (p.cols[r] == 0) continue;
        char* dst = (char*)gathered + (size_t)p.off[r] * p.per_col;
        rc = t.recv(r, dst, p.block_bytes(r));
        if (rc == 0) rc = t.send(r, blocks[r], p.block_bytes(r));
    }
    const int re = t.end();
    if (rc == 0) rc = re;
    const int rw = t.wait();
    return rc ? rc : rw;
}

// rank r's block into the callers' arrays (its columns r, r+N, … of every field):
//   copy2d(dst, dpitch, src, spitch, width, height) -> int (0 = ok)
template <class Copy2D>
int scatter_rank(const Plan& p, int r, const std::vector<Field>& fields, const void* block, Copy2D&& copy2d)
{
    if (p.cols[r] == 0) return 0;
    const char* blk = (const char*)block;
    const std::vector<size_t> fo = field_offsets(p, r, fields);
    for (size_t i = 0; i < fields.size(); i++) {
        const Field& f = fields[i];
        if (!f.host) continue;
        const size_t row = (size_t)p.n_u * f.per_pt * f.esz;
        const int rc = copy2d((char*)f.host + (size_t)r * row, (size_t)p.N * row, blk + fo[i], row, row,
                              (size_t)p.cols[r]);
        if (rc) return rc;
    }
    return 0;
}

// every rank's block from the gathered buffer (rank 0's memory) into the callers' arrays
template <class Copy2D>
int scatter(const Plan& p, const std::vector<Field>& fields, const void* gathered, Copy2D&& copy2d)
{
    for (int r = 0; r < p.N; r++) {
        const int rc = scatter_rank(p, r, fields, (const char*)gathered + (size_t)p.off[r] * p.per_col, copy2d);
        if (rc) return rc;
    }
    return 0;
}

// Host loopback transport: sends and receives are matched by rank at end() and moved with memcpy.
struct LoopbackTransport : Transport {
    struct Op {
        int rank;
        void* dst;
        const void* src;
        size_t bytes;
    };
    std::vector<Op> recvs, sends;
    int begin() override
    {
        recvs.clear();
        sends.clear();
        return 0;
    }
    int local_copy(void* dst, const void* src, size_t bytes) override
    {
        memcpy(dst, src, bytes);
        return 0;
    }
    int recv(int from, void* dst, size_t bytes) override
    {
        recvs.push_back({from, dst, nullptr, bytes});
        return 0;
    }
    int send(int from, const void* src, size_t bytes) override
    {
        sends.push_back({from, nullptr, src, bytes});
        return 0;
    }
    int end() override
    {
        if (recvs.size() != sends.size()) return -1;
        for (const Op& r : recvs) {
            bool hit = false;
            for (const Op& s : sends)
                if (s.rank == r.rank) {
                    if (s.bytes != r.bytes) return -1;
                    memcpy(r.dst, s.src, r.bytes);
                    hit = true;
                    break;
                }
            if (!hit) return -1;
        }
        return 0;
    }
    int wait() override { return 0; }
};

inline int host_copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height)
{
    for (size_t h = 0; h < height; h++) memcpy((char*)dst + h * dpitch, (const char*)src + h * spitch, width);
    return 0;
}

}  // namespace sbr_shard
