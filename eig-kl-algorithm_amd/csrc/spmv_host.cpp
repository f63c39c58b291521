// Host preparation of the Lanczos SpMV operand (the rows ek_spmv_setup
// uploads): CSR-adaptive row blocks, the dictionary coding of the values and
// the per-block segments of the coded words (layouts: ek_internal.hpp
// SpmvMat, kernels_spmv.hip).  On the file -> cut path of every solve, so
// the coding and the segments are built on all host threads.
#include <algorithm>
#include <cstring>

#include "ek_internal.hpp"

namespace ek {
namespace dev {

std::vector<int32_t> spmv_row_blocks(const int32_t* rowptr, int64_t nrows, int block_nnz) {
    std::vector<int32_t> starts{0};
    int64_t rows_in = 0, nnz_in = 0;
    for (int64_t r = 0; r < nrows; ++r) {
        const int64_t len = rowptr[r + 1] - rowptr[r];
        if (rows_in > 0 && (nnz_in + len > block_nnz || rows_in == SPMV_THREADS)) {
            starts.push_back(int32_t(r));
            rows_in = nnz_in = 0;
        }
        ++rows_in;
        nnz_in += len;
        if (len > block_nnz) {  // long row: a workgroup of its own (vector mode)
            starts.push_back(int32_t(r + 1));
            rows_in = nnz_in = 0;
        }
    }
    if (starts.back() != int32_t(nrows)) starts.push_back(int32_t(nrows));
    // one {row0, nrows, nnz0, cnt} record per block
    std::vector<int32_t> desc;
    desc.reserve((starts.size() - 1) * 4);
    for (size_t b = 0; b + 1 < starts.size(); ++b) {
        const int32_t r0 = starts[b], r1 = starts[b + 1];
        desc.push_back(r0);
        desc.push_back(r1 - r0);
        desc.push_back(rowptr[r0]);
        desc.push_back(rowptr[r1] - rowptr[r0]);
    }
    return desc;
}

namespace {

// Open-addressing set of fp64 bit patterns: slot -> index into `first`
// (first-seen order) with a count per value.
struct ValueSet {
    std::vector<uint64_t> keys;
    std::vector<int32_t> slot;
    std::vector<uint64_t> first;
    std::vector<int64_t> cnt;
    size_t cap = 0;
    static size_t hash(uint64_t k) { return size_t(((k ^ (k >> 29)) * 0x9E3779B97F4A7C15ull) >> 20); }
    explicit ValueSet(size_t c = 1024) : keys(c), slot(c, -1), cap(c) {}
    // index of k, inserting it (count += add) when new
    int32_t insert(uint64_t k, int64_t add) {
        size_t h = hash(k) & (cap - 1);
        while (slot[h] >= 0 && keys[h] != k) h = (h + 1) & (cap - 1);
        if (slot[h] < 0) {
            slot[h] = int32_t(first.size());
            keys[h] = k;
            first.push_back(k);
            cnt.push_back(0);
            if (first.size() * 2 > cap) {
                grow();
                h = find_slot(k);
            }
        }
        cnt[size_t(slot[h])] += add;
        return slot[h];
    }
    size_t find_slot(uint64_t k) const {
        size_t h = hash(k) & (cap - 1);
        while (!(slot[h] >= 0 && keys[h] == k)) h = (h + 1) & (cap - 1);
        return h;
    }
    int32_t find(uint64_t k) const { return slot[find_slot(k)]; }
    void grow() {
        cap *= 2;
        keys.assign(cap, 0);
        slot.assign(cap, -1);
        for (size_t c = 0; c < first.size(); ++c) {
            size_t g = hash(first[c]) & (cap - 1);
            while (slot[g] >= 0) g = (g + 1) & (cap - 1);
            slot[g] = int32_t(c);
            keys[g] = first[c];
        }
    }
};

}  // namespace

// Dictionary coding of the Laplacian values (see SpmvMat in ek_internal.hpp).
// Codes are ranked by descending frequency, ties by first appearance, so the
// hot off-diagonal values (-2/|e| for the few net sizes) share one cache line.
// Each thread collects the distinct values of a contiguous range in
// first-seen order; merging the ranges in order reproduces the sequential
// first-seen order exactly, so the codes do not depend on the thread count.
bool spmv_pack(int64_t n, int64_t nnz, const int32_t* col, const double* val, std::vector<uint32_t>& pk,
               std::vector<double>& dict, int& colbits) {
    colbits = 1;
    while (colbits < 31 && (int64_t(1) << colbits) < n) ++colbits;
    if (colbits > 28) return false;
    const size_t max_codes = size_t(1) << (32 - colbits);
    const int T = int(std::min<int64_t>(host_threads(), std::max<int64_t>(1, nnz / 65536)));
    std::vector<ValueSet> local(static_cast<size_t>(T));
    std::vector<char> over(static_cast<size_t>(T), 0);
    run_threads(T, [&](int t) {
        const int64_t lo = nnz * t / T, hi = nnz * (t + 1) / T;
        ValueSet& vs = local[size_t(t)];
        for (int64_t p = lo; p < hi; ++p) {
            uint64_t k;
            std::memcpy(&k, &val[p], 8);
            vs.insert(k, 1);
            if (vs.first.size() > max_codes) {
                over[size_t(t)] = 1;
                return;
            }
        }
    });
    for (char o : over)
        if (o) return false;
    ValueSet all;
    for (const ValueSet& vs : local) {
        for (size_t c = 0; c < vs.first.size(); ++c) all.insert(vs.first[c], vs.cnt[c]);
        if (all.first.size() > max_codes) return false;
    }
    std::vector<uint32_t> order(all.first.size());
    for (size_t c = 0; c < order.size(); ++c) order[c] = uint32_t(c);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return all.cnt[a] > all.cnt[b]; });
    std::vector<uint32_t> rank(order.size());
    dict.resize(order.size());
    for (size_t r = 0; r < order.size(); ++r) {
        rank[order[r]] = uint32_t(r);
        std::memcpy(&dict[r], &all.first[order[r]], 8);
    }
    pk.resize(size_t(std::max<int64_t>(nnz, 0)));
    run_threads(T, [&](int t) {
        const int64_t lo = nnz * t / T, hi = nnz * (t + 1) / T;
        for (int64_t p = lo; p < hi; ++p) {
            uint64_t k;
            std::memcpy(&k, &val[p], 8);
            pk[size_t(p)] = (rank[size_t(all.find(k))] << colbits) | uint32_t(col[p]);
        }
    });
    return true;
}

// Per-block segments of the coded entries: block b's entries at
// [b*seg_nnz, +cnt), padded with word 0; a long row (vector mode) goes
// to an overflow area after the segments and its descriptor's nnz0 points
// there.  rel[b*SPMV_REL_STRIDE + t] = start of the block's row t inside the
// segment for t <= nrows, cnt beyond.
void spmv_segment(std::vector<int32_t>& desc, const int32_t* rowptr, const std::vector<uint32_t>& pk, int seg_nnz,
                  std::vector<uint32_t>& seg, std::vector<uint16_t>& rel) {
    const size_t SEG = size_t(seg_nnz);
    const size_t nb = desc.size() / 4;
    std::vector<size_t> over_at(nb + 1, 0);  // overflow offsets of the long rows, in block order
    for (size_t b = 0; b < nb; ++b) over_at[b + 1] = over_at[b] + (size_t(desc[4 * b + 3]) > SEG ? size_t(desc[4 * b + 3]) : 0);
    seg.resize(nb * SEG + over_at[nb]);
    rel.resize(nb * SPMV_REL_STRIDE);
    parallel_for(int64_t(nb), [&](int64_t lo, int64_t hi) {
        for (int64_t bb = lo; bb < hi; ++bb) {
            const size_t b = size_t(bb);
            const int32_t r0 = desc[4 * b], nr = desc[4 * b + 1], p0 = desc[4 * b + 2], cnt = desc[4 * b + 3];
            uint32_t* s = seg.data() + b * SEG;
            uint16_t* rl = rel.data() + b * SPMV_REL_STRIDE;
            if (size_t(cnt) > SEG) {
                std::copy(pk.begin() + p0, pk.begin() + p0 + cnt, seg.begin() + std::ptrdiff_t(nb * SEG + over_at[b]));
                desc[4 * b + 2] = int32_t(nb * SEG + over_at[b]);
                std::fill(s, s + SEG, 0u);
                std::fill(rl, rl + SPMV_REL_STRIDE, uint16_t(0));
                continue;
            }
            std::copy(pk.begin() + p0, pk.begin() + p0 + cnt, s);
            std::fill(s + cnt, s + SEG, 0u);
            for (int t = 0; t < SPMV_REL_STRIDE; ++t) rl[t] = uint16_t(t <= nr ? rowptr[r0 + t] - p0 : cnt);
        }
    });
}


// Workgroup row ranges of the column-panel form: contiguous, an equal share
// of the entries each, at most PANEL_MAX_ROWS rows (the LDS accumulators).
std::vector<int32_t> panel_row_ranges(const int32_t* rowptr, int64_t nrows, int target_groups) {
    const int64_t nnz = rowptr[nrows];
    const int64_t want = std::max<int64_t>(1, (nnz + target_groups - 1) / std::max(1, target_groups));
    std::vector<int32_t> w{0};
    int64_t r = 0;
    while (r < nrows) {
        const int64_t r_nnz = std::upper_bound(rowptr + r, rowptr + nrows + 1, int64_t(rowptr[r]) + want - 1) - rowptr;
        int64_t r1 = std::min<int64_t>({nrows, std::max<int64_t>(r + 1, r_nnz), r + PANEL_MAX_ROWS});
        w.push_back(int32_t(r1));
        r = r1;
    }
    return w;
}

}  // namespace dev
}  // namespace ek
