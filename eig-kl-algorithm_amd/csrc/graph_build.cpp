// Clique expansions of the hypergraph (host side):
//   * fp64 Laplacian, restating initializeMatrix (cEIG.cpp:86-133);
//   * fp32 KL adjacency in cKL summation order, restating
//     InitializeSparsMatrix (cKL.cpp:84-149) + the iteration order of its
//     std::unordered_map<uint32_t,float> rows, emulated
//     here so the product does not depend on the host's libstdc++.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <memory>
#include <numeric>

#include "ek_internal.hpp"

namespace ek {

// ---------------------------------------------------------------------------
// libstdc++ (GCC 11) _Hashtable<uint32_t, ...> with _Prime_rehash_policy,
// max_load_factor 1, std::hash<uint32_t> = identity, bucket = key % B.
//
// Bucket counts a default-constructed map passes through; the first insert
// rehashes to 13 (_M_next_bkt(12) via the small-size table), after that a
// rehash to the smallest listed prime >= 2B happens when the element count
// reaches B.  Checked against the live libstdc++ by
// tests/test_host_logic.py::test_kl_row_order_large_rows (live libstdc++ rows).
static const uint64_t kBucketSeq[] = {13,     29,     59,      127,     257,     541,     1109,
                                      2357,   5087,   10273,   20753,   42043,   85229,   172933,
                                      351061, 712697, 1447153, 2938679, 5967347, 12117689};

uint64_t hashtable_next_buckets(uint64_t cur) {
    for (uint64_t b : kBucketSeq)
        if (b > cur) return b;
    fail(EK_EINVAL, "hash-order emulation: row exceeds %llu keys", (unsigned long long)cur);
}

// Emulates insertion of `cnt` distinct keys (first-insertion order) and
// writes the resulting begin()->end() iteration order.
//   insert (_M_insert_bucket_begin): non-empty bucket -> after the bucket's
//     "before" node; empty bucket -> list front, the old front's bucket now
//     points at the new node, this bucket points at before-begin;
//   rehash (_M_rehash_aux, unique keys): walk the old list in order; a node
//     whose new bucket is empty goes to the front (and the previous front's
//     bucket is re-pointed at it); otherwise after its bucket's before node.
void hashtable_order(const uint32_t* keys, int64_t cnt, uint32_t* out, std::vector<int32_t>& scratch) {
    std::vector<int32_t> b0, b1;
    hashtable_order(keys, cnt, out, scratch, b0, b1);
}
// (bk0 / bk1: the bucket arrays, reused across calls: no allocation per row)
void hashtable_order(const uint32_t* keys, int64_t cnt, uint32_t* out, std::vector<int32_t>& scratch,
                     std::vector<int32_t>& bk0, std::vector<int32_t>& bk1) {
    std::vector<int32_t> idx(static_cast<size_t>(cnt));
    hashtable_order_index(keys, cnt, idx.data(), scratch, bk0, bk1);
    for (int64_t q = 0; q < cnt; ++q) out[q] = keys[idx[size_t(q)]];
}
// the same iteration order as indices into keys (out_idx[q] = p: keys[p] is
// the q-th key iterated)
void hashtable_order_index(const uint32_t* keys, int64_t cnt, int32_t* out_idx, std::vector<int32_t>& scratch,
                           std::vector<int32_t>& bk0, std::vector<int32_t>& bk1) {
    constexpr int32_t NIL = -1, BB = -2, EMPTY = -3;
    if (cnt == 0) return;
    if (cnt <= 13) {
        // the first insert rehashes to 13 buckets and the next rehash comes
        // at the 14th key: a short row's whole life at B = 13 (the loop
        // below with a constant modulus and stack arrays)
        int32_t bkt[13], next[13], head = NIL;
        for (int32_t& x : bkt) x = EMPTY;
        for (int32_t node = 0; node < int32_t(cnt); ++node) {
            const uint32_t b = keys[node] % 13u;
            if (bkt[b] == EMPTY) {
                next[node] = head;
                head = node;
                if (next[node] != NIL) bkt[keys[next[node]] % 13u] = node;
                bkt[b] = BB;
            } else if (bkt[b] == BB) {
                next[node] = head;
                head = node;
            } else {
                next[node] = next[bkt[b]];
                next[bkt[b]] = node;
            }
        }
        int64_t q = 0;
        for (int32_t p = head; p != NIL; p = next[p]) out_idx[q++] = p;
        return;
    }
    scratch.resize(size_t(cnt));
    int32_t* next = scratch.data();
    std::vector<int32_t>* cur_b = &bk0;
    std::vector<int32_t>* spare = &bk1;
    cur_b->assign(1, EMPTY);
    uint64_t B = 1, next_resize = 0, count = 0;
    int32_t head = NIL;
    auto rehash = [&](uint64_t nb) {
        std::vector<int32_t>& nbk = *spare;
        nbk.assign(nb, EMPTY);
        int32_t p = head;
        head = NIL;
        uint64_t bbegin = 0;
        while (p != NIL) {
            const int32_t nx = next[p];
            const uint64_t b = keys[p] % nb;
            if (nbk[b] == EMPTY) {
                next[p] = head;
                head = p;
                nbk[b] = BB;
                if (next[p] != NIL) nbk[bbegin] = p;
                bbegin = b;
            } else if (nbk[b] == BB) {
                next[p] = head;
                head = p;
            } else {
                next[p] = next[nbk[b]];
                next[nbk[b]] = p;
            }
            p = nx;
        }
        std::swap(cur_b, spare);
        B = nb;
    };
    for (int64_t i = 0; i < cnt; ++i) {
        // _M_need_rehash(B, count, 1)
        if (count + 1 > next_resize) {
            const double min_bkts = double(std::max<uint64_t>(count + 1, next_resize ? 0 : 11));
            if (min_bkts >= double(B)) {
                const uint64_t want = std::max<uint64_t>(uint64_t(std::floor(min_bkts)) + 1, B * 2);
                uint64_t nb = want <= 13 ? 13 : 0;  // _M_next_bkt: small table gives 13 for 12..13
                if (!nb)
                    for (uint64_t b : kBucketSeq)
                        if (b >= want) {
                            nb = b;
                            break;
                        }
                if (!nb) fail(EK_EINVAL, "hash-order emulation: row too large");
                rehash(nb);
                next_resize = nb;
            } else {
                next_resize = B;
            }
        }
        const int32_t node = int32_t(i);
        const uint64_t b = keys[i] % B;
        if ((*cur_b)[b] == EMPTY) {
            next[node] = head;
            head = node;
            if (next[node] != NIL) (*cur_b)[keys[next[node]] % B] = node;
            (*cur_b)[b] = BB;
        } else if ((*cur_b)[b] == BB) {
            next[node] = head;
            head = node;
        } else {
            next[node] = next[(*cur_b)[b]];
            next[(*cur_b)[b]] = node;
        }
        ++count;
    }
    int64_t q = 0;
    for (int32_t p = head; p != NIL; p = next[p]) out_idx[q++] = p;
}

// ---------------------------------------------------------------------------
// cEIG.cpp:86-133.  Pairs (j<k) of every net contribute -2/|e| to (a,b) and
// (b,a); duplicates are summed (in net order here; setFromTriplets' order is
// thread-dependent in the reference); then diag = -(sum of row i in ascending
// column order, including any (i,i) triplets from repeated pins).
//
// Row-major form: every row is assembled from its own pin incidences (nets in
// ascending order, so each (row, col) sum runs in net order; contributions of
// one net are equal, so their order inside the net cannot change a bit),
// sorted by column, merged, and given its diagonal.  Threads own contiguous
// row ranges and write their rows to private buffers that are then copied into
// place, so there is no per-row allocation.  Rows [r0, r1) only: the shard of
// one rank of the sharded Lanczos (col keeps global ids).
void build_laplacian_rows(const ek_hgr& h, int64_t r0, int64_t r1, ek_csr& L) {
    const int64_t n = h.nodes, nr = r1 - r0;
    if (r0 < 0 || r1 > n || nr < 0) fail(EK_EINVAL, "Laplacian rows [%lld, %lld) outside [0, %lld)", (long long)r0,
                                         (long long)r1, (long long)n);
    PhaseTimer pt("laplacian");
    // incidences (pin position, net) of the owned rows, nets ascending: each
    // thread counts its own range of nets, and the per-thread counts give
    // every (thread, row) its slot range, so the parallel fill keeps net order
    const int TI = int(std::min<int64_t>(host_threads(), std::max<int64_t>(1, int64_t(h.pins.size()) / 65536)));
    std::vector<int64_t> ebeg(size_t(TI) + 1, 0);  // net ranges with balanced pin counts
    {
        const int64_t np = int64_t(h.pins.size());
        int64_t e = 0;
        for (int t = 1; t < TI; ++t) {
            const int64_t want = np * t / TI;
            while (e < h.nets && h.net_ptr[size_t(e)] < want) ++e;
            ebeg[size_t(t)] = e;
        }
        ebeg[size_t(TI)] = h.nets;
    }
    dvec<int32_t> tcnt(size_t(TI) * size_t(nr));
    run_threads(TI, [&](int t) {
        int32_t* c = tcnt.data() + size_t(t) * size_t(nr);
        std::fill(c, c + nr, 0);
        for (int64_t e = ebeg[size_t(t)]; e < ebeg[size_t(t) + 1]; ++e) {
            const int64_t p0 = h.net_ptr[size_t(e)], p1 = h.net_ptr[size_t(e) + 1];
            if (p1 - p0 < 2) continue;
            for (int64_t p = p0; p < p1; ++p) {
                const int64_t v = h.pins[size_t(p)];
                if (v >= r0 && v < r1) ++c[v - r0];
            }
        }
    });
    std::vector<int64_t> ip(size_t(nr) + 1, 0);
    for (int64_t i = 0; i < nr; ++i) {
        int64_t tot = 0;
        for (int t = 0; t < TI; ++t) tot += tcnt[size_t(t) * size_t(nr) + size_t(i)];
        ip[size_t(i) + 1] = ip[size_t(i)] + tot;
    }
    parallel_for(nr, [&](int64_t lo, int64_t hi) {  // counts -> each thread's first slot per row
        for (int64_t i = lo; i < hi; ++i) {
            int64_t at = ip[size_t(i)];
            for (int t = 0; t < TI; ++t) {
                int32_t& c = tcnt[size_t(t) * size_t(nr) + size_t(i)];
                const int32_t k = c;
                c = int32_t(at - ip[size_t(i)]);
                at += k;
            }
        }
    });
    dvec<int64_t> inc(size_t(ip[size_t(nr)]));  // pin position p
    dvec<int32_t> inc_net(inc.size());
    run_threads(TI, [&](int t) {
        int32_t* c = tcnt.data() + size_t(t) * size_t(nr);
        for (int64_t e = ebeg[size_t(t)]; e < ebeg[size_t(t) + 1]; ++e) {
            const int64_t p0 = h.net_ptr[size_t(e)], p1 = h.net_ptr[size_t(e) + 1];
            if (p1 - p0 < 2) continue;
            for (int64_t p = p0; p < p1; ++p) {
                const int64_t v = h.pins[size_t(p)];
                if (v >= r0 && v < r1) {
                    const int64_t q = ip[size_t(v - r0)] + c[v - r0]++;
                    inc[size_t(q)] = p;
                    inc_net[size_t(q)] = int32_t(e);
                }
            }
        }
    });
    pt.mark("incidences");
    const int T = int(std::min<int64_t>(host_threads(), std::max<int64_t>(1, nr / 4096)));
    std::vector<std::vector<int32_t>> tcol{size_t(T)};
    std::vector<std::vector<double>> tval{size_t(T)};
    std::vector<int32_t> rlen(size_t(nr), 0);
    auto work = [&](int t) {
        const int64_t lo = nr * t / T, hi = nr * (t + 1) / T;
        // (built in locals and moved out at the end: the threads' vectors sit
        // side by side in tcol / tval, and push_back writes their ends)
        std::vector<int32_t> oc;
        std::vector<double> ov;
        oc.reserve(size_t(ip[size_t(hi)] - ip[size_t(lo)]) * 4 + 16);
        ov.reserve(oc.capacity());
        std::vector<std::pair<int32_t, double>> row;
        for (int64_t i = lo; i < hi; ++i) {
            const int32_t r = int32_t(r0 + i);
            row.clear();
            for (int64_t q = ip[size_t(i)]; q < ip[size_t(i) + 1]; ++q) {
                const int64_t e = inc_net[size_t(q)], p0 = h.net_ptr[size_t(e)], p1 = h.net_ptr[size_t(e) + 1];
                const double w = -(2.0 / double(p1 - p0));
                for (int64_t p = p0; p < p1; ++p)
                    if (p != inc[size_t(q)]) row.push_back({h.pins[size_t(p)], w});
            }
            // stable by column: insertion sort (rows average ~6 entries)
            if (row.size() <= 48) {
                for (size_t a = 1; a < row.size(); ++a) {
                    const auto x = row[a];
                    size_t b = a;
                    for (; b > 0 && row[b - 1].first > x.first; --b) row[b] = row[b - 1];
                    row[b] = x;
                }
            } else {
                std::stable_sort(row.begin(), row.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
            }
            size_t m = 0;  // merge duplicates in order
            for (size_t a = 0; a < row.size(); ++a) {
                if (m > 0 && row[m - 1].first == row[a].first) row[m - 1].second += row[a].second;
                else row[m++] = row[a];
            }
            row.resize(m);
            double s = 0.0;
            bool has_diag = false;
            for (auto& [c, v] : row) {
                s += v;
                has_diag |= (c == r);
            }
            const size_t base = oc.size();
            bool placed = has_diag;
            for (auto& [c, v] : row) {
                if (!placed && c > r) {
                    oc.push_back(r);
                    ov.push_back(-s);
                    placed = true;
                }
                oc.push_back(c);
                ov.push_back(c == r ? -s : v);
            }
            if (!placed) {
                oc.push_back(r);
                ov.push_back(-s);
            }
            rlen[size_t(i)] = int32_t(oc.size() - base);
        }
        tcol[size_t(t)] = std::move(oc);
        tval[size_t(t)] = std::move(ov);
    };
    run_threads(T, work);
    pt.mark("rows");
    L.nrows = nr;
    L.value_bytes = 8;
    L.rowptr.assign(size_t(nr) + 1, 0);
    for (int64_t i = 0; i < nr; ++i) {
        if (int64_t(L.rowptr[size_t(i)]) + rlen[size_t(i)] > INT32_MAX) fail(EK_EINVAL, "Laplacian nnz exceeds int32");
        L.rowptr[size_t(i) + 1] = L.rowptr[size_t(i)] + rlen[size_t(i)];
    }
    L.col.resize(size_t(L.rowptr[size_t(nr)]));
    L.val64.resize(L.col.size());
    run_threads(T, [&](int t) {
        const int64_t at = L.rowptr[size_t(nr * t / T)];
        std::copy(tcol[size_t(t)].begin(), tcol[size_t(t)].end(), L.col.begin() + at);
        std::copy(tval[size_t(t)].begin(), tval[size_t(t)].end(), L.val64.begin() + at);
    });
    pt.mark("assemble");
}

void build_laplacian(const ek_hgr& h, ek_csr& L) { build_laplacian_rows(h, 0, h.nodes, L); }

// ---------------------------------------------------------------------------
// cKL.cpp:107-131 + connections() order (cKL.cpp:229-248).
// Every phase parallel, no atomics, no per-row allocations, and no per-thread
// arrays of n counts (round 6: the T x n count matrix of round 4, 128 MB at
// the 10x graph on 16 threads, was zeroed and walked four times).  Rows go to
// T owners by a multiply-shift (owner(r) = r M >> 32, nondecreasing), so each
// owner holds a contiguous row range.  Thread t walks the nets
// [nets t/T, nets (t+1)/T) in phase A and owner t's rows in phases B and C:
//   A. pairs (j < q) of every net, by smaller endpoint: counted per (thread,
//      owner), then written to the owner's bucket in thread order — so each
//      row's pairs lie in the reference's loop order — and sorted by row
//      within the owner (a stable counting sort over its own rows);
//   B. per row: distinct keys in first-pair order (the map's insertion
//      order) with their pairs' fp32 sums in loop order, then through the
//      emulated map iteration, into the thread's own buffer;
//   C. backward parts (for node k, the rows i < k holding k): every forward
//      entry is bucketed by k's owner in row order and counting-sorted by k,
//      which puts each list in ascending row order without a comparison sort.
// The result is the round-3 form's, bit for bit (test_kl_graph_matches_oracle,
// test_kl_row_order_*, test_kl_graph_repeated_pins).
void build_kl_graph(const ek_hgr& h, ek_csr& G) {
    PhaseTimer pt("kl_graph");
    const int64_t n = h.nodes, nets = h.nets;
    const int T = int(std::max<int64_t>(1, std::min<int64_t>(host_threads(), std::max<int64_t>(1, n / 4096))));
    const uint64_t M = n > 0 ? (uint64_t(T) << 32) / uint64_t(n) : 0;
    auto owner = [M](uint64_t r) { return int(uint64_t(r * M) >> 32); };  // < T for r < n
    std::vector<int64_t> lo(size_t(T) + 1);  // owner u's rows: [lo[u], lo[u + 1])
    for (int u = 0; u <= T; ++u) {
        int64_t r = (u == T || M == 0) ? n : std::min<int64_t>(n, int64_t((uint64_t(u) << 32) / M));
        while (r > 0 && owner(uint64_t(r - 1)) >= u) --r;
        while (r < n && owner(uint64_t(r)) < u) ++r;
        lo[size_t(u)] = r;
    }
    // per (thread, owner) counts -> slot bases: bucket u holds threads 0..T-1 in order
    // (rows HS int64 apart, HS a whole number of 64-B lines plus one: no two
    // threads' counters share a cache line — the counts are incremented per
    // pair, and a shared line cost the rows phase most of its thread scaling)
    const size_t HS = (size_t(T) + 7) / 8 * 8 + 8;
    std::vector<int64_t> hc(size_t(T) * HS);
    std::vector<int64_t> base(size_t(T) + 1);
    auto bucket_bases = [&]() {
        int64_t run = 0;
        for (int u = 0; u < T; ++u) {
            base[size_t(u)] = run;
            for (int t = 0; t < T; ++t) {
                int64_t& x = hc[size_t(t) * HS + size_t(u)];
                const int64_t v = x;
                x = run;
                run += v;
            }
        }
        base[size_t(T)] = run;
    };
    // A. pairs by smaller endpoint
    run_threads(T, [&](int t) {
        int64_t* c = hc.data() + size_t(t) * HS;
        for (int64_t e = nets * t / T; e < nets * (t + 1) / T; ++e) {
            const int64_t p0 = h.net_ptr[size_t(e)], k = h.net_ptr[size_t(e) + 1] - p0;
            const int32_t* pe = h.pins.data() + p0;
            for (int64_t j = 0; j + 1 < k; ++j)
                for (int64_t q = j + 1; q < k; ++q) ++c[owner(uint32_t(std::min(pe[j], pe[q])))];
        }
    });
    bucket_bases();
    const int64_t npairs = base[size_t(T)];
    dvec<uint32_t> tr(static_cast<size_t>(npairs)), tk(static_cast<size_t>(npairs));  // bucketed (row, key)
    dvec<float> tw(static_cast<size_t>(npairs));
    run_threads(T, [&](int t) {
        int64_t* c = hc.data() + size_t(t) * HS;
        for (int64_t e = nets * t / T; e < nets * (t + 1) / T; ++e) {
            const int64_t p0 = h.net_ptr[size_t(e)], k = h.net_ptr[size_t(e) + 1] - p0;
            if (k < 2) continue;
            const float weight = 1.0f / float(k - 1);  // cKL.cpp:117
            const int32_t* pe = h.pins.data() + p0;
            for (int64_t j = 0; j + 1 < k; ++j)
                for (int64_t q = j + 1; q < k; ++q) {
                    const uint32_t a = uint32_t(std::min(pe[j], pe[q])), b = uint32_t(std::max(pe[j], pe[q]));
                    const int64_t at = c[owner(a)]++;
                    tr[size_t(at)] = a;
                    tk[size_t(at)] = b;
                    tw[size_t(at)] = weight;
                }
        }
    });
    dvec<int64_t> cnt(static_cast<size_t>(n) + 1);
    dvec<uint32_t> pk(static_cast<size_t>(npairs));
    dvec<float> pw(static_cast<size_t>(npairs));
    run_threads(T, [&](int u) {  // owner u: its bucket counting-sorted by row (stable)
        const int64_t r0 = lo[size_t(u)], r1 = lo[size_t(u) + 1], s0 = base[size_t(u)], s1 = base[size_t(u) + 1];
        std::vector<int64_t> cur(size_t(r1 - r0) + 1, 0);
        for (int64_t x = s0; x < s1; ++x) ++cur[size_t(tr[size_t(x)] - r0) + 1];
        cur[0] = s0;
        for (int64_t r = r0; r < r1; ++r) cur[size_t(r - r0) + 1] += cur[size_t(r - r0)];
        for (int64_t r = r0; r <= r1; ++r)
            if (r < r1 || u == T - 1) cnt[size_t(r)] = cur[size_t(r - r0)];
        for (int64_t x = s0; x < s1; ++x) {
            const int64_t at = cur[size_t(tr[size_t(x)] - r0)]++;
            pk[size_t(at)] = tk[size_t(x)];
            pw[size_t(at)] = tw[size_t(x)];
        }
    });
    if (n == 0) cnt[0] = 0;
    pt.mark("pairs");
    // B. rows: forward lists in map order, per thread, rows in order
    struct alignas(64) Part {  // (own cache lines: push_back writes the vectors' ends)
        std::vector<uint32_t> key;
        std::vector<float> w;
        std::vector<int64_t> off;  // row r's entries at [off[r - lo], off[r - lo + 1])
    };
    std::vector<Part> parts(static_cast<size_t>(T));
    dvec<int32_t> fcnt(static_cast<size_t>(n));
    std::atomic<bool> too_big{false};
    std::fill(hc.begin(), hc.end(), 0);  // now: thread t's backward entries by their node's owner
    run_threads(T, [&](int t) {
        const int64_t r0 = lo[size_t(t)], r1 = lo[size_t(t) + 1];
        Part& P = parts[size_t(t)];
        P.off.assign(size_t(r1 - r0) + 1, 0);
        P.key.clear();
        P.w.clear();
        P.key.reserve(size_t(cnt[size_t(r1)] - cnt[size_t(r0)]));
        P.w.reserve(size_t(cnt[size_t(r1)] - cnt[size_t(r0)]));
        int64_t* bc = hc.data() + size_t(t) * HS;
        std::vector<int64_t> idx;
        std::vector<int32_t> scratch, bk0, bk1;
        std::vector<std::pair<int64_t, std::pair<uint32_t, float>>> first;  // (first pair, (key, sum))
        std::vector<uint32_t> keys, order;
        std::vector<std::pair<uint32_t, float>> bykey;
        std::vector<float> dsum;
        std::vector<int32_t> oidx;
        for (int64_t a = r0; a < r1; ++a) {
            const int64_t b = cnt[size_t(a)], e = cnt[size_t(a) + 1];
            if (b == e) {
                P.off[size_t(a - r0) + 1] = int64_t(P.key.size());
                fcnt[size_t(a)] = 0;
                continue;
            }
            if (e - b <= 64) {
                // a short row (all but hubs): its distinct keys in first-
                // occurrence order and their sums in pair order, by a linear
                // search — the sort path's keys and fp32 sums, without sorting
                keys.clear();
                dsum.clear();
                for (int64_t x = b; x < e; ++x) {
                    const uint32_t key = pk[size_t(x)];
                    size_t u = 0;
                    while (u < keys.size() && keys[u] != key) ++u;
                    if (u == keys.size()) {
                        keys.push_back(key);
                        dsum.push_back(0.0f + pw[size_t(x)]);  // operator[]'s 0.0f, then += in pair order
                    } else {
                        dsum[u] += pw[size_t(x)];
                    }
                }
                oidx.resize(keys.size());
                try {
                    hashtable_order_index(keys.data(), int64_t(keys.size()), oidx.data(), scratch, bk0, bk1);
                } catch (const Error&) {
                    too_big = true;
                    return;
                }
                for (int32_t p : oidx) {
                    const uint32_t key = keys[size_t(p)];
                    P.key.push_back(key);
                    P.w.push_back(dsum[size_t(p)]);
                    if (int64_t(key) != a) ++bc[owner(key)];
                }
                fcnt[size_t(a)] = int32_t(oidx.size());
                P.off[size_t(a - r0) + 1] = int64_t(P.key.size());
                continue;
            }
            idx.resize(size_t(e - b));
            std::iota(idx.begin(), idx.end(), b);
            std::stable_sort(idx.begin(), idx.end(), [&](int64_t x, int64_t y) { return pk[size_t(x)] < pk[size_t(y)]; });
            first.clear();
            bykey.clear();
            for (size_t u = 0; u < idx.size();) {
                const uint32_t key = pk[size_t(idx[u])];
                float sum = 0.0f;  // operator[] value-initialises to 0.0f, then += in net order
                const int64_t seq0 = idx[u];
                for (; u < idx.size() && pk[size_t(idx[u])] == key; ++u) sum += pw[size_t(idx[u])];
                first.push_back({seq0, {key, sum}});
                bykey.push_back({key, sum});  // (ascending keys)
            }
            std::sort(first.begin(), first.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
            keys.resize(first.size());
            for (size_t u = 0; u < first.size(); ++u) keys[u] = first[u].second.first;
            order.resize(keys.size());
            try {
                hashtable_order(keys.data(), int64_t(keys.size()), order.data(), scratch, bk0, bk1);
            } catch (const Error&) {
                too_big = true;
                return;
            }
            for (uint32_t key : order) {
                const auto it = std::lower_bound(bykey.begin(), bykey.end(), std::make_pair(key, -INFINITY));
                P.key.push_back(key);
                P.w.push_back(it->second);
                if (int64_t(key) != a) ++bc[owner(key)];
            }
            fcnt[size_t(a)] = int32_t(order.size());
            P.off[size_t(a - r0) + 1] = int64_t(P.key.size());
        }
    });
    if (too_big) fail(EK_EINVAL, "hash-order emulation: a row exceeds the bucket table");
    pt.mark("rows + map order");
    // C. assemble: backward entries bucketed by their node's owner, rows ascending
    bucket_bases();
    run_threads(T, [&](int t) {  // (reuses the pair buckets: backward entries <= pairs)
        const int64_t r0 = lo[size_t(t)], r1 = lo[size_t(t) + 1];
        const Part& P = parts[size_t(t)];
        int64_t* c = hc.data() + size_t(t) * HS;
        for (int64_t r = r0; r < r1; ++r)
            for (int64_t q = P.off[size_t(r - r0)]; q < P.off[size_t(r - r0) + 1]; ++q) {
                const uint32_t k = P.key[size_t(q)];
                if (int64_t(k) == r) continue;
                const int64_t at = c[owner(k)]++;
                tk[size_t(at)] = k;
                tr[size_t(at)] = uint32_t(r);
                tw[size_t(at)] = P.w[size_t(q)];
            }
    });
    std::vector<int64_t> rsum(size_t(T) + 1, 0);  // per owner: its rows' lengths, then their offsets
    std::vector<std::vector<int32_t>> bcur(static_cast<size_t>(T));
    run_threads(T, [&](int u) {
        const int64_t r0 = lo[size_t(u)], r1 = lo[size_t(u) + 1];
        std::vector<int32_t>& bk = bcur[size_t(u)];
        bk.assign(size_t(r1 - r0), 0);
        for (int64_t x = base[size_t(u)]; x < base[size_t(u) + 1]; ++x) ++bk[size_t(tk[size_t(x)] - r0)];
        int64_t s = 0;
        for (int64_t r = r0; r < r1; ++r) s += int64_t(fcnt[size_t(r)]) + bk[size_t(r - r0)];
        rsum[size_t(u) + 1] = s;
    });
    for (int u = 0; u < T; ++u) rsum[size_t(u) + 1] += rsum[size_t(u)];
    if (rsum[size_t(T)] > INT32_MAX) fail(EK_EINVAL, "KL graph nnz exceeds int32");
    G.nrows = n;
    G.value_bytes = 4;
    G.rowptr.resize(size_t(n) + 1);
    G.nfwd.resize(size_t(n));
    G.rowptr[0] = 0;
    G.col.resize(size_t(rsum[size_t(T)]));
    G.val32.resize(size_t(rsum[size_t(T)]));
    run_threads(T, [&](int u) {
        const int64_t r0 = lo[size_t(u)], r1 = lo[size_t(u) + 1];
        const Part& P = parts[size_t(u)];
        std::vector<int32_t>& bk = bcur[size_t(u)];
        int64_t p = rsum[size_t(u)];
        for (int64_t r = r0; r < r1; ++r) {  // rowptr; forward part; bk becomes the backward cursor
            G.nfwd[size_t(r)] = fcnt[size_t(r)];
            for (int64_t q = P.off[size_t(r - r0)]; q < P.off[size_t(r - r0) + 1]; ++q) {
                G.col[size_t(p)] = int32_t(P.key[size_t(q)]);
                G.val32[size_t(p++)] = P.w[size_t(q)];
            }
            const int32_t nb = bk[size_t(r - r0)];
            bk[size_t(r - r0)] = int32_t(p);
            p += nb;
            G.rowptr[size_t(r) + 1] = int32_t(p);
        }
        for (int64_t x = base[size_t(u)]; x < base[size_t(u) + 1]; ++x) {  // backward parts, rows ascending
            const int32_t at = bk[size_t(tk[size_t(x)] - r0)]++;
            G.col[size_t(at)] = int32_t(tr[size_t(x)]);
            G.val32[size_t(at)] = tw[size_t(x)];
        }
    });
    pt.mark("assemble");
}

}  // namespace ek

extern "C" {

int ek_laplacian_build(const ek_hgr* h, ek_csr** out) {
    EK_TRY
    if (!h || !out) ek::fail(EK_EINVAL, "ek_laplacian_build: null argument");
    auto c = std::make_unique<ek_csr>();
    ek::build_laplacian(*h, *c);
    *out = c.release();
    return EK_OK;
    EK_CATCH
}

int ek_laplacian_build_rows(const ek_hgr* h, int64_t row0, int64_t nrows, ek_csr** out) {
    EK_TRY
    if (!h || !out || row0 < 0 || nrows < 0) ek::fail(EK_EINVAL, "ek_laplacian_build_rows: bad argument");
    auto c = std::make_unique<ek_csr>();
    ek::build_laplacian_rows(*h, row0, row0 + nrows, *c);
    *out = c.release();
    return EK_OK;
    EK_CATCH
}

int ek_kl_graph_build(const ek_hgr* h, ek_csr** out) {
    EK_TRY
    if (!h || !out) ek::fail(EK_EINVAL, "ek_kl_graph_build: null argument");
    auto c = std::make_unique<ek_csr>();
    ek::build_kl_graph(*h, *c);
    *out = c.release();
    return EK_OK;
    EK_CATCH
}

int ek_csr_dims(const ek_csr* c, int64_t* nrows, int64_t* nnz, int32_t* value_bytes) {
    if (!c) {
        ek::set_error("ek_csr_dims: null handle");
        return EK_EINVAL;
    }
    if (nrows) *nrows = c->nrows;
    if (nnz) *nnz = int64_t(c->col.size());
    if (value_bytes) *value_bytes = c->value_bytes;
    return EK_OK;
}

int ek_csr_copy(const ek_csr* c, int32_t* rowptr, int32_t* col, void* val, int32_t* nfwd) {
    if (!c) {
        ek::set_error("ek_csr_copy: null handle");
        return EK_EINVAL;
    }
    if (rowptr) std::copy(c->rowptr.begin(), c->rowptr.end(), rowptr);
    if (col) std::copy(c->col.begin(), c->col.end(), col);
    if (val) {
        if (c->value_bytes == 8) std::memcpy(val, c->val64.data(), c->val64.size() * 8);
        else std::memcpy(val, c->val32.data(), c->val32.size() * 4);
    }
    if (nfwd && !c->nfwd.empty()) std::copy(c->nfwd.begin(), c->nfwd.end(), nfwd);
    return EK_OK;
}

void ek_csr_free(ek_csr* c) { delete c; }

int ek_shard_rows(int64_t n, int nranks, int rank, int64_t* row0, int64_t* nrows, int64_t* nloc) {
    if (n < 0 || nranks < 1 || rank < 0 || rank >= nranks) {
        ek::set_error("ek_shard_rows: bad argument");
        return EK_EINVAL;
    }
    int64_t blk = (n + nranks - 1) / nranks;
    blk = (blk + 63) / 64 * 64;  // 512-byte aligned fp64 slices for the all-gather
    const int64_t r0 = std::min<int64_t>(n, blk * rank);
    if (row0) *row0 = r0;
    if (nrows) *nrows = std::min<int64_t>(n, blk * (rank + 1)) - r0;
    if (nloc) *nloc = blk;
    return EK_OK;
}

// nnz-balanced 1-D row partition.  Row weight = the Laplacian
// row's entries before duplicate pairs merge: 1 (diagonal) + sum over its
// nets of |e| - 1, i.e. its share of the triplets initializeMatrix hands to
// setFromTriplets (cEIG.cpp:86-133).  O(pins) and identical on every rank;
// the exact merged count would need the clique expansion itself.  Measured
// on the shipped circuits the exact per-rank nnz stays within 1.045 x the
// mean at 2/4/8 ranks (tests/test_host_logic.py), where equal row blocks
// reach 2.57 x on industry2 (hub rows of 1,634 entries).  Rank r owns
// [off[r], off[r+1]): the first row whose weight prefix reaches r/R of the
// total starts rank r.
int ek_shard_map(int64_t n, int64_t nets, const int64_t* net_ptr, const int32_t* pins, int nranks,
                 int64_t* row_offsets) {
    EK_TRY
    if (n < 0 || nets < 0 || nranks < 1 || !row_offsets || (nets && !net_ptr) || (nets && net_ptr[nets] > 0 && !pins))
        ek::fail(EK_EINVAL, "ek_shard_map: bad argument");
    if (nranks == 1) {
        row_offsets[0] = 0;
        row_offsets[1] = n;
        return EK_OK;
    }
    std::unique_ptr<std::atomic<int64_t>[]> wgt(new std::atomic<int64_t>[size_t(std::max<int64_t>(n, 1))]);
    ek::parallel_for(n, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i) wgt[size_t(i)].store(1, std::memory_order_relaxed);
    });
    std::atomic<bool> bad{false};
    ek::parallel_for(nets, [&](int64_t lo, int64_t hi) {
        for (int64_t e = lo; e < hi; ++e) {
            const int64_t p0 = net_ptr[e], k = net_ptr[e + 1] - p0;
            if (k < 2) continue;
            for (int64_t p = p0; p < p0 + k; ++p) {
                const int32_t v = pins[p];
                if (v < 0 || v >= n) {
                    bad = true;
                    continue;
                }
                wgt[size_t(v)].fetch_add(k - 1, std::memory_order_relaxed);
            }
        }
    });
    if (bad) ek::fail(EK_EINVAL, "ek_shard_map: pin out of range");
    int64_t tot = 0;
    for (int64_t i = 0; i < n; ++i) tot += wgt[size_t(i)].load(std::memory_order_relaxed);
    row_offsets[0] = 0;
    int r = 1;
    int64_t acc = 0;
    for (int64_t i = 0; i < n && r < nranks; ++i) {
        // rank r starts at the first row whose prefix (rows before it) reaches r/R of the total
        while (r < nranks && acc * nranks >= tot * r) row_offsets[r++] = i;
        acc += wgt[size_t(i)].load(std::memory_order_relaxed);
    }
    while (r < nranks) row_offsets[r++] = n;
    row_offsets[nranks] = n;
    return EK_OK;
    EK_CATCH
}

}  // extern "C"

