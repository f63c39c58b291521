// ORACLE — test infrastructure only.
//
// CPU restatement of the reference KL path (yhinai/EIG-KL-Algorithm, cKL.cpp)
// used as the parity checker for the MI355X product.  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load or run
// anything under oracle/; the product (libeigkl_hip.so and the
// cEIG/cKL/gKL/gKL2 CLIs) never links it and has no CPU fallback.
//
// Pinned by (tests/test_oracle_golden.py):
//   * the REAL reference cKL, compiled from /root/reference/cKL.cpp into
//     oracle/_ref/ by oracle/ref.mk and run by oracle/gen_golden.py; its
//     results files are committed under tests/golden/ref_results/ and must
//     match this restatement row for row;
//   * SURVEY §8c known answers, swap-log md5 prefixes, best-prefix
//     iterations and integer net cuts.
//
// It is deliberately written the reference's way — rows are real
// std::unordered_map<uint32_t,float> filled in net order, so forward
// summation order is the real libstdc++ iteration order — which keeps it
// independent of the product's hash-order emulator (graph_build.cpp).
// Only the asymptotics differ: the O(n) hash-set rebuild per gain call
// (cKL.cpp:227) and the O(n) backward scan (cKL.cpp:239-248) are replaced by
// a precomputed backward list with the same ascending order, so the fp32
// operation sequence per gain is unchanged.

#include "eko.h"
#include "eko_internal.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <fstream>
#include <limits>
#include <random>

#include <omp.h>
#include <sstream>
#include <string>

namespace {

// cKL.cpp:107-131: w = 1.0f/(k-1); adjacencyList[min][max] += w, nets in file order.
void build_adjacency(eko_graph& g) {
    g.adj.assign(g.nodes, {});
    for (uint32_t e = 0; e < g.nets; ++e) {
        const int64_t p0 = g.net_ptr[e], p1 = g.net_ptr[e + 1];
        const size_t k = size_t(p1 - p0);
        const float weight = 1.0f / (k - 1);
        for (size_t j = 0; j < k; j++)
            for (size_t q = j + 1; q < k; q++) {
                uint32_t a = uint32_t(g.pins[p0 + j]), b = uint32_t(g.pins[p0 + q]);
                if (a > b) std::swap(a, b);
                g.adj[a][b] += weight;
            }
    }
}

// Row u of the KL graph in connections() order (cKL.cpp:229-248): forward
// entries in unordered_map iteration order, then every i < u with u in adj[i],
// ascending i.
void build_csr(eko_graph& g) {
    if (!g.rowptr.empty()) return;
    const uint32_t n = g.nodes;
    std::vector<std::vector<std::pair<uint32_t, float>>> back(n);
    for (uint32_t i = 0; i < n; ++i)
        for (const auto& [k, wt] : g.adj[i])
            if (k != i) back[k].push_back({i, wt});  // i ascending by construction
    g.rowptr.assign(n + 1, 0);
    g.nfwd.assign(n, 0);
    for (uint32_t u = 0; u < n; ++u) {
        g.nfwd[u] = int32_t(g.adj[u].size());
        g.rowptr[u + 1] = g.rowptr[u] + int32_t(g.adj[u].size() + back[u].size());
    }
    g.col.resize(g.rowptr[n]);
    g.w.resize(g.rowptr[n]);
    for (uint32_t u = 0; u < n; ++u) {
        int32_t p = g.rowptr[u];
        for (const auto& [k, wt] : g.adj[u]) { g.col[p] = int32_t(k); g.w[p] = wt; ++p; }
        for (const auto& [i, wt] : back[u]) { g.col[p] = int32_t(i); g.w[p] = wt; ++p; }
    }
}

// connections(node) (cKL.cpp:225-251): sequential fp32 sums in row order,
// internal = neighbour in split[0].
inline float connections(const eko_graph& g, const std::vector<uint8_t>& side, uint32_t u,
                         float* external_out = nullptr) {
    float external = 0.0f, internal = 0.0f;
    for (int32_t p = g.rowptr[u]; p < g.rowptr[u + 1]; ++p) {
        if (side[g.col[p]] == 0) internal += g.w[p];
        else external += g.w[p];
    }
    if (external_out) *external_out = external;
    return external - internal;
}

// getEdgeWeight (cKL.cpp:75-82)
inline float edge_weight(const eko_graph& g, uint32_t a, uint32_t b) {
    if (a > b) std::swap(a, b);
    auto it = g.adj[a].find(b);
    return it != g.adj[a].end() ? it->second : 0.0f;
}

int finish_graph(eko_graph* g, eko_graph** out) {
    build_adjacency(*g);
    *out = g;
    return 0;
}

}  // namespace

extern "C" {

int eko_read(const char* path, eko_graph** out) {
    std::ifstream fin(path);
    if (!fin.is_open()) return -2;
    std::string line;
    std::getline(fin, line);
    uint32_t nets = 0, nodes = 0;
    std::stringstream(line) >> nets >> nodes;  // cKL.cpp:93-95
    auto* g = new eko_graph;
    g->nets = nets;
    g->nodes = nodes;
    g->net_ptr.push_back(0);
    for (uint32_t i = 0; i < nets; i++) {  // cKL.cpp:107-116
        std::getline(fin, line);
        std::stringstream ss(line);
        uint32_t node;
        while (ss >> node) {
            if (node < 1 || node > nodes) { delete g; return -1; }
            g->pins.push_back(int32_t(node - 1));
        }
        g->net_ptr.push_back(int64_t(g->pins.size()));
    }
    return finish_graph(g, out);
}

int eko_from_pins(int64_t nets, int64_t nodes, const int64_t* net_ptr, const int32_t* pins,
                  eko_graph** out) {
    auto* g = new eko_graph;
    g->nets = uint32_t(nets);
    g->nodes = uint32_t(nodes);
    g->net_ptr.assign(net_ptr, net_ptr + nets + 1);
    g->pins.assign(pins, pins + net_ptr[nets]);
    return finish_graph(g, out);
}

void eko_free(eko_graph* g) { delete g; }
int64_t eko_nodes(const eko_graph* g) { return g->nodes; }
int64_t eko_nets(const eko_graph* g) { return g->nets; }

int64_t eko_kl_csr(const eko_graph* cg, int32_t* rowptr, int32_t* col, float* w, int32_t* nfwd) {
    auto* g = const_cast<eko_graph*>(cg);
    build_csr(*g);
    const int64_t nnz = g->rowptr[g->nodes];
    if (rowptr) std::copy(g->rowptr.begin(), g->rowptr.end(), rowptr);
    if (col) std::copy(g->col.begin(), g->col.end(), col);
    if (w) std::copy(g->w.begin(), g->w.end(), w);
    if (nfwd) std::copy(g->nfwd.begin(), g->nfwd.end(), nfwd);
    return nnz;
}

int64_t eko_net_cut(const eko_graph* g, const uint8_t* side) {
    int64_t cut = 0;
    for (uint32_t e = 0; e < g->nets; ++e) {
        const int64_t p0 = g->net_ptr[e], p1 = g->net_ptr[e + 1];
        bool crosses = false;
        for (int64_t p = p0 + 1; p < p1 && !crosses; ++p) crosses = side[g->pins[p]] != side[g->pins[p0]];
        cut += crosses;
    }
    return cut;
}

// KL() (cKL.cpp:288-406) with the remain[] lists given (shuffleSparceMatrix,
// cKL.cpp:151-197, is done by the caller: EIG file order or a seeded shuffle).
int eko_kl(const eko_graph* cg, const int32_t* order0, int64_t n0, const int32_t* order1, int64_t n1,
           int32_t limit, eko_swap* log, int64_t cap, eko_kl_result* res) {
    auto* g = const_cast<eko_graph*>(cg);
    build_csr(*g);
    const uint32_t n = g->nodes;
    std::vector<uint8_t> side(n, 2), locked(n, 0);
    for (int64_t i = 0; i < n0; ++i) side[order0[i]] = 0;
    for (int64_t i = 0; i < n1; ++i) side[order1[i]] = 1;
    const std::vector<uint8_t> side_init = side;
    // terminateLimit (cKL.cpp:303)
    const uint32_t terminateLimit =
        limit >= 0 ? uint32_t(limit) : static_cast<uint32_t>(std::log2(double(n))) + 5;

    // Initial cut (cKL.cpp:199-223): every left-right edge counted once from its
    // left endpoint.  The reference's OpenMP fp32 reduction has no fixed order;
    // here: fp32 per-node external sums (row order), added in fp64 by ascending
    // node id, rounded once to fp32 (DESIGN.md "initial cut").
    std::vector<float> gains(n, 0.0f), ext(n, 0.0f);
#pragma omp parallel for schedule(static)  // initial gains (cKL.cpp:317-321, omp parallel for there too)
    for (int64_t u = 0; u < int64_t(n); ++u) gains[u] = connections(*g, side, uint32_t(u), &ext[u]);
    double cut64 = 0.0;
    for (uint32_t u = 0; u < n; ++u)
        if (side[u] == 0) cut64 += double(ext[u]);
    float cutSize = float(cut64);
    const float initialCutSize = cutSize;
    float minCutSize = cutSize;
    int64_t best_iter = 0;

    uint32_t iteration = 0, terminate = 0;
    int64_t alive0 = n0, alive1 = n1;
    std::vector<uint32_t> affected;
    while (alive0 > 0 && alive1 > 0) {  // cKL.cpp:334
        // cKL.cpp:341-355 (locked == erased): first position with the max
        // (strict >) gain over remain[0], the min (strict <) over remain[1].
        // Sequential in the reference; split over threads here, each keeping
        // its first best, merged by (gain, then lower position): the same pick.
        float maxGain = -std::numeric_limits<float>::max();
        float minGain = std::numeric_limits<float>::max();
        int64_t maxIdx = -1, minIdx = -1;
        const int nth = omp_get_max_threads();
        if (nth <= 1 || n0 + n1 < 8192) {
            for (int64_t i = 0; i < n0; ++i) {
                const uint32_t u = uint32_t(order0[i]);
                if (!locked[u] && gains[u] > maxGain) { maxGain = gains[u]; maxIdx = i; }
            }
            for (int64_t i = 0; i < n1; ++i) {
                const uint32_t u = uint32_t(order1[i]);
                if (!locked[u] && gains[u] < minGain) { minGain = gains[u]; minIdx = i; }
            }
        } else {
#pragma omp parallel
            {
                float mx = -std::numeric_limits<float>::max(), mn = std::numeric_limits<float>::max();
                int64_t ix = -1, in = -1;
#pragma omp for schedule(static) nowait
                for (int64_t i = 0; i < n0; ++i) {
                    const uint32_t u = uint32_t(order0[i]);
                    if (!locked[u] && gains[u] > mx) { mx = gains[u]; ix = i; }
                }
#pragma omp for schedule(static) nowait
                for (int64_t i = 0; i < n1; ++i) {
                    const uint32_t u = uint32_t(order1[i]);
                    if (!locked[u] && gains[u] < mn) { mn = gains[u]; in = i; }
                }
#pragma omp critical
                {
                    if (ix >= 0 && (maxIdx < 0 || mx > maxGain || (mx == maxGain && ix < maxIdx))) { maxGain = mx; maxIdx = ix; }
                    if (in >= 0 && (minIdx < 0 || mn < minGain || (mn == minGain && in < minIdx))) { minGain = mn; minIdx = in; }
                }
            }
        }
        if (maxIdx < 0 || minIdx < 0) break;  // cKL.cpp:387-388
        const uint32_t node1 = uint32_t(order0[maxIdx]), node2 = uint32_t(order1[minIdx]);
        const float gain = maxGain - minGain - 2.0f * edge_weight(*g, node1, node2);  // :360
        cutSize -= gain;                                                               // :362
        if (cutSize < minCutSize) { minCutSize = cutSize; best_iter = iteration + 1; } // :363
        // swip (cKL.cpp:274-286)
        locked[node1] = locked[node2] = 1;
        --alive0; --alive1;
        side[node1] = 1;
        side[node2] = 0;
        // updateAffectedNodeGains (cKL.cpp:253-272): nodeConnections = row neighbours
        affected.clear();
        for (int32_t p = g->rowptr[node1]; p < g->rowptr[node1 + 1]; ++p) affected.push_back(uint32_t(g->col[p]));
        for (int32_t p = g->rowptr[node2]; p < g->rowptr[node2 + 1]; ++p) affected.push_back(uint32_t(g->col[p]));
        std::sort(affected.begin(), affected.end());
        affected.erase(std::unique(affected.begin(), affected.end()), affected.end());
#pragma omp parallel for schedule(dynamic, 8) if (affected.size() > 64)  // cKL.cpp:267
        for (size_t a = 0; a < affected.size(); ++a) gains[affected[a]] = connections(*g, side, affected[a]);
        iteration++;
        if (log && int64_t(iteration) <= cap)
            log[iteration - 1] = eko_swap{iteration, node1, node2, maxGain, minGain, gain, cutSize, 0};
        if (gain <= 0.0f) {  // cKL.cpp:382-386
            if (++terminate > terminateLimit) break;
        } else {
            terminate = 0;
        }
    }
    if (res) {
        res->iterations = iteration;
        res->initial_cut = initialCutSize;
        res->best_cut = minCutSize;
        res->final_cut = cutSize;
        res->best_iter = best_iter;
        res->net_cut_initial = eko_net_cut(g, side_init.data());
        res->net_cut_final = eko_net_cut(g, side.data());
        // replay the best prefix
        std::vector<uint8_t> sb = side_init;
        if (log && best_iter <= cap)
            for (int64_t i = 0; i < best_iter; ++i) { sb[log[i].node_left] = 1; sb[log[i].node_right] = 0; }
        res->net_cut_best = (log && best_iter <= cap) ? eko_net_cut(g, sb.data()) : -1;
    }
    return 0;
}

// shuffleSparceMatrix's random branch (cKL.cpp:176-192) with the
// std::random_device seed replaced by `seed`.
int eko_random_split(int64_t n, uint32_t seed, int32_t* order0, int32_t* order1) {
    std::vector<uint32_t> nodes(n);
    for (int64_t i = 0; i < n; ++i) nodes[i] = uint32_t(i);
    std::mt19937 gen(seed);
    std::shuffle(nodes.begin(), nodes.end(), gen);
    const int64_t mid = n / 2;
    for (int64_t i = 0; i < mid; ++i) order0[i] = int32_t(nodes[i]);
    for (int64_t i = mid; i < n; ++i) order1[i - mid] = int32_t(nodes[i]);
    return 0;
}

// Thread count of the oracle's OpenMP regions (the CPU baseline's core count).
void eko_set_threads(int t) { omp_set_num_threads(t > 0 ? t : 1); }
int eko_get_threads(void) { return omp_get_max_threads(); }

int eko_bucket_growth(int64_t nkeys, int64_t* out) {
    std::unordered_map<uint32_t, float> m;
    for (int64_t i = 0; i < nkeys; ++i) {
        m[uint32_t(i)] += 1.0f;
        out[i] = int64_t(m.bucket_count());
    }
    return 0;
}

}  // extern "C"
