/* ORACLE — test infrastructure only (see oracle/eko_kl.cpp header).
 *
 * C interface of liboracle (oracle/build/libekoracle.so), loaded through ctypes
 * by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only.
 * The product (libeigkl_hip.so, the cEIG/cKL/gKL/gKL2 CLIs) never links it.
 */
#ifndef EKO_H
#define EKO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct eko_graph eko_graph;

/* One KL swap exactly as cKL.cpp:357-380 computes it. */
typedef struct {
    uint32_t iter;      /* 1-based iteration (cKL.cpp:371) */
    uint32_t node_left; /* node1 = argmax over remain[0] (cKL.cpp:341-347) */
    uint32_t node_right;/* node2 = argmin over remain[1] (cKL.cpp:349-355) */
    float max_gain;     /* nodeGains[node1] */
    float min_gain;     /* nodeGains[node2] */
    float gain;         /* maxGain - minGain - 2*w(node1,node2) (cKL.cpp:360) */
    float cut;          /* running fp32 cut after the swap (cKL.cpp:362) */
    uint32_t pad;
} eko_swap;

typedef struct {
    int64_t iterations;
    float initial_cut; /* fp32(fp64 sum of per-node fp32 external weights), see DESIGN.md */
    float best_cut;    /* running minimum, first occurrence (cKL.cpp:363) */
    float final_cut;
    int64_t best_iter; /* iteration at which best_cut was first reached (0 = initial) */
    int64_t net_cut_initial, net_cut_best, net_cut_final; /* integer hyperedge cuts */
} eko_kl_result;

/* .hgr read (cKL.cpp:84-116) or explicit pins (0-based). Builds cKL's
 * upper-triangle unordered_map adjacency (cKL.cpp:107-131) and keeps the pins. */
int eko_read(const char* path, eko_graph** out);
int eko_from_pins(int64_t nets, int64_t nodes, const int64_t* net_ptr, const int32_t* pins,
                  eko_graph** out);
void eko_free(eko_graph* g);
int64_t eko_nodes(const eko_graph* g);
int64_t eko_nets(const eko_graph* g);

/* KL adjacency in cKL summation order: per row, forward keys in the REAL
 * libstdc++ unordered_map iteration order, then backward neighbours ascending
 * (cKL.cpp:229-248).  Null arrays -> returns nnz only. */
int64_t eko_kl_csr(const eko_graph* g, int32_t* rowptr, int32_t* col, float* w, int32_t* nfwd);

/* cKL KL() with the given initial remain[] lists (positions = list order). */
int eko_kl(const eko_graph* g, const int32_t* order0, int64_t n0, const int32_t* order1, int64_t n1,
           int32_t limit, eko_swap* log, int64_t cap, eko_kl_result* res);

/* Integer hyperedge cut of a side assignment (nets with pins on both sides). */
int64_t eko_net_cut(const eko_graph* g, const uint8_t* side);

/* Clique Laplacian (cEIG.cpp:86-133) as CSR with ascending columns. */
int64_t eko_laplacian(const eko_graph* g, int32_t* rowptr, int32_t* col, double* val);
void eko_spmv(const eko_graph* g, const double* x, double* y);

/* CPU fp64 thick-restart Lanczos for the Fiedler pair (restates Spectra
 * SymEigsSolver(nev=2, ncv, SmallestAlge) as called at cEIG.cpp:194-207). */
typedef struct {
    int32_t ncv;      /* <=0: min(100, n/2) as cEIG.cpp:195 */
    int32_t maxit;    /* restarts, Spectra default 1000 */
    double tol;       /* Spectra default 1e-10 */
    int32_t deflate;  /* 1: deflate the constant null vector and solve nev=1 */
    int32_t max_matvec; /* >0: stop after this many matvecs (bounded CPU baseline) */
} eko_lanczos_opts;
typedef struct {
    int32_t restarts, matvecs, converged;
    double residual; /* ||L v - lambda v|| */
} eko_lanczos_stats;
int eko_lanczos(const eko_graph* g, const eko_lanczos_opts* o, double* lambda, double* v,
                eko_lanczos_stats* st);

/* cKL.cpp:176-192 (random init) with std::mt19937(seed) instead of random_device. */
int eko_random_split(int64_t n, uint32_t seed, int32_t* order0, int32_t* order1);
/* OpenMP threads of the restatement (the KL gain sweep/update/selection and
 * the Lanczos SpMV/projections run on them; results do not depend on it). */
void eko_set_threads(int t);
int eko_get_threads(void);

/* libstdc++ bucket-count growth observed on THIS host's std::unordered_map:
 * fills out[i] = bucket_count() after inserting i+1 distinct keys. */
int eko_bucket_growth(int64_t nkeys, int64_t* out);

#ifdef __cplusplus
}
#endif
#endif
