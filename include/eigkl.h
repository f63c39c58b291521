/*
 * eigkl.h — C-ABI of libeigkl_hip.so, the MI355X (gfx950) EIG+KL hypergraph
 * bipartitioner.  Plain pointers and sizes only; no torch / HIP types.
 *
 * The reference (yhinai/EIG-KL-Algorithm) has no library or FFI: its seams
 * are (1) the process/CLI + file boundary of cEIG/cKL/gKL/gKL2,
 * (2) Spectra's MatOp `perform_op(x_in, y_out)` consumed by SymEigsSolver at
 * cEIG.cpp:194-198, (3) gKL's `gpuConnections(...)` gain seam at
 * gKL.cu:188-227 driven by the KL loop at cKL.cpp:334-390.  Each entry point
 * below names the reference interface it replaces.
 *
 * Conventions: every int-returning call returns EK_OK (0) or a negative
 * ek_status; ek_last_error() gives a thread-local message.  The library never
 * calls exit() (unlike CHECK_CUDA at gKL.cu:87-94).  A context is bound to
 * one GPU and is not thread-safe; use one host thread (or process) per GPU.
 * There is NO CPU fallback: GPU entry points fail with EK_EHIP when no
 * gfx950 device is usable.
 */
#ifndef EIGKL_H
#define EIGKL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum ek_status {
    EK_OK = 0,
    EK_EINVAL = -1,  /* bad argument / malformed input file */
    EK_EIO = -2,     /* file cannot be opened / written */
    EK_EHIP = -3,    /* HIP runtime error or no usable GPU */
    EK_ENOMEM = -4,
    EK_ENOCONV = -5, /* eigensolver did not converge ("Eigenvalue computation failed", cEIG.cpp:200-202) */
    EK_ESTATE = -6,  /* call out of order (e.g. ek_kl_run before ek_kl_graph_setup) */
    EK_ECOMM = -7    /* RCCL error */
};

const char* ek_last_error(void);
const char* ek_version(void);
/* The struct layouts of this header (ek_lanczos_opts / _stats, ek_solve_opts,
 * ek_swap ...) carry no size field; a binding checks ek_abi_version() ==
 * EIGKL_ABI_VERSION before passing any of them.  Bumped whenever a public
 * struct changes layout (4: reorth_thresh, the stats' projected_steps /
 * reprojected / ortho_max, and reorth 3 as the default). */
#define EIGKL_ABI_VERSION 4
int ek_abi_version(void);

/* ------------------------------------------------------------------ */
/* Hypergraph ingest (host, no GPU)                                     */
/* ------------------------------------------------------------------ */
typedef struct ek_hgr ek_hgr;

/* Read a .hgr file: header "nets nodes", then one line per net of 1-based
 * pins.  Replaces the per-executable readers cEIG.cpp:177-182,91-101 and
 * cKL.cpp:84-116 (same line semantics: exactly `nets` lines are read). */
int ek_hgr_read(const char* path, ek_hgr** out);
/* Seeded ISPD98-shaped synthetic circuit: floor(201920*mult) nodes,
 * floor(210613*mult) nets, net sizes {2:84,3:2,4:6,5:2,6:4,8:2}/100, distinct
 * sorted pins.  Replaces circuit_generator.py:41-59 (whose RNG is unseeded). */
int ek_hgr_generate(double multiplier, uint64_t seed, ek_hgr** out);
/* Build from 0-based pins: net e owns pins[net_ptr[e] .. net_ptr[e+1]). */
int ek_hgr_from_pins(int64_t nets, int64_t nodes, const int64_t* net_ptr, const int32_t* pins,
                     ek_hgr** out);
/* Largest connected component of the pin graph (nets with >= 2 pins join
 * their pins; the largest component, ties to the one holding the smallest
 * node id), as a new hypergraph: its nets in file order, nodes renumbered in
 * ascending original id.  node_map (nodes of h, may be NULL) gets the new id
 * or -1.  No reference counterpart: the connected ibm18-scale workload the
 * disconnected synthetic lacks (SURVEY §0 finding 8). */
int ek_hgr_largest_component(const ek_hgr* h, ek_hgr** out, int32_t* node_map);
/* Write in the reference .hgr text format (circuit_generator.py:61-68). */
int ek_hgr_write(const ek_hgr* h, const char* path);
int ek_hgr_dims(const ek_hgr* h, int64_t* nets, int64_t* nodes, int64_t* pins);
int ek_hgr_copy_pins(const ek_hgr* h, int64_t* net_ptr /* nets+1 */, int32_t* pins /* pins */);
void ek_hgr_free(ek_hgr* h);

/* ------------------------------------------------------------------ */
/* Clique expansions (host, no GPU)                                     */
/* ------------------------------------------------------------------ */
typedef struct ek_csr ek_csr;

/* fp64 clique Laplacian, -2/|e| per pin pair, diagonal = -(row sum); rows
 * with ascending columns, diagonal included.  Replaces initializeMatrix,
 * cEIG.cpp:86-133. */
int ek_laplacian_build(const ek_hgr* h, ek_csr** out);
/* Rows [row0, row0+nrows) only (global column ids): one rank's shard of the
 * sharded Lanczos, as ek_shard_rows assigns it. */
int ek_laplacian_build_rows(const ek_hgr* h, int64_t row0, int64_t nrows, ek_csr** out);
/* fp32 KL adjacency, w = 1/(|e|-1) accumulated in net order; each row holds
 * its forward (upper-triangle) entries in the iteration order of cKL's
 * std::unordered_map<uint32_t,float> (libstdc++ _Hashtable, emulated), then
 * its backward entries by ascending id — the exact summation order of
 * connections(), cKL.cpp:225-251.  Replaces InitializeSparsMatrix,
 * cKL.cpp:84-149. */
int ek_kl_graph_build(const ek_hgr* h, ek_csr** out);
/* nrows, nnz, value size in bytes (8 = fp64 Laplacian, 4 = fp32 KL graph). */
int ek_csr_dims(const ek_csr* c, int64_t* nrows, int64_t* nnz, int32_t* value_bytes);
/* Copy out: rowptr[nrows+1], col[nnz], val[nnz] (double* or float*),
 * nfwd[nrows] (KL graph: forward entries per row; may be NULL). */
int ek_csr_copy(const ek_csr* c, int32_t* rowptr, int32_t* col, void* val, int32_t* nfwd);
void ek_csr_free(ek_csr* c);

/* 1-D row-block partition for the sharded Lanczos: rank r owns
 * rows [row0, row0+nrows) with nrows <= nloc (equal padded blocks). */
int ek_shard_rows(int64_t n, int nranks, int rank, int64_t* row0, int64_t* nrows, int64_t* nloc);
/* The nnz-balanced partition (SURVEY §8e "1-D row block partition balanced
 * by nnz"), the one ek_spmv_setup_pins uses: rank r owns rows
 * [row_offsets[r], row_offsets[r+1]) (nranks + 1 offsets), cut where the
 * prefix of the Laplacian rows' entries (1 + sum over the row's nets of
 * |e| - 1: initializeMatrix's triplets, cEIG.cpp:86-133) reaches r/nranks of
 * the total.  Deterministic: every rank computes the same map.  No reference
 * counterpart (the reference has no multi-GPU path). */
int ek_shard_map(int64_t n, int64_t nets, const int64_t* net_ptr, const int32_t* pins, int nranks,
                 int64_t* row_offsets);

/* ------------------------------------------------------------------ */
/* GPU context                                                          */
/* ------------------------------------------------------------------ */
typedef struct ek_ctx ek_ctx;

int ek_init(int device, ek_ctx** out);
void ek_destroy(ek_ctx* ctx);
/* The context's hipStream_t (every kernel of this context runs on it). */
int ek_get_stream(ek_ctx* ctx, void** stream_out);
/* Wait for everything queued on the context's stream. */
int ek_synchronize(ek_ctx* ctx);
int ek_device_count(int* count);

/* RCCL over xGMI: one process per GPU.  Rank 0 calls ek_comm_unique_id and
 * ships the 128 bytes to the other ranks (e.g. torch.distributed broadcast). */
int ek_comm_unique_id(void* id128);
/* Resets the context's row ownership: call ek_spmv_setup afterwards. */
int ek_comm_init(ek_ctx* ctx, int nranks, int rank, const void* id128);
/* Host-staged exchange instead of RCCL (no reference counterpart; the
 * reference has no multi-GPU path).  Every collective of the sharded Lanczos
 * drains the context stream, copies its operand to pinned host memory, calls
 * the caller's collective and copies the result back.  Lets several ranks
 * share one GPU (RCCL refuses that) and lets any host transport (e.g.
 * torch.distributed gloo) drive the exchange: the multi-rank tests and
 * debugging.  RCCL (ek_comm_init) is the production path.  Callbacks return
 * 0 on success; recv holds nranks*count doubles, rank-major. */
typedef int (*ek_allgather_fn)(void* user, const double* send, int64_t count, double* recv);
typedef int (*ek_allreduce_fn)(void* user, double* buf, int64_t count); /* in-place sum */
int ek_comm_init_host(ek_ctx* ctx, int nranks, int rank, ek_allgather_fn allgather, ek_allreduce_fn allreduce,
                      void* user);

/* ------------------------------------------------------------------ */
/* SpMV seam: Spectra SparseSymMatProd<double>::perform_op, cEIG.cpp:194  */
/* ------------------------------------------------------------------ */
/* Upload the Laplacian rows this context owns.  n = global size; rowptr has
 * nrows+1 entries starting at 0; col holds global column ids.  Host arrays
 * are copied; the caller keeps ownership.  Sharded contexts: every rank
 * calls it; the ranks' [row0, row0+nrows) must tile [0, n) in rank order
 * (learned with one all-gather; ek_shard_map or ek_shard_rows). */
int ek_spmv_setup(ek_ctx* ctx, int64_t n, int64_t row0, int64_t nrows, const int32_t* rowptr,
                  const int32_t* col, const double* val);
/* The same rows built on the GPU straight from the hypergraph's pins (net e
 * owns pins[net_ptr[e] .. net_ptr[e+1]), 0-based): the clique Laplacian of
 * initializeMatrix (cEIG.cpp:86-133) assembled by device kernels into the
 * SpMV's coded form, the rows of this context's shard only (ek_shard_map).
 * The values and the row blocks are the host build's (ek_laplacian_build),
 * so every SpMV and Lanczos result is bit-identical to ek_spmv_setup on
 * those rows.  Falls back to the host build for a row too long for the
 * device sort (or with EK_HOST_LAPLACIAN set); *on_device (may be NULL)
 * tells which ran. */
int ek_spmv_setup_pins(ek_ctx* ctx, int64_t n, int64_t nets, const int64_t* net_ptr, const int32_t* pins,
                       int32_t* on_device);
/* The rows the context owns after the last ek_spmv_setup (any of the
 * pointers may be NULL). */
int ek_spmv_dims(ek_ctx* ctx, int64_t* n, int64_t* row0, int64_t* nrows);
/* y[0:nrows] = L[row0:row0+nrows, :] x.  x_dev: n doubles, y_dev: nrows
 * doubles, device pointers borrowed.  stream = hipStream_t or NULL (ctx
 * stream).  Asynchronous. */
int ek_spmv(ek_ctx* ctx, const double* x_dev, double* y_dev, void* stream);
/* Same with host buffers (x: n, y: nrows); synchronous. */
int ek_spmv_host(ek_ctx* ctx, const double* x, double* y);
/* Algorithmic (compulsory) bytes of one ek_spmv over the owned rows, SURVEY
 * §8d: 12*nnz (col+val) + 4*(nrows+1) (rowptr) + 8*n (x read once) +
 * 8*nrows (y).  Single GPU: 12 nnz + 4(n+1) + 16 n. */
int64_t ek_spmv_bytes(ek_ctx* ctx);
/* Storage form the SpMV reads (no reference counterpart; the reference keeps
 * an Eigen CSC of fp64 values, cEIG.cpp:49-50).  *packed = 1 when the entries
 * are dictionary-coded 32-bit words (column | code of the exact fp64 value in
 * a per-matrix table; bit-identical products), 0 for plain CSR (int32 col +
 * fp64 val; chosen when the distinct values overflow the code bits, or with
 * EK_SPMV_PLAIN=1 at setup).  *stored_bytes = bytes of one launch as stored:
 * entries + table + rowptr + 8*n (x) + 8*nrows (y).  Either pointer may be
 * NULL. */
int ek_spmv_format(ek_ctx* ctx, int32_t* packed, int64_t* stored_bytes);
/* The sharded step's exchange of f as set up: *halo = 1 when each rank
 * receives only the rows its columns read (point-to-point messages in one
 * RCCL group), 0 for the all-gather of whole slots; the doubles this rank
 * receives and sends per Lanczos step (each message carries the sender's
 * ||f||^2 partial).  A single context: 0, 0, 0.  No reference counterpart
 * (the reference has no sharded path). */
int ek_spmv_exchange(ek_ctx* ctx, int32_t* halo, int64_t* recv_doubles, int64_t* send_doubles);
/* The sharded Lanczos solves' exchange accounting since the last
 * ek_spmv_setup: exchanges of f (one per Lanczos step) and the point-to-point
 * messages this rank posted (halo form: ONE send and ONE receive per peer per
 * exchange, each message the rows the receiver reads closed by the sender's
 * ||f||^2 partial; host-staged: its pieces of the one all-gather).  With
 * ek_lanczos_opts::time_spmv set on a solve, that solve's collectives are
 * also timed: *exchange_ms over *exchanges_timed exchanges of f (RCCL: HIP
 * events around the send/recv group or all-gather on its stream, waits for
 * the peers included; host-staged: the host's view of the callback round
 * trip) and *allreduce_ms over *allreduces_timed all-reduces.  The timings
 * are reset by ek_spmv_setup and by a timed solve.  Any pointer may be NULL.
 * No reference counterpart (the reference has no sharded path). */
int ek_comm_stats(ek_ctx* ctx, int64_t* exchanges, int64_t* sends, int64_t* recvs, double* exchange_ms,
                  int64_t* exchanges_timed, double* allreduce_ms, int64_t* allreduces_timed);
/* Back-to-back SpMV launches on context-owned buffers, timed with HIP events
 * around the batch: *avg_us = average per launch (a sharded context: this
 * rank's rows over the all-gather layout, no collective).  fused = 2: also the
 * solve's folded finalize and ||w||^2 partials (the SpMV as the Lanczos step
 * launches it).  fused = 1 times the
 * Lanczos form (y scaled by 1/||x||, basis column + alpha partials written:
 * + 16*nrows bytes over ek_spmv_bytes).  Measurement helper for bench.py's
 * size sweep; no reference counterpart. */
int ek_spmv_bench(ek_ctx* ctx, int iters, int fused, double* avg_us);
/* The gather-only ceiling of the context's SpMV (a roofline
 * fraction read against its access pattern's own limit): back-to-back
 * launches of a kernel with the SpMV's grid that streams the same matrix words
 * (segments or column panels) and makes the same x and value-table gathers in
 * the same order, summing the products in registers: no row reduction, no y,
 * no epilogue.  *avg_us as in ek_spmv_bench.  No reference counterpart. */
int ek_spmv_gather_bench(ek_ctx* ctx, int iters, double* avg_us);

/* ------------------------------------------------------------------ */
/* Lanczos / Fiedler: Spectra SymEigsSolver(op, 2, min(100,n/2)),        */
/* compute(SmallestAlge), cEIG.cpp:194-207                               */
/* ------------------------------------------------------------------ */
typedef struct {
    int32_t ncv;        /* <= 0: min(80, n/2) under partial reorthogonalisation
                           (reorth 3, the default) below 1M rows, else
                           min(100, n/2) (cEIG.cpp:195) */
    int32_t maxit;      /* restarts; <= 0: 1000 (Spectra default) */
    double tol;         /* <= 0: 1e-10 (Spectra default) */
    int32_t deflate;    /* 1 (default): deflate the constant null vector, nev=1;
                           0: Spectra-equivalent nev=2, Fiedler = 2nd smallest */
    int32_t time_spmv;  /* 1: bracket every SpMV launch with HIP events (stats) */
    int32_t reorth;     /* 3 (default): partial reorthogonalisation — the three-term
                           recurrence, and the full classical Gram-Schmidt pass of 1
                           only on the steps Simon's omega recurrence asks for (loss of
                           orthogonality estimate > reorth_thresh), the step after each,
                           every cycle's first and last step (single context and
                           sharded alike; the sharded step all-reduces alpha and
                           ||w||^2 first).  CHANGED DEFAULT (EIGKL_ABI_VERSION 4): rounds 1-3
                           defaulted to 1.  1: that pass on every step (Spectra's
                           full reorthogonalisation, the reference's algorithm;
                           `--spectra` / `--reorth full` on the CLI); 2: CGS2 (twice)
                           from the matvec; 0: as 1 */
    int32_t check_every; /* after the first restart cycle, test Spectra's convergence
                            criterion on the projected matrix every this many steps
                            (and stop there) instead of at cycle ends only; 0: cycle
                            ends only (Spectra's schedule).  Default 8. */
    int32_t basis32;     /* 1 (default): the reorthogonalisation's update f = f' - V h reads
                            an fp32 shadow of the basis when sum|h| <= 2^-29 ||f'|| (its
                            effect then stays below fp64 rounding), else V;
                            0: always the fp64 basis.  Single-context steps only. */
    int32_t alpha_last;  /* 0 (default): every projection workgroup re-reduces the SpMV's
                            alpha = v_i . w partials; 1: the SpMV's last workgroup does
                            (a serial tail on the SpMV; the same bits) */
    int32_t keep_min;    /* implicit restarts keep at least this many vectors (floor on
                            Spectra's nev_adjusted, which on these Laplacians often keeps
                            2-4: DESIGN.md); < 0 (default): ncv / 5; 0: Spectra's rule */
    double reorth_thresh; /* reorth 3: project when the estimated |v_{i+1}^T v_j| exceeds
                             this; <= 0 (default): 1e-10 (Simon's
                             sqrt(DBL_EPSILON) lets the loss compound across implicit
                             restarts) */
} ek_lanczos_opts;

typedef struct {
    int32_t restarts;
    int32_t matvecs;
    int32_t converged;
    double residual;      /* ||L v - lambda v||_2 of the returned vector */
    double total_ms;      /* wall time of the solve */
    double spmv_ms;       /* sum of SpMV launch durations (time_spmv=1) */
    int32_t spmv_timed;   /* SpMV launches timed */
    double comm_ms;       /* time inside RCCL calls (host-observed, sharded) */
    int32_t allgathers;   /* collectives issued by this rank during the solve (sharded; */
    int32_t allreduces;   /* one of each per Lanczos step, plus restarts/injections/end) */
    int32_t update32_steps;     /* steps whose update was enqueued with the fp32 shadow */
    int32_t update32_fallbacks; /* ... of which took the fp64 basis (the accuracy test failed) */
    int32_t projected_steps;    /* steps that ran the Gram-Schmidt pass (= matvecs unless reorth 3) */
    int32_t reprojected;        /* sharded steps whose f' cancelled (||f'||^2 < 2^-20 ||w||^2) and
                                   whose next vector was projected again (a second CGS pass) */
    double ortho_max;           /* EK_LANCZOS_ORTHO=1: max |[V u0]^T [V u0] - I| at the restarts */
} ek_lanczos_stats;

void ek_lanczos_default_opts(ek_lanczos_opts* o);
/* Fiedler pair of the Laplacian given to ek_spmv_setup.  v_host_out: n
 * doubles (full vector on every rank when sharded).  Sign: the entry of
 * largest magnitude is made positive (cKL bit parity for odd n
 * may need ek_align_sign against the reference file). */
int ek_lanczos_fiedler(ek_ctx* ctx, const ek_lanczos_opts* o, double* lambda_out, double* v_host_out,
                       ek_lanczos_stats* stats);

/* ------------------------------------------------------------------ */
/* Median split + EIG file (cEIG.cpp:55-65, 209-220)                    */
/* ------------------------------------------------------------------ */
/* median (even n: mean of the two middle values), bits[i] = (median > v[i]). */
int ek_median_split(int64_t n, const double* v, double* median_out, uint8_t* bits_out);
/* Flip v if its dot product with ref is negative (--sign-ref). */
int ek_align_sign(int64_t n, double* v, const double* ref);
/* pre_saved_EIG/<base>_out.txt writer / reader (%.12g; cEIG.cpp:213-220,
 * read as cKL.cpp:155-174).  The reader returns remain[] lists in file order. */
int ek_eig_write(const char* path, int64_t n, double lambda, double median, const uint8_t* bits,
                 const double* v);
int ek_eig_read(const char* path, int64_t n, double* lambda, double* median, uint8_t* bits, double* v,
                int32_t* order0, int64_t* n0, int32_t* order1, int64_t* n1);

/* ------------------------------------------------------------------ */
/* KL: KL() cKL.cpp:288-406; GPU gain seam gpuConnections gKL.cu:188-227 */
/* ------------------------------------------------------------------ */
typedef struct {
    uint32_t iter;       /* 1-based (cKL.cpp:371) */
    uint32_t node_left;  /* node1: argmax gain over remain[0] (cKL.cpp:341-347) */
    uint32_t node_right; /* node2: argmin gain over remain[1] (cKL.cpp:349-355) */
    float max_gain, min_gain;
    float gain;          /* maxGain - minGain - 2 w(node1,node2) (cKL.cpp:360) */
    float cut;           /* running fp32 cut (cKL.cpp:362) */
    uint32_t pad;
} ek_swap;

typedef struct {
    int64_t iterations;
    float initial_cut, best_cut, final_cut;
    int64_t best_iter;   /* first iteration reaching best_cut (0 = initial) */
    int64_t net_cut_initial, net_cut_best, net_cut_final; /* integer hyperedge cuts */
    double loop_ms;      /* device time of the swap loop */
    double total_ms;     /* device time of gain scan + loop + cuts */
} ek_kl_result;

/* Upload the KL graph (from ek_kl_graph_build, or any rows in cKL order). */
int ek_kl_graph_setup(ek_ctx* ctx, int64_t n, const int32_t* rowptr, const int32_t* col, const float* w);
/* Upload the hypergraph pins (for the integer net cut). */
int ek_kl_nets_setup(ek_ctx* ctx, int64_t nets, const int64_t* net_ptr, const int32_t* pins);
/* Initial remain[] lists (shuffleSparceMatrix, cKL.cpp:151-197): positions
 * are list order; the sides are split[0] = order0, split[1] = order1. */
int ek_kl_set_partition(ek_ctx* ctx, const int32_t* order0, int64_t n0, const int32_t* order1, int64_t n1);
/* The random branch of shuffleSparceMatrix (cKL.cpp:176-192), host only:
 * nodes 0..n-1 shuffled by std::shuffle with std::mt19937(seed) (the
 * reference seeds it from std::random_device; the seed makes it
 * reproducible), the first n/2 to remain[0] (order0, n/2 entries), the rest
 * to remain[1] (order1, n - n/2 entries). */
int ek_random_split(int64_t n, uint32_t seed, int32_t* order0, int32_t* order1);
/* The -EIG branch of shuffleSparceMatrix (cKL.cpp:155-174): node i goes to
 * split[bits[i]] in ascending node order (the EIG file's line order). */
int ek_kl_set_partition_bits(ek_ctx* ctx, int64_t n, const uint8_t* bits);
/* The -EIG branch of ek_solve_file on the device: the median split of the
 * Fiedler vector the last ek_lanczos_fiedler on this context returned (kept
 * on the device, normalised and sign-fixed as v_out), with the remain[]
 * lists in node order — the lists ek_median_split + ek_kl_set_partition_bits
 * give on the host (cEIG.cpp:204-209 median, cKL.cpp:155-174 lists), without
 * the vector's round trip.  median_out, n0_out, n1_out may be null. */
int ek_kl_set_partition_fiedler(ek_ctx* ctx, double* median_out, int64_t* n0_out, int64_t* n1_out);
/* Run the swap loop to termination on the device (one persistent
 * workgroup; no host round trip per iteration).  limit < 0: floor(log2 n)+5
 * (cKL.cpp:303).  log_out may be NULL. */
int ek_kl_run(ek_ctx* ctx, int32_t limit, ek_swap* log_out, int64_t cap, ek_kl_result* res);
/* Side of every node: which = 0 initial, 1 best prefix, 2 final. */
int ek_kl_sides(ek_ctx* ctx, int32_t which, uint8_t* sides_out);

/* ------------------------------------------------------------------ */
/* Whole path, .hgr in -> results/ out, in-process: the body of          */
/* gKL2 <in> -EIG (GPU Fiedler split) and cKL/gKL <in> (random split),   */
/* main() + KL() of cKL.cpp:288-468 with cEIG.cpp:138-237 in front.      */
/* ------------------------------------------------------------------ */
typedef struct {
    int32_t eig;          /* 1: Fiedler split on the GPU (gKL2 -EIG); 0: random split (seed) */
    uint32_t seed;        /* random split: std::mt19937 seed (ek_random_split) */
    int32_t write_results;/* 1: results/<base>_KL_CutSize[_EIG]_output.txt under out_dir */
    int32_t limit;        /* KL termination limit; < 0: floor(log2 n)+5 (cKL.cpp:303) */
    const char* out_dir;  /* NULL: the CWD (the reference's convention) */
    const char* sign_ref; /* optional pre_saved_EIG file whose sign the Fiedler vector takes */
    ek_lanczos_opts lanczos;
} ek_solve_opts;

typedef struct {
    int64_t nets, nodes, pins;
    double lambda, median;
    ek_lanczos_stats lanczos; /* eig = 1 */
    ek_kl_result kl;          /* rank 0 only */
    /* wall seconds of the phases on this rank (host clock); t_lanczos
     * includes t_spmv_setup (the rows' coding and upload) */
    double t_read, t_laplacian, t_lanczos, t_split, t_kl_graph_wait, t_kl_setup, t_kl, t_write, t_total;
    double t_spmv_setup;
} ek_solve_result;

void ek_solve_default_opts(ek_solve_opts* o);
/* Multi-rank contexts (ek_comm_init*): every rank calls it with the same
 * file; the Lanczos rows are sharded (each rank builds and uploads its own
 * rows), the KL loop and the results file are rank 0's.  log_out (may be
 * NULL, cap entries) receives rank 0's swap log. */
int ek_solve_file(ek_ctx* ctx, const char* path, const ek_solve_opts* o, ek_swap* log_out, int64_t cap,
                  ek_solve_result* res);

/* ------------------------------------------------------------------ */
/* Drop-in CLIs: argv exactly as cEIG.cpp:138-237 / cKL.cpp:424-468 /    */
/* gKL.cu:672-713 / gKL2.cu:989-1033, outputs relative to the CWD.       */
/* tool = "cEIG" | "cKL" | "gKL" | "gKL2".  Returns the process exit code. */
/* ------------------------------------------------------------------ */
int ek_cli_main(const char* tool, int argc, char** argv);
/* As ek_cli_main.  flags & EK_CLI_NO_TEARDOWN: the GPU context is not
 * destroyed on return (every output is written and every stream drained
 * first); for an executable that then ends with _exit, leaving the context
 * to the process exit instead of the runtime's orderly teardown. */
#define EK_CLI_NO_TEARDOWN 1
int ek_cli_main_ex(const char* tool, int argc, char** argv, int flags);

#ifdef __cplusplus
}
#endif
#endif /* EIGKL_H */
