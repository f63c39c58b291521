// Internal declarations shared by the host (.cpp) and device (.hip) units of
// libeigkl_hip.so.  Public surface: include/eigkl.h.
#pragma once

#include <cstdint>
#include <cstdio>
#include <functional>
#include <memory>
#include <utility>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/eigkl.h"

// ---------------------------------------------------------------------------
// error plumbing: every C-ABI entry returns a status and sets a thread-local
// message; nothing calls exit().
namespace ek {
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
struct Error {
    int code;
};
[[noreturn]] void fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int guard_exceptions();  // maps the in-flight exception to a status (call from catch(...))

// bounded host parallelism (std::thread); EK_THREADS or OMP_NUM_THREADS caps it,
// and a ThreadCap on the calling thread lowers it for the work that thread starts
int host_threads();
struct ThreadCap {
    explicit ThreadCap(int cap);
    ~ThreadCap();
    int prev;
};
// EK_TRACE=1: host phase timings on stderr ("[tag] what ms")
struct PhaseTimer {
    explicit PhaseTimer(const char* tag);
    void mark(const char* what);
    const char* tag;
    double t0;
    bool on;
};
void cold_stamp(const char* what);  // EK_COLD_TRACE: epoch-time stamp of a start-up event
template <class F>
void parallel_for(int64_t n, F&& fn);  // fn(begin, end)
template <class F>
void run_threads(int T, F&& fn);  // fn(t) for t < T, t = 0 on the calling thread
// fn(ctx, t) for t < T on a persistent worker pool (t = 0 on the caller);
// spawned threads when another caller holds the pool
void pool_run(int T, void (*fn)(void*, int), void* ctx);
}  // namespace ek

#define EK_TRY try {
#define EK_CATCH \
    }            \
    catch (...) { return ek::guard_exceptions(); }

// ---------------------------------------------------------------------------
// host objects.  Large arrays use dvec: std::vector whose resize leaves new
// elements default-initialised (not zeroed), so the threads that fill them
// also first-touch their pages instead of one thread zeroing them first.
namespace ek {
template <class T>
struct default_init_allocator : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = default_init_allocator<U>;
    };
    default_init_allocator() = default;
    template <class U>
    default_init_allocator(const default_init_allocator<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
template <class T>
using dvec = std::vector<T, default_init_allocator<T>>;
}  // namespace ek

struct ek_hgr {
    int64_t nets = 0, nodes = 0;
    ek::dvec<int64_t> net_ptr;  // nets + 1
    ek::dvec<int32_t> pins;     // 0-based
    // sum over nets of k (k - 1), k >= 2 pins (the clique expansion's raw
    // entries), when the reader counted it; -1: not known
    int64_t raw_pairs = -1;
};
namespace ek {
// ek_spmv_setup_pins for an ek_hgr (ctx.cpp): its pins need no range scan
int spmv_setup_hgr(ek_ctx* c, const ek_hgr& h, int32_t* on_device);
}  // namespace ek

struct ek_csr {
    int64_t nrows = 0;
    int32_t value_bytes = 8;
    ek::dvec<int32_t> rowptr, col, nfwd;
    ek::dvec<double> val64;
    ek::dvec<float> val32;
};

namespace ek {
// graph_build.cpp
void build_laplacian(const ek_hgr& h, ek_csr& out);
void build_laplacian_rows(const ek_hgr& h, int64_t r0, int64_t r1, ek_csr& out);  // rows [r0, r1), global cols
void build_kl_graph(const ek_hgr& h, ek_csr& out);
// libstdc++ unordered_map<uint32_t,...> iteration order for keys inserted
// (first insertion) in the given order; writes the iteration order to out.
void hashtable_order(const uint32_t* keys, int64_t cnt, uint32_t* out, std::vector<int32_t>& scratch);
void hashtable_order(const uint32_t* keys, int64_t cnt, uint32_t* out, std::vector<int32_t>& scratch,
                     std::vector<int32_t>& bk0, std::vector<int32_t>& bk1);
void hashtable_order_index(const uint32_t* keys, int64_t cnt, int32_t* out_idx, std::vector<int32_t>& scratch,
                           std::vector<int32_t>& bk0, std::vector<int32_t>& bk1);  // (reused bucket arrays)
uint64_t hashtable_next_buckets(uint64_t cur);  // bucket count after the rehash that follows `cur`

// host_linalg.cpp — small dense/tridiagonal kernels for the IRL driver
// eigenvalues (ascending) of the symmetric tridiagonal (d, e), e[i] = T(i+1,i);
// zlast[j] = last component of eigenvector j; full Z (m x m col-major) if Z != null.
bool tridiag_eig(int m, const double* d, const double* e, double* evals, double* zlast, double* Z);
// The k smallest eigenvalues (ascending, bisection on Sturm counts to full
// precision) and the last component of each unit eigenvector (inverse
// iteration): what the Lanczos driver's mid-cycle convergence test reads, in
// O(k m log) instead of tridiag_eig's O(m^2) QL sweeps.  False if the
// iteration did not settle.
bool tridiag_smallest(int m, const double* d, const double* e, int k, double* evals, double* zlast);
// one implicit symmetric QR step with shift mu on (d, e); the rotations of
// its Q factor appended to rots in order: {p, c, s} is Q <- Q G_p, i.e.
// Q[i][p], Q[i][p+1] <- c a + s b, -s a + c b (a, b their old values)
struct QRot {
    int32_t p;
    double c, s;
};
void tridiag_qr_shift(int m, double* d, double* e, double mu, std::vector<QRot>& rots);
// tridiag_qr_shift with mus[0], ..., mus[ns-1] in turn (the same bits and
// rotations, in the same order), two consecutive chases interleaved
void tridiag_qr_shifts(int m, double* d, double* e, const double* mus, int ns, std::vector<QRot>& rots);
// columns [0, kk) of Q = I G_1 ... G_R (rots in order) into Qcm (col-major
// m x kk); X is scratch
void accumulate_q(int m, const std::vector<QRot>& rots, int kk, double* Qcm, std::vector<double>& X);
}  // namespace ek

// ---------------------------------------------------------------------------
// the in-process pipeline (solve.cpp) and the context's rank (ctx.cpp)
namespace ek {
void ctx_ranks(ek_ctx* ctx, int* rank, int* nranks);
// get_ctx is called when the GPU is first needed (the CLI initialises it on
// a helper thread meanwhile); rank / nranks are the context's.
void solve(const std::function<ek_ctx*()>& get_ctx, int rank, int nranks, const ek_hgr& h, const std::string& base,
           const ek_solve_opts& o, ek_swap* log_out, int64_t cap, ek_solve_result& r);
void fiedler_vector(ek_ctx* ctx, int rank, int nranks, const ek_hgr& h, const ek_solve_opts& o, double& lambda,
                    std::vector<double>& v, ek_lanczos_stats& st, double* t_laplacian, double* t_lanczos,
                    const std::function<void()>& after_laplacian = {}, double* t_spmv_setup = nullptr,
                    bool host_v = true);
}  // namespace ek

// ---------------------------------------------------------------------------
// device-side launchers (kernels_*.hip).  All asynchronous on `stream`.
typedef struct ihipStream_t* hipStream_t;

namespace ek {
namespace dev {

typedef struct ihipEvent_t* hipEvent_t;

// The finalize of Lanczos step `step`, folded into the next step's first
// kernel (k_finalize_step's a3 form): fn2_out = sum(npart[0:nb]) — every
// block sums the same partials in the same order — and block 0 publishes
// fn2_out, alpha[step] = *a3 + h2[step], offd[step] = beta_step + h2[step-1]
// with beta_step = *bov_i unless NaN, else sqrt(*fn2_i).  npart == null: none.
constexpr int MAX_HALO_RANKS = 16;  // ranks of the halo exchange (ctx.cpp halo_build); more: the full all-gather
struct StepFin {
    const double* npart = nullptr;
    int nb = 0;
    double* fn2_out = nullptr;
    const double* h2 = nullptr;
    int step = -1;
    double* alpha = nullptr;
    double* offd = nullptr;
    const double* a3 = nullptr;
    const double* fn2_i = nullptr;
    const double* bov_i = nullptr;
    int nstride = 1;  // npart[k * nstride], k < nb (the sharded step: each rank's ||f||^2 in its all-gather slot)
    // the halo layout: rank k's partial at npart[nidx[k]] (its block end in
    // the compact x, where the peer's one message put it); null: nstride
    const int* nidx = nullptr;
    // ||f||^2 from the update (||f'||^2 - ||h||^2, k_update B32) when not
    // NaN; NaN: summed from npart
    const double* fast = nullptr;
    // partial reorthogonalisation: the block's partial of ||w||^2 (w = the
    // scaled product) beside its alpha partial, for k_pro's estimate of
    // beta_{i+1}.  Read whether or not npart is set.
    double* wpart = nullptr;
    // the sharded step's halo SpMV (overlapped with the all-gather): entries
    // whose column lies in [own_lo, own_hi) (the rank's own slot, summed by
    // the owned-slot SpMV beforehand) contribute 0, and every row's sum starts
    // from ybase[row] (that SpMV's unscaled partial); own_lo == own_hi: none
    int own_lo = 0, own_hi = 0;
    const double* ybase = nullptr;
    // the update inside the projection launch (ctx.cpp, PROI merged): the
    // fp32 shadow of the basis column (fl32(v), written with v) and the
    // projection's decision words + done counter, zeroed by block 0
    float* v32col = nullptr;
    unsigned* pub_rearm = nullptr;
    // the Lanczos mid-cycle check's copy, folded into the chunk's last SpMV
    // (ctx.cpp chk_poll): block 0, once its finalize has published, copies
    // alpha / offd [0, chk_b) and fn2 [0, chk_b) into the pinned slot chk_dst
    // (alpha at 0, offd at chk_m, fn2 at 2 chk_m), releases them to the
    // system and stores chk_seq to *chk_word, which the host polls
    double* chk_dst = nullptr;
    unsigned* chk_word = nullptr;
    const double* chk_fn2 = nullptr;  // the fn2 array (fn2_out points at its entry `step + 1`)
    // the sequence number to store, read at run time from pinned host memory
    // the host sets before the launch (a captured graph replays the pointer)
    const unsigned* chk_seq_src = nullptr;
    int chk_b = 0, chk_m = 0;
};

// kernels_spmv.hip — CSR-adaptive fp64 SpMV (row blocks precomputed on host)
constexpr int SPMV_THREADS = 256;
std::vector<int32_t> spmv_row_blocks(const int32_t* rowptr, int64_t nrows, int block_nnz);
// y[r] = scale * sum_c L[r,c] x[c]; scale = 1/sqrt(*fn2) when fn2 != null else 1.
// If vcol != null also writes vcol[r] = f[r] * scale (Lanczos basis column), and
// if apart != null the per-block partials of vcol . y (one per block).
// desc: 4 ints per block {row0, nrows, nnz0, cnt} from spmv_row_blocks.
// fin: the previous step's finalize folded in (then ||f||^2 comes from it, not *fn2).
// ev_start/ev_stop: kernel start/end timestamps (hipExtLaunchKernelGGL), optional.
//
// Column-panel form (kernels_panel.hip) for an x larger than an XCD's L2
// share: G persistent workgroups over equal-nnz row ranges (<= PANEL_MAX_ROWS
// rows each), the entries bucketed by (workgroup, panel of 2^pb columns):
// bucket (w, p) = [start[w*P + p], start[w*P + p + 1]), each entry a word
// (code << pb) | column-in-panel and a row index relative to wrow[w].
constexpr int MAX_PANELS = 64;
constexpr int PANEL_MAX_ROWS = 8192;
constexpr int PANEL_LDS_DICT = 2048;  // value-table entries the panel SpMV keeps in LDS
struct SpmvPanel {
    int G = 0, P = 0, pb = 0, max_rows = 0, ndict = 0;
    const int32_t* wrow = nullptr;   // G + 1
    const long long* start = nullptr;  // G * P + 1
    const uint32_t* word = nullptr;
    const uint16_t* rid = nullptr;
};
size_t panel_lds_bytes(int max_rows, int ndict);
void panel_count(hipStream_t s, int G, const int32_t* rowptr, const uint32_t* pk, int colbits, const int32_t* wrow,
                 int pb, int P, int* cnt);
void panel_fill(hipStream_t s, int G, const int32_t* rowptr, const uint32_t* pk, int colbits, const int32_t* wrow,
                int pb, int P, const long long* start, uint32_t* word, uint16_t* rid);
void spmv_panel(hipStream_t s, const SpmvPanel& m, const double* dict, const double* x, double* y, const double* fn2,
                const double* f, double* vcol, double* apart, const StepFin* fin, hipEvent_t ev_start,
                hipEvent_t ev_stop, double* alpha_out, unsigned* actr);
// the panel form's gather-only ceiling (kernels_panel.hip; ek_spmv_gather_bench)
void panel_gather_only(hipStream_t s, const SpmvPanel& m, const double* dict, const double* x, double* sink);
// host: the workgroup row ranges (equal nnz, <= PANEL_MAX_ROWS rows each)
std::vector<int32_t> panel_row_ranges(const int32_t* rowptr, int64_t nrows, int target_groups);
// pk[e] = (code << colbits) | col[e] from the device build's value table
void encode_words(hipStream_t s, long long nnz, const int* col, const double* val, const unsigned long long* table,
                  int tsize, const long long* code_of_slot, int colbits, uint32_t* pk);
// Matrix storage: plain CSR (col int32 + val fp64, 12 B per entry) or the
// value-dictionary form (pk != null): one 32-bit word per entry,
// (code << colbits) | col, with val = dict[code].  A clique Laplacian holds few
// distinct values (-2/|e| sums and the row sums: 840 at ibm18 shape, 4,890 in
// ibm01), so the exact fp64 values come back from a table of a few KB that
// stays in L1/L2, and each entry streams 4 B instead of 12.  Same products,
// same summation order: results are bit-identical to the plain form.
struct SpmvMat {
    int nblocks = 0, block_nnz = 512, colbits = 0;
    bool has_long = true;  // some block is one row longer than block_nnz (vector mode); false: that code is compiled out
    const int32_t* desc = nullptr;
    const int32_t* rowptr = nullptr;
    const int32_t* col = nullptr;
    const double* val = nullptr;
    const uint32_t* pk = nullptr;  // per-block segments of the coded words (spmv_segment)
    const uint16_t* rel = nullptr;  // row starts inside each segment
    const double* dict = nullptr;
    SpmvPanel panel;  // panel.G > 0: the column-panel form (pk/rel/col/val unused)
};
#ifndef EK_SPMV_SEG
#define EK_SPMV_SEG 768
#endif
constexpr int SPMV_SEG_NNZ = EK_SPMV_SEG;  // block_nnz (segment size) of the coded form (a multiple of 256)
constexpr int SPMV_REL_STRIDE = 258;  // rel entries per block (nrows + 1 <= 257, padded)
// dictionary coding of (col, val): false (pk untouched) when the distinct
// values do not fit the 32 - colbits code bits.  dict is ordered by frequency.
bool spmv_pack(int64_t n, int64_t nnz, const int32_t* col, const double* val, std::vector<uint32_t>& pk,
               std::vector<double>& dict, int& colbits);
// desc (from spmv_row_blocks with SPMV_SEG_NNZ) is updated for long rows.
void spmv_segment(std::vector<int32_t>& desc, const int32_t* rowptr, const std::vector<uint32_t>& pk, int seg_nnz,
                  std::vector<uint32_t>& seg, std::vector<uint16_t>& rel);
constexpr int ALPHA_SUB = 32;  // first-level counters of the SpMV's last-block hand-off (64 uints apart)
// alpha_out (with apart): the last block to finish also reduces every block's
// alpha partial (k_three_term's order and bits) into *alpha_out; actr: a
// device counter, zero before the first such launch (re-armed by each)
// the gather-only ceiling of either form: its grid, matrix stream and x /
// value gathers with nothing else (ek_spmv_gather_bench); sink: never written
// in practice (>= one double per workgroup)
void spmv_gather_only(hipStream_t s, const SpmvMat& m, const double* x, double* sink);
// (lab) the skipped step's SpMV + update as two launches (mode 1) or one grid
// with an in-launch wait (mode 2; needs nblocks <= lab_step_capacity()), or the
// update alone (mode 3): ek_spmv_gather_bench's EK_GATHER_MODE
int lab_step_capacity();
void lab_gather_step(hipStream_t s, const SpmvMat& m, int mode, const double* x, double* part, unsigned* ctr,
                     unsigned target, int n, const double* w, const double* v, const double* u, double* f,
                     double* fpart);
void spmv(hipStream_t s, const SpmvMat& m, const double* x, double* y, const double* fn2, const double* f,
          double* vcol, double* apart, const StepFin* fin = nullptr, hipEvent_t ev_start = nullptr,
          hipEvent_t ev_stop = nullptr, double* alpha_out = nullptr, unsigned* actr = nullptr);

// kernels_build.hip — the Laplacian rows built on the device from the pins
struct LapBuild {
    long long nets = 0, r0 = 0, r1 = 0;  // rows [r0, r1) of the global matrix
    const int64_t* net_ptr = nullptr;
    const int32_t* pins = nullptr;
    int *icnt = nullptr, *rcnt = nullptr, *cur = nullptr;  // per row: incidences, raw entries, fill cursor
    long long *ip = nullptr, *rp = nullptr;                // their exclusive scans (nr + 1)
    int32_t* inc = nullptr;                                // (net, position in net) pairs, by row
    int* scol = nullptr;                                   // raw entries of each row at rp[i]
    double *sval = nullptr, *tval = nullptr;
    int *ulen = nullptr, *len = nullptr;  // merged entries; final row length (+ the diagonal if absent)
    double* diag = nullptr;
    int* long_rows = nullptr;  // rows past the per-thread sort
    int* counters = nullptr;   // [0] long rows, [1] rows too long for the LDS sort
};
// out[0..n] = exclusive scan of in[0..n) (out[n] = total); tiles: ceil(n/1024) scratch
void exclusive_scan(hipStream_t s, const int* in, long long n, long long* out, long long* tiles);
void lap_count(hipStream_t s, const LapBuild& b);
void lap_fill_rows(hipStream_t s, const LapBuild& b);
void lap_long_rows(hipStream_t s, const LapBuild& b, int n_long);
void lap_write(hipStream_t s, const LapBuild& b, const long long* off, int* rowptr, int* col, double* val);
// value dictionary: table[tsize] (power of two) of the distinct fp64 bit
// patterns; code_of_slot[tsize] = the number of distinct values
void dict_build(hipStream_t s, long long nnz, const double* val, unsigned long long* table, int tsize, int* overflow,
                int* flags, long long* code_of_slot, long long* tiles);
void dict_values(hipStream_t s, const unsigned long long* table, int tsize, const long long* code_of_slot,
                 double* dict);
void encode_segments(hipStream_t s, int nblocks, const int32_t* desc, const int* rowptr, const int* col,
                     const double* val, const unsigned long long* table, int tsize, const long long* code_of_slot,
                     int colbits, uint32_t* seg, uint16_t* rel);

// col[p] (global ids) -> r * slot + (col - off[r]) for the owner r of col
// (off: nranks + 1 row offsets of the shard map): the all-gather slot layout
void remap_cols(hipStream_t s, long long nnz, int* col, const long long* off, int nranks, long long slot);
// the entries of each of nr local rows whose column lies in [lo, hi), with
// columns rebased to col - lo: a first call with ocol == null counts them
// (cnt: nr ints, off: nr + 1, tiles: scan scratch) and returns the total;
// a second call with the output arrays (orp: nr + 1) fills them
long long own_split(hipStream_t s, long long nr, const int* rowptr, const int* col, const double* val, int lo, int hi,
                    int* cnt, long long* off, long long* tiles, int* orp, int* ocol, double* oval);
// the halo exchange (ctx.cpp halo_build): sbuf[t] = f[sidx[t]] for t <
// nsend, the rank's own block X[base + k] = f[k] (k < nrows), and its
// ||f||^2 partial P[0] = f[ldv]
void halo_pack(hipStream_t s, const double* f, int ldv, const int* sidx, long long nsend, double* sbuf, double* X,
               long long base, long long nrows, double* P);
// X[t] = x[gidx[t]], 0.0 where gidx[t] < 0
void gather_idx(hipStream_t s, const double* x, const int* gidx, long long len, double* X);

// The memory order of the counter adds that pick the last workgroup of an
// in-launch hand-off (kernels_spmv/lanczos/panel.hip).  The partials travel
// as agent-scope atomic stores and loads (sc1: performed at the memory side,
// past the per-XCD L2s, so coherent across XCDs by themselves); each block's
// thread 0 waits for its own partial stores (s_waitcnt vmcnt(0)) before its
// relaxed counter add, and the last block issues its partial loads after the
// add returned.  EK_HANDOFF_ACQREL: acquire-release adds, the memory model's
// formal guarantee — on gfx950 an agent-scope release is a buffer_wbl2 (a
// write-back of the XCD's whole L2) in every workgroup: measured 27.6 ->
// 54.3 ms per resident Lanczos solve at the headline (tools/pro_ab.py,
// reorth 1), so it stays an A/B build.
#ifdef EK_HANDOFF_ACQREL
#define EK_HANDOFF_ORDER __ATOMIC_ACQ_REL
#else
#define EK_HANDOFF_ORDER __ATOMIC_RELAXED
#endif

// kernels_lanczos.hip
#ifndef EK_GT_ROWS
#define EK_GT_ROWS 1024
#endif
constexpr int GT_ROWS = EK_GT_ROWS;  // rows per gemv-T block; ldv is a multiple of this
constexpr int GT_COLS = 8;     // basis columns per gemv-T block (16: 18.9 vs 16.6 us, 204 VGPRs)
constexpr int UPD_ROWS = 512;  // rows per update block
constexpr int MAX_NCV = 128;
// part[j*nrb + b] = sum_{rows of block b} V[row, j] * w[row]; column `ncols` is
// the implicit deflation vector u0 (value u0val on rows < nreal) if has_u0.
// nrm: part column ncols + has_u0 also gets ||w||^2 over each row block
// (the fp32-shadow update's accuracy test, k_update B32)
// nt: the basis is read non-temporally (a basis larger than the MALL)
// gctr / h_out (nrb <= 256): the column sums are also reduced in the launch
// (the last workgroup of each column group; col_sum2's order) into h_out;
// gctr: GT_HANDOFF_UINTS zeroed uints, re-armed by each launch (the last
// 9 x 64: the in-launch decision form's own hand-off of the ||f'||^2 column)
constexpr int GT_NORM_CTR = ((MAX_NCV + 2 + GT_COLS - 1) / GT_COLS) * 9 * 64;
constexpr int GT_HANDOFF_UINTS = GT_NORM_CTR + 9 * 64;
void gemvt(hipStream_t s, int ldv, int nrb, const double* V, int ncols, int has_u0, double u0val,
           int nreal, const double* w, double* part, int nrm = 0, unsigned* gctr = nullptr, double* h_out = nullptr,
           bool nt = false);
// the sharded step (ctx.cpp factorize_mr): part for three vectors w, va, vb at
// once, part[(k*tot + j)*nrb + b], tot = ncols + has_u0, and ||w||^2 partials
// at part[3*tot*nrb + b]
void gemvt3(hipStream_t s, int ldv, int nrb, const double* V, int ncols, int has_u0, double u0val, int nreal,
            const double* w, const double* va, const double* vb, double* part);
// hall = the all-reduced column sums of gemvt3 (3 x tot): alpha = hall[i],
// h = hall[0:tot] - alpha hall[tot:2tot] - beta hall[2tot:3tot] (i = ncols-1),
// dst = w - alpha vi - beta vim1 - V h - u0 h[ncols] (+ ||dst||^2 partials);
// block 0 writes alpha[i] = alpha + h[i] and offd[i] = beta_i + h[i-1], and
// cflag[i] = 1.0 when ||f'||^2 < cancel ||w||^2 (hall[3*tot] = ||w||^2).
// beta = sqrt(*fn2_i) unless the override *bov_i is not NaN; vim1 null: 0.
void update_mr(hipStream_t s, int ldv, const double* V, int ncols, int has_u0, double u0val, int nreal,
               const double* hall, const double* w, const double* vi, const double* vim1, const double* fn2_i,
               const double* bov_i, double* dst, double* npart, double* alpha, double* offd, double* cflag,
               double cancel);
// gemvt of the three-term residual f' = w - *alpha vi - beta_i vim1 (vim1 may
// be null; beta_i as three_term), formed per row; f' is also stored to fp.
// v32col != null: the fp32 basis shadow's column i = fl32(vi) is written and
// ||f'||^2 partials go to part column ncols + has_u0 (as gemvt's nrm).
// apart != null: alpha is not read from *alpha but reduced by every workgroup
// from the SpMV's nparts partials (k_three_term's order), and *alpha written
void gemvt_tt(hipStream_t s, int ldv, int nrb, const double* V, int ncols, int has_u0, double u0val, int nreal,
              const double* w, const double* alpha, const double* vi, const double* vim1, const double* fn2_i,
              const double* bov_i, double* fp, double* part, float* v32col = nullptr, const double* apart = nullptr,
              int nparts = 0, unsigned* gctr = nullptr, double* h_out = nullptr, bool nt = false,
              const int* flag = nullptr, double* fn2_fast = nullptr, const struct ProLaunch* pl = nullptr);
// h[j] = sum_b part[j*nrb + b]  for j < ncols_total
void reduce_cols(hipStream_t s, const double* part, int nrb, int ncols_total, double* h);

// Fused single-GPU step (reorth 1):
// update_r: h = column sums of part (every block, fixed order; block 0 writes
// h_out), then dst = src - V h - u0 h[ncols] with ||dst||^2 partials -> npart
// V32 != null: the basis is read from its fp32 shadow when sum|h| <= 2^-29
// ||src|| (exact to fp64 rounding; ||src||^2 is the partials' / h's entry
// after u0's), else from V (*fb += 1 when fb != null)
void update_r(hipStream_t s, int ldv, const double* V, int ncols, int has_u0, double u0val, int nreal,
              const double* part, int nrb, double* h_out, const double* src, double* dst, double* npart,
              const float* V32 = nullptr, unsigned* fb = nullptr, double* fn2_fast = nullptr, bool nt = false);
// dst = src - V[:, :ncols] h[:ncols] - u0 h[ncols]; optional per-block sum of dst^2 -> npart
void update(hipStream_t s, int ldv, const double* V, int ncols, int has_u0, double u0val, int nreal,
            const double* h, const double* src, double* dst, double* npart, const float* V32 = nullptr,
            unsigned* fb = nullptr, double* fn2_fast = nullptr, bool nt = false, const int* flag = nullptr,
            unsigned* pub_rearm = nullptr);
// Partial reorthogonalisation (Lanczos reorth 3; one workgroup per step,
// between the SpMV and the projection): alpha = sum(apart) (k_three_term's
// order: the bits every other alpha path gives) -> *a3; beta_{i+1} estimated
// as sqrt(||w||^2 - alpha^2 - beta_i^2); Simon's omega recurrence (PROPACK
// update_mu) for the next vector against v_0..v_i and u0 from the two
// previous rows of the ring `omega` (3 rows of OMEGA_LD) and the projected
// matrix (alpha[j], offd[j] for j < i: final; the kept ones uploaded after a
// restart); flags[i] = 1 when max |omega| > thresh or the step is forced (the
// first step of a run, the step after a triggered one, the cycle's last step,
// an estimate lost to cancellation).  The projection and the update of the
// step read flags[i] (0: f = f', no pass over the basis).
constexpr int OMEGA_LD = MAX_NCV + 8;  // ring row: [0, MAX_NCV) basis columns, [MAX_NCV] u0
struct ProState {
    double anorm;   // running estimate of ||L|| (max |alpha_j| + beta_j + beta_{j+1})
    int force;      // the next step projects (the second of a pair)
    int projected;  // steps that projected, this solve
    int timeouts;   // in-launch waits that gave up (PROI; the host fails the solve on any)
    int pad;
};
// dst[i], dst[m + i] (, dst[flags_off + i]) = alpha, offd (, flags) [i] for
// i < b and dst[2m + i] = fn2[i] for i < bf (< 0: b): the mid-cycle check's
// copy, one launch into pinned host memory.  done != null: then *done = seq
// (system scope), after every store of the slot is released to the system
void chk_gather(hipStream_t s, const double* alpha, const double* offd, const double* fn2, const double* flags, int b,
                int m, size_t flags_off, double* dst, int bf = -1, unsigned* done = nullptr, unsigned seq = 0);
// the implicit restart's uploads from pinned host staging in one launch:
// qd[0:nq) = q_src, alpha[0:na) = kp[0:na) and offd[1:na) = kp[na+1:2na) when
// kp != null, bov[0:nbov) = NaN (all-ones bits)
void restart_upload(hipStream_t s, const double* q_src, int nq, double* qd, const double* kp, int na, double* alpha,
                    double* offd, double* bov, int nbov);
// out[0..1] = the sums of a[0:n) and b[0:n) (one workgroup; pro_decide's order)
void sum_pair(hipStream_t s, const double* a, const double* b, int n, double* out);
void pro_step(hipStream_t s, const double* apart, const double* wpart, int nparts, double* a3, const double* fn2_i,
              const double* bov_i, const double* alpha, const double* offd, double* omega, ProState* st, int* flags,
              int i, int seg0, int m, double thresh, double eps1);
// The decision inside the projection launch (PROI, no k_pro launch): its
// first workgroup runs k_pro's body and publishes 1 + decision to PRO_PUB
// words (one 256-B line each; workgroup b polls word b % 8, its XCD's); the
// other column groups wait for it before their basis loads, column group 0
// after forming f'.  The step's update re-arms the words (zero) for the next
// launch.  i = ncols - 1; alpha / a3 as k_pro.
constexpr int PRO_PUB = 8;
constexpr int PRO_PUB_STRIDE = 64;  // uints between two words (256 B)
// (merged update: word PRO_PUB is the launch's done counter — the column
// groups' and the norm's last workgroups, once their h entries are stored)
constexpr int PRO_PUB_WORDS = PRO_PUB + 1;
struct ProLaunch {
    const double* wpart = nullptr;
    const double* alpha = nullptr;
    const double* offd = nullptr;
    double* omega = nullptr;
    ProState* st = nullptr;
    int* flags = nullptr;
    unsigned* pub = nullptr;  // PRO_PUB_WORDS words, zero before the launch
    double* a3 = nullptr;
    // merged (the update's workgroups follow the projection's in the launch):
    double* npart = nullptr;      // the update's ||f||^2 partials
    const float* V32 = nullptr;   // the fp32 shadow (B32 update), column i from the SpMV
    unsigned* fb = nullptr;       // B32 fp64-fallback count
    int merged = 0;               // the update's workgroups in this launch (no update launch)
    // > 0: at most cgw workgroups per row block, each walking the column
    // groups cg0, cg0 + cgw, ... (f' formed once per workgroup; a skipped
    // step dispatches nrb * cgw projection workgroups instead of nrb * ncg).
    // The partials of every (row block, column group) tile, and so every
    // bit, are the same as with one workgroup per tile (cgw = 0)
    int cgw = 0;
    int seg0 = 0, m = 0;
    double thresh = 0.0, eps1 = 0.0;
    // dispatch-order independence: every workgroup takes its logical index
    // from a ticket (8 counters by blockIdx % 8, PRO_PUB_STRIDE uints apart,
    // zero before the launch; the last ticket of each re-arms it), so the
    // jobs are handed out in dependency order whatever order the hardware
    // dispatches the workgroups in.  null: logical index = blockIdx
    unsigned* tix = nullptr;
    int rev = 0;  // (test) the physical index reversed before anything else (EK_DISPATCH_REVERSE)
    // > 0: workgroups of this kernel resident at once on the device; a launch
    // whose grid fits is order-free by itself (every waiter's job is resident
    // or runs as others finish), so it takes no tickets (gemvt_tt)
    int cap = 0;
};
// resident capacity (workgroups) of the k_gemvt_pro instantiation gemvt_tt
// launches for these flags on a device of num_cu compute units
int gemvt_pro_capacity(bool nt, bool wide, bool merged, bool b32u, int num_cu);
// the grid gemvt_tt launches with the in-launch decision (ncgl workgroups per row block)
int gemvt_pro_grid(int nrb, int ncgl, int ldv, bool merged);
// fn2_out[0] = sum(npart[0:nb]); if step >= 0: CGS2 (a3 == null):
// alpha[step] = h1[step]+h2[step], offd[step] = h1[step-1]+h2[step-1]; three-term:
// alpha[step] = *a3 + h2[step], offd[step] = sqrt(*fn2_i) + h2[step-1]
void finalize_step(hipStream_t s, const double* npart, int nb, double* fn2_out, const double* h1,
                   const double* h2, int step, double* alpha, double* offd, const double* a3 = nullptr,
                   const double* fn2_i = nullptr, const double* bov_i = nullptr);
// fp = w - alpha vi - beta_i vim1 (vim1 may be null), beta_i = sqrt(*fn2_i) unless the override
// *bov_i is not NaN (0 after an injected restart vector); alpha = sum(apart[0:nparts]) when
// nparts > 0 (written to *alpha_io), else read from *alpha_io
void three_term(hipStream_t s, int ldv, const double* apart, int nparts, double* alpha_io, const double* w,
                const double* vi, const double* vim1, const double* fn2_i, const double* bov_i, double* fp,
                float* v32col = nullptr);
// out[:, j] = V[:, :m] Q[:, j] for j < kk (Q col-major m x kk, device); out32: also fl32 of it
void gemm_vq(hipStream_t s, int ldv, const double* V, int m, const double* Q, int kk, double* out,
             float* out32 = nullptr);
void inject_random(hipStream_t s, double* f, int ldv, long long row0, long long nrows, unsigned long long st0);
// zero the padded rows [nreal, ldv) of the first ncols columns of V
void zero_pad_rows(hipStream_t s, double* V, int ldv, int nreal, int ncols);
// device median split of the Fiedler vector (kernels_kl.hip)
size_t split_tmp_bytes(int n);
void fiedler_scale(hipStream_t s, const double* x, double sgn, int n, double* out);
// the sort keys of the values at ranks k0 and k1 of v (radix select) into
// keys_out[0..1] (device); key_value turns a key back into its double
void split_select(hipStream_t s, void* tmp, const double* v, int n, unsigned k0, unsigned k1,
                  unsigned long long* keys_out);
double key_value(unsigned long long key);
// the remain[] lists, plist and initial sides of the split at med; n0_out
// (device): the side-0 count
void split_partition(hipStream_t s, void* tmp, const double* v, int n, double med, int32_t* order0, int32_t* order1,
                     uint32_t* plist, uint8_t* side, unsigned* n0_out);
// f = f*sigma + x*hk ; per-block sum of f^2 -> npart
void axpby_norm(hipStream_t s, int ldv, double* f, double sigma, const double* x, double hk, double* npart);
// x = x / sqrt(*n2) ... and deflate helpers
void scale_sub_mean(hipStream_t s, int ldv, double* x, int nreal, const double* mean_sum, double inv_n);
void sum_partial(hipStream_t s, int ldv, const double* x, int nreal, double* npart, int squares);
// part[b] = sum over block b's real rows (512 a block) of (w - lambda x)^2
void resid_partial(hipStream_t s, int ldv, const double* w, const double* x, double lambda, int nreal, double* part);
// x[0:ldv) = Park-Miller start vector over global rows row0.. (0 past nreal)
void start_vector(hipStream_t s, int ldv, long long row0, int nreal, double* x);

// kernels_kl.hip
#ifndef EK_KL_THREADS
#define EK_KL_THREADS 512  // (A/B builds: EXTRA_DEFS=-DEK_KL_THREADS=768)
#endif
constexpr int KL_LOOP_THREADS = EK_KL_THREADS;  // 8 waves: 256 VGPRs per lane, no spills in the swap loop
// 2048 since round 6: against 1024, 1.5 % a swap at the headline and 3-19 %
// from the 2x to the 10x synthetic (fewer chunk keys to select from);
// 512 and 4096 were slower (profiles/r06/kl/kl_chunk_*.txt)
#ifndef EK_KL_CHUNK
#define EK_KL_CHUNK 2048  // (A/B builds: EXTRA_DEFS=-DEK_KL_CHUNK=1024)
#endif
constexpr int KL_CHUNK = EK_KL_CHUNK;  // positions per chunk key (a few keys per lane: barrier-free selection)
// the off-chip-bitmap loop's chunks (k_kl_swap_loop<.., GB>, graphs past the
// LDS budget): 4096 positions, 3.11 -> 2.90 us a swap at 10x and equal at
// 3x / 5x (profiles/r06/kl/kl_chunk_big_2048_4096.txt)
#ifndef EK_KL_CHUNK_GB
#define EK_KL_CHUNK_GB 4096
#endif
constexpr int KL_CHUNK_GB = EK_KL_CHUNK_GB;
// positions the gain / descriptor arrays are padded to: whole chunks of either size
constexpr int KL_CHUNK_PAD = KL_CHUNK > KL_CHUNK_GB ? KL_CHUNK : KL_CHUNK_GB;
static_assert(KL_CHUNK_PAD % KL_CHUNK == 0 && KL_CHUNK_PAD % KL_CHUNK_GB == 0, "chunk sizes must nest");
struct alignas(16) KLInfo {
    int32_t a, b, c, d;
};
struct KLDev {
    int n = 0;
    long long nnz = 0;  // rowptr[n]
    const int32_t* rowptr = nullptr;
    const int32_t* col = nullptr;
    const float* w = nullptr;
    uint8_t* side = nullptr;        // current split (0/1); final sides after the loop
    const uint8_t* side_init = nullptr;
    // erased from remain[] (global-state mode only); the on-chip loop whose
    // side / locked bitmaps exceed its LDS budget keeps them here instead
    // (k_kl_swap_loop<.., GB>: 2 ceil(n/32) words)
    uint8_t* locked = nullptr;
    float* gp0 = nullptr;           // gains of remain[0] nodes, by POSITION (NaN = erased)
    float* gp1 = nullptr;           // gains of remain[1] nodes, by position
    const int32_t* order0 = nullptr;  // remain[0] positions -> node
    const int32_t* order1 = nullptr;
    const uint32_t* plist = nullptr;  // node -> position | (list << 31)
    int n0 = 0, n1 = 0, nck0 = 0, nck1 = 0;
    unsigned long long* ckey0 = nullptr;  // per-chunk best (gain, first position) keys
    unsigned long long* ckey1 = nullptr;
    double* cut_part = nullptr;
    float* cut0 = nullptr;
    // row descriptors: by position in each list {node, rowptr, rowlen, 0} and
    // by node {rowptr, rowlen, plist, 0}; chunk winners' descriptors
    const KLInfo* pinfo0 = nullptr;
    const KLInfo* pinfo1 = nullptr;
    const KLInfo* nd = nullptr;
    KLInfo* cinfo0 = nullptr;
    KLInfo* cinfo1 = nullptr;
    // per CSR entry p: the neighbour's descriptor {col[p], rowptr, rowlen, plist}
    const KLInfo* aux = nullptr;
    // per CSR entry p: the first 2*KL_SEG_LANES {col, w} entries of row col[p]
    // as KL_SEG_LANES 16-B pieces (zero-padded); null when it would not fit
    const KLInfo* seg = nullptr;
    // the same 32 entries weight-coded (preferred; seg is then null): one
    // 32-bit word (code << wcolbits) | col per entry, 4 per 16-B piece,
    // KL_SEGC_PIECES pieces per p; word 0 pads (wdict[0] == 0.0f).  Half the
    // bytes, so the segments and descriptors fit the Infinity Cache together.
    const KLInfo* segc = nullptr;
    const float* wdict = nullptr;  // exact fp32 weight of each code (nwd entries)
    int nwd = 0, wcolbits = 0;
};
constexpr int KL_SEGC_PIECES = 8;
constexpr int KL_WDICT_CAP = 4096;  // codes kept in LDS; more distinct weights: plain segments
constexpr int KL_SEG_LANES = 16;  // 16-B pieces of 2 entries: 32 entries inline (all but 0.05% of touched rows; 16 inline: 70 vs 59 ms swap loop at ibm18 shape)
constexpr int KL_ITEM_CAP = 256;  // updated rows whose new key/descriptor are kept in LDS (more: rederived, tagged)
// LDS bytes the loop kernel needs to keep side/locked bitmaps, chunk keys and
// chunk winners on chip (0 when they do not fit: global-state mode).
size_t kl_loop_lds_bytes(const KLDev& d, bool bitmaps = true, bool fixed = false);
struct KLOut {
    long long iterations;
    long long best_iter;
    float initial_cut, best_cut, final_cut;
    unsigned int status;
    unsigned long long prof[16];  // EK_KL_PROF: [0..11] 100 MHz ticks per loop phase (thread 0's view)
                                  // or event counts x100, [14] shader cycles, [15] 100 MHz ticks of the loop;
                                  // [8] shader cycles, [9] 100 MHz ticks of the whole loop
    unsigned long long warr[42];  // EK_KL_PROF: per wave, shader cycles from its loop top to its arrival
                                  // at barrier 1 ([wave]) and barrier 2 ([8 + wave]), to the end of G2a
                                  // ([16 + wave]), to the end of the selection ([24 + wave]) and to G2a's reads consumed ([32 + wave]);
                                  // [40], [41]: swaps whose node1 / node2 the prefetch predicted
};
void kl_prepare(hipStream_t s, const KLDev& d);  // gains, initial cut, chunk keys
// aux[p] = {col[p], nd[col[p]].{rowptr, len, plist}} for p < nnz (after the partition is set)
void kl_build_aux(hipStream_t s, int64_t nnz, const int32_t* col, const KLInfo* nd, KLInfo* aux);
void kl_build_seg(hipStream_t s, int64_t nnz, const int32_t* rowptr, const int32_t* col, const float* w, KLInfo* seg);
// pinfo0/pinfo1 (by position, zero-padded to pad0/pad1) and nd (by node) of a partition
void kl_build_desc(hipStream_t s, int n, int n0, int n1, int pad0, int pad1, const int32_t* order0,
                   const int32_t* order1, const uint32_t* plist, const int32_t* rowptr, KLInfo* p0, KLInfo* p1,
                   KLInfo* nd);
// segc from the coded words kw[p] = (code << wcolbits) | col[p]
void kl_build_segc(hipStream_t s, int64_t nnz, const int32_t* rowptr, const int32_t* col, const uint32_t* kw,
                   KLInfo* segc);
// weight dictionary of the KL graph (code 0 = 0.0f); false when it does not fit
bool kl_weight_codes(int64_t n, int64_t nnz, const int32_t* col, const float* w, std::vector<uint32_t>& kw,
                     std::vector<float>& wdict, int& wcolbits);
void kl_loop(hipStream_t s, const KLDev& d, int limit, ek_swap* log, long long cap, KLOut* out);
// sides_out = side_init with the first `count` swaps of `log` applied (count on device: *best or *iters)
void kl_replay(hipStream_t s, int n, const uint8_t* side_init, const ek_swap* log, const long long* count,
               long long cap, uint8_t* sides_out);
// the net cuts of the three sides as per-workgroup partials: the cut of
// side k is the sum of part[k * net_cut_blocks(nets) + b] over b
int net_cut_blocks(int64_t nets);
void net_cut(hipStream_t s, int64_t nets, const int64_t* net_ptr, const int32_t* pins, const uint8_t* side_a,
             const uint8_t* side_b, const uint8_t* side_c, unsigned* part);

}  // namespace dev
}  // namespace ek

// ---------------------------------------------------------------------------
// parallel_for implementation
#include <algorithm>
#include <thread>
template <class F>
void ek::parallel_for(int64_t n, F&& fn) {
    const int64_t T = std::min<int64_t>(host_threads(), std::max<int64_t>(1, n / 4096));
    if (T <= 1) {
        fn(int64_t(0), n);
        return;
    }
    run_threads(int(T), [&](int t) { fn(n * t / T, n * (t + 1) / T); });
}

template <class F>
void ek::run_threads(int T, F&& fn) {
    if (T <= 1) {
        if (T == 1) fn(0);
        return;
    }
    using Fn = std::remove_reference_t<F>;
    pool_run(T, [](void* c, int t) { (*static_cast<Fn*>(c))(t); }, const_cast<void*>(static_cast<const void*>(&fn)));
}
