// GPU context, SpMV seam, implicitly restarted Lanczos driver and KL driver
// of libeigkl_hip.so (host code over the HIP runtime + RCCL).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <limits>
#include <map>
#include <memory>
#include <tuple>

#include "ek_internal.hpp"

#ifndef EK_UPD_RED_MAX_NRB
#define EK_UPD_RED_MAX_NRB 256  // row blocks up to which the update workgroups sum the partials themselves
#endif

#define HIPCHK(call)                                                                                 \
    do {                                                                                             \
        const hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess) {                                                                      \
            (void)hipGetLastError(); /* a failed call leaves no sticky error for the next entry */    \
            ek::fail(EK_EHIP, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, __LINE__); \
        }                                                                                            \
    } while (0)
#define NCCLCHK(call)                                                                                 \
    do {                                                                                              \
        const ncclResult_t r_ = (call);                                                               \
        if (r_ != ncclSuccess) ek::fail(EK_ECOMM, "%s failed: %s", #call, ncclGetErrorString(r_));    \
    } while (0)

namespace {

// Owning device allocation.
struct DBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { reset(); }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    void ensure(size_t b) {
        if (b <= bytes && p) return;
        reset();
        HIPCHK(hipMalloc(&p, b ? b : 16));
        bytes = b;
    }
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

template <class T>
void upload(DBuf& d, const T* h, size_t n, hipStream_t s) {
    d.ensure(n * sizeof(T));
    if (n) HIPCHK(hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, s));
}

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

}  // namespace

// Setup uploads through the context's pinned staging: a copy from pageable
// memory makes the runtime pin (or bounce) the user pages on every call,
// which on freshly parsed arrays costs milliseconds; a memcpy into pinned
// memory and an async DMA do not.  The caller sizes the arena for all the
// uploads of one setup call and drains the stream before the next call.
// The main stream and the KL stream each have an arena of their own: the KL
// graph setup runs on ek_solve_file's host thread while the main thread
// uploads the pins for the Laplacian build.
struct Uploader {
    ek_ctx* c;
    hipStream_t s;
    unsigned char*& buf;  // c->up (main stream) or c->kup (KL stream)
    size_t& cap;
    size_t off = 0;
    Uploader(ek_ctx* ctx, hipStream_t st, size_t total);
    template <class T>
    void put(DBuf& d, const T* h, size_t n);
};

namespace {
inline int64_t chunk_pad(int64_t n) { return std::max<int64_t>(round_up(n, ek::dev::KL_CHUNK_PAD), ek::dev::KL_CHUNK_PAD); }

}  // namespace

struct ek_ctx {
    int device = 0;
    int num_cu = 256;  // compute units (the panel SpMV's resident workgroups)
    hipStream_t stream = nullptr;
    // the KL graph's setup (ek_kl_graph_setup / ek_kl_nets_setup) runs on its
    // own stream: ek_solve_file calls it from its host thread while the
    // Lanczos solve occupies `stream`
    hipStream_t kstream = nullptr;
    // RCCL, or the host-staged exchange of ek_comm_init_host
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    // the sharded layout and exchange (slot-padded all-gather, the one-all-
    // reduce step): nranks > 1, or a forced 1-rank communicator (EK_COMM_FORCE,
    // which runs the RCCL production path on one GPU: tests)
    bool mr = false;
    ek_allgather_fn host_ag = nullptr;
    ek_allreduce_fn host_ar = nullptr;
    void* host_user = nullptr;
    double* stage = nullptr;  // pinned staging of the host-staged exchange
    size_t stage_doubles = 0;
    unsigned char* up = nullptr;  // pinned staging of the setup uploads on `stream` (see Uploader)
    size_t up_bytes = 0;
    unsigned char* kup = nullptr;  // ... and on `kstream`
    size_t kup_bytes = 0;
    double comm_ms = 0.0;     // host-observed time inside collectives (current solve)
    int64_t n_ag = 0, n_ar = 0;  // collectives issued (current solve; sharded contexts)
    // Laplacian rows owned by this context.  Sharded: rank r owns
    // [shard_off[r], shard_off[r+1]) (nnz-balanced, so the slices differ);
    // nloc = the largest slice; each rank's f is all-gathered into a slot of
    // `slot` doubles (its rows, zero padding, its ||f||^2 partial at [ldv]),
    // and the matrix's columns are remapped to that padded layout.
    int64_t n = 0, row0 = 0, nrows = 0, nloc = 0, nnz = 0;
    std::vector<int64_t> shard_off;
    int64_t slot = 0;
    DBuf off_d, xexp;
    DBuf spx;  // ek_spmv's x in the all-gather layout (sharded), sized when the shard map is set
    // The halo exchange of the sharded step (halo_build): instead of every
    // rank's whole slot, each rank receives only the rows of f its columns
    // read, into a compact x: block q (ranks in order) holds the rows of rank
    // q this rank reads, ascending (its own block: all its rows), then q's
    // ||f||^2 partial at the block end (hx_pidx[q]): one message per peer, the
    // sender's packed rows closed by its partial.  The columns are remapped
    // monotonically to it, so rows stay sorted and every product is summed in
    // the same order as over the slot layout: the same bits.  Used where it
    // moves fewer bytes than the all-gather (EK_MR_HALO=0/1 forces either).
    bool halo = false;
    int halo_calls = 0;  // halo_build calls since the shard map was set (exactly one per setup: it is collective)
    std::vector<int64_t> hx_base;             // nranks + 1: block q at [hx_base[q], hx_base[q+1]), its partial last
    std::vector<int64_t> hx_rcnt;             // rows received from q (own: nrows); the block is hx_rcnt[q] + 1
    std::vector<int64_t> hx_scnt, hx_soff;    // rows sent to q, and that message's offset in hx_sbuf (+1: the partial)
    std::vector<int64_t> hx_src;              // host-staged: q's message to this rank inside q's (padded) sbuf
    std::vector<int32_t> hx_gidx_h;           // X[t]'s global row (-1: a partial slot)
    int64_t hx_nsend = 0, hx_smax = 0;
    DBuf hx_sidx, hx_sbuf, hx_X, hx_pidx, hx_gidx, hx_gbuf;
    // exchange accounting (sharded solves): exchanges, point-to-point
    // messages posted, and (with timing on) the exchanges' and all-reduces'
    // durations on the device (HIP events around them on their streams) or,
    // host-staged, as the host saw them
    int64_t hx_exchanges = 0, hx_sends = 0, hx_recvs = 0;
    double x_ms = 0.0, ar_ms = 0.0;
    int64_t x_timed = 0, ar_timed = 0;
    bool comm_time = false;
    std::vector<hipEvent_t> cm_ev;            // event pool, reused across solves
    std::vector<std::pair<int, int>> cm_rec;  // (kind: 0 exchange, 1 all-reduce; first event) of this solve
    size_t cm_used = 0;
    // the owned-slot part of a sharded rank's rows (plain CSR, local column
    // ids), summed while the all-gather of the other slots runs on `gstream`
    DBuf own_rowptr, own_col, own_val, own_rb, yown;
    int own_nrb = 0;
    int64_t own_nnz = 0;
    bool own_ready = false;
    hipStream_t gstream = nullptr;
    hipEvent_t ag_ev[2] = {nullptr, nullptr};
    // the column-panel form of the SpMV (pn_G > 0; kernels_panel.hip)
    int pn_G = 0, pn_P = 0, pn_pb = 0, pn_max_rows = 0, pn_ndict = 0;
    DBuf pn_wrow, pn_start, pn_word, pn_rid;
    int block_nnz = 1024, nrb_spmv = 0;
    bool spmv_long = true;  // a row block is one row longer than block_nnz (the SpMV's vector mode)
    DBuf rb, rowptr, col, val, pk, rel, dict;
    int colbits = 0;  // > 0: the dictionary-coded matrix (pk, dict) is the one the SpMV reads
    int64_t mat_bytes = 0;  // bytes of the matrix arrays one SpMV reads, as stored
    // Lanczos workspace
    DBuf V, Vn, f, w, xfull, part, h1, h2, alpha, offd, fn2, npart, apart, Qd, scal, bov;
    DBuf V32, Vn32;  // the basis's fp32 shadow (ek_lanczos_opts::basis32) and its restart buffer
    DBuf fbk;        // launches whose fp32-shadow update fell back to V (a device counter)
    DBuf actr;  // the SpMV's last-block counter (alpha hand-off), zero between launches
    DBuf gctr;  // the projection's column-group counters (k_gemvt hand-off), zero between launches
    // partial reorthogonalisation (reorth 3): the SpMV's ||w||^2 partials, the
    // omega ring (3 x OMEGA_LD), k_pro's state and its per-step decisions
    DBuf wpart, omega, prost, pflags;
    DBuf cflag;  // the sharded step's cancellation flags (update_mr), one double per step
    // HIP graphs of the single-context Lanczos step chunks (factorize_fused),
    // keyed by (first step, end, run start, V, V32): captured on a chunk's
    // second launch, replayed from its third; dropped when any buffer or
    // parameter the launches carry changes (lz_sig)
    std::map<std::tuple<int, int, int, const void*, const void*>, hipGraphExec_t> lz_graphs;
    std::map<std::tuple<int, int, int, const void*, const void*>, int> lz_seen;
    std::vector<uint64_t> lz_sig;
    // KL state
    int64_t kl_n = 0, kl_n0 = 0, kl_n1 = 0, kl_nets = 0;
    DBuf kl_rowptr, kl_col, kl_w, kl_side, kl_side_init, kl_locked, kl_gp0, kl_gp1, kl_order0, kl_order1, kl_plist, kl_pinfo0, kl_pinfo1, kl_nd, kl_cinfo0, kl_cinfo1,
        kl_ckey0, kl_ckey1, kl_aux, kl_seg, kl_cutpart, kl_cut0, kl_log, kl_out, kl_sides_tmp, kl_count, kl_netptr, kl_pins;
    bool kl_graph_ready = false, kl_part_ready = false, kl_seg_ok = false, kl_segc_ok = false;
    DBuf kl_segc, kl_wdict;
    // device build of the Laplacian rows (ek_spmv_setup_pins)
    DBuf lb_netptr, lb_pins, lb_icnt, lb_rcnt, lb_cur, lb_ip, lb_rp, lb_tiles, lb_inc, lb_scol, lb_sval, lb_tval,
        lb_ulen, lb_len, lb_diag, lb_long, lb_cnt, lb_off, lb_table, lb_flags, lb_codes;
    int kl_nwd = 0, kl_wcolbits = 0;
    std::vector<int32_t> kl_rowptr_h;  // host copy (row descriptors)
    std::vector<hipEvent_t> spmv_ev;   // SpMV timing events, created once per context
    double* pin = nullptr;             // pinned host staging (Ritz vector + residual rows)
    size_t pin_doubles = 0;
    // mid-cycle convergence checks of the Lanczos driver: a copy stream, two
    // pinned slots of {alpha, offd, fn2} and their events (created on first use)
    hipStream_t cstream = nullptr;
    hipEvent_t chk_done[2] = {nullptr, nullptr}, chk_copied[2] = {nullptr, nullptr};
    hipEvent_t fin_ev = nullptr;  // the final Ritz vector's host copy landed
    double* chk_pin = nullptr;
    // the checks' completion words (EK_CHK_POLL): one per slot, 256 B apart, in
    // pinned host memory the check's gather writes last; the host polls them
    unsigned* chk_word = nullptr;
    unsigned chk_seq = 0;
    double* q_pin = nullptr;  // pinned staging of the restart's Q (MAX_NCV x (MAX_NCV + 1)), then the kept
                              // projected matrix for k_pro (2 x (MAX_NCV + 2))
    // the last Fiedler vector as returned (normalised, sign fixed), kept on
    // the device for ek_kl_set_partition_fiedler, and that split's scratch
    DBuf fied, sp_out, sp_tmp;
    int64_t fied_n = 0;
};

Uploader::Uploader(ek_ctx* ctx, hipStream_t st, size_t total)
    : c(ctx), s(st), buf(st == ctx->kstream ? ctx->kup : ctx->up), cap(st == ctx->kstream ? ctx->kup_bytes : ctx->up_bytes) {
    total = (total + 64) * 2;  // alignment slack
    if (cap < total) {
        // the arena's previous user drained its stream before returning
        if (buf) HIPCHK(hipHostFree(buf));
        buf = nullptr;
        cap = 0;
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&buf), total, hipHostMallocDefault));
        cap = total;
    }
}

template <class T>
void Uploader::put(DBuf& d, const T* h, size_t n) {
    d.ensure(n * sizeof(T));
    if (!n) return;
    off = (off + 63) / 64 * 64;
    if (off + n * sizeof(T) > cap) ek::fail(EK_EINVAL, "upload staging overflow");
    std::memcpy(buf + off, h, n * sizeof(T));
    HIPCHK(hipMemcpyAsync(d.p, buf + off, n * sizeof(T), hipMemcpyHostToDevice, s));
    off += n * sizeof(T);
}

namespace {

void set_device(ek_ctx* c) { HIPCHK(hipSetDevice(c->device)); }

ek_ctx* check_ctx(ek_ctx* c) {
    if (!c) ek::fail(EK_EINVAL, "null ek_ctx");
    set_device(c);
    return c;
}

ek::dev::SpmvMat spmv_mat(const ek_ctx* c) {
    ek::dev::SpmvMat m;
    m.nblocks = c->nrb_spmv;
    if (c->pn_G > 0) {
        m.panel.G = c->pn_G;
        m.panel.P = c->pn_P;
        m.panel.pb = c->pn_pb;
        m.panel.max_rows = c->pn_max_rows;
        m.panel.ndict = c->pn_ndict;
        m.panel.wrow = c->pn_wrow.as<int32_t>();
        m.panel.start = c->pn_start.as<long long>();
        m.panel.word = c->pn_word.as<uint32_t>();
        m.panel.rid = c->pn_rid.as<uint16_t>();
        m.dict = c->dict.as<double>();
        return m;
    }
    m.block_nnz = c->block_nnz;
    m.has_long = c->spmv_long;
    m.desc = c->rb.as<int32_t>();
    m.rowptr = c->rowptr.as<int32_t>();
    if (c->colbits > 0) {
        m.colbits = c->colbits;
        m.pk = c->pk.as<uint32_t>();
        m.rel = c->rel.as<uint16_t>();
        m.dict = c->dict.as<double>();
    } else {
        m.col = c->col.as<int32_t>();
        m.val = c->val.as<double>();
    }
    return m;
}

// the owned-slot rows (c->own_*): plain CSR over local columns, x = the rank's f
ek::dev::SpmvMat own_mat(const ek_ctx* c) {
    ek::dev::SpmvMat m;
    m.nblocks = c->own_nrb;
    m.block_nnz = 512;
    m.desc = c->own_rb.as<int32_t>();
    m.rowptr = c->own_rowptr.as<int32_t>();
    m.col = c->own_col.as<int32_t>();
    m.val = c->own_val.as<double>();
    return m;
}

double* stage_for(ek_ctx* c, size_t doubles) {
    if (c->stage_doubles < doubles) {
        if (c->stage) HIPCHK(hipHostFree(c->stage));
        c->stage = nullptr;
        c->stage_doubles = 0;
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->stage), doubles * 8, hipHostMallocDefault));
        c->stage_doubles = doubles;
    }
    return c->stage;
}

struct CommTimer {  // host-observed time of one collective (kind 0: an exchange of f, 1: an all-reduce)
    ek_ctx* c;
    int kind;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~CommTimer() {
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        c->comm_ms += ms;
        if (!c->comm_time) return;
        (kind ? c->ar_ms : c->x_ms) += ms;
        ++(kind ? c->ar_timed : c->x_timed);
    }
};

// Device-side timing of the RCCL collectives of a sharded solve (comm_time:
// the solve's time_spmv): a pair of events from the context's pool around
// one exchange (kind 0) or all-reduce (kind 1) on its stream.  Their elapsed
// time holds the wait for the peers, i.e. what the step pays for the
// collective.  comm_collect sums them once the solve has drained.
int comm_mark(ek_ctx* c, hipStream_t st) {
    if (!c->comm_time || !c->comm) return -1;
    while (c->cm_used + 2 > c->cm_ev.size()) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        c->cm_ev.push_back(e);
    }
    const int i = int(c->cm_used);
    c->cm_used += 2;
    HIPCHK(hipEventRecord(c->cm_ev[size_t(i)], st));
    return i;
}

void comm_done(ek_ctx* c, int i, int kind, hipStream_t st) {
    if (i < 0) return;
    HIPCHK(hipEventRecord(c->cm_ev[size_t(i) + 1], st));
    c->cm_rec.emplace_back(kind, i);
}

void comm_collect(ek_ctx* c) {
    for (const auto& r : c->cm_rec) {
        HIPCHK(hipEventSynchronize(c->cm_ev[size_t(r.second) + 1]));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, c->cm_ev[size_t(r.second)], c->cm_ev[size_t(r.second) + 1]));
        (r.first ? c->ar_ms : c->x_ms) += double(ms);
        ++(r.first ? c->ar_timed : c->x_timed);
    }
    c->cm_rec.clear();
    c->cm_used = 0;
}

}  // namespace

void ek::ctx_ranks(ek_ctx* c, int* rank, int* nranks) {
    if (!c) fail(EK_EINVAL, "null ek_ctx");
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
}

namespace {

// In-place sum all-reduce of `count` device doubles, ordered on the context
// stream.  RCCL: enqueued on the stream.  Host-staged: stream drained, the
// operand staged through pinned memory around the caller's collective.
void allreduce(ek_ctx* c, double* p, size_t count) {
    if (!c->mr || !count) return;
    ++c->n_ar;
    if (c->comm) {
        const int e = comm_mark(c, c->stream);
        NCCLCHK(ncclAllReduce(p, p, count, ncclDouble, ncclSum, c->comm, c->stream));
        comm_done(c, e, 1, c->stream);
        return;
    }
    CommTimer t{c, 1};
    double* h = stage_for(c, count);
    HIPCHK(hipMemcpyAsync(h, p, count * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->host_ar(c->host_user, h, int64_t(count)) != 0) ek::fail(EK_ECOMM, "host all-reduce callback failed");
    HIPCHK(hipMemcpyAsync(p, h, count * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));  // the staging buffer is reused by the next collective
}

// recv[r*count .. (r+1)*count) = rank r's send block (rank-major), on the
// stream (default: the context's).
void allgather(ek_ctx* c, const double* send, size_t count, double* recv, hipStream_t st = nullptr) {
    ++c->n_ag;
    if (!st) st = c->stream;
    if (c->comm) {
        const int e = comm_mark(c, st);
        NCCLCHK(ncclAllGather(send, recv, count, ncclDouble, c->comm, st));
        comm_done(c, e, 0, st);
        return;
    }
    CommTimer t{c, 0};
    const size_t tot = count * size_t(c->nranks);
    double* h = stage_for(c, count + tot);
    HIPCHK(hipMemcpyAsync(h, send, count * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (c->host_ag(c->host_user, h, int64_t(count), h + count) != 0)
        ek::fail(EK_ECOMM, "host all-gather callback failed");
    HIPCHK(hipMemcpyAsync(recv, h + count, tot * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
}

void comm_reset(ek_ctx* c) {
    if (c->comm) ncclCommDestroy(c->comm);
    c->comm = nullptr;
    c->host_ag = nullptr;
    c->host_ar = nullptr;
    c->host_user = nullptr;
    c->nranks = 1;
    c->rank = 0;
    c->mr = false;
}

// EK_COMM_FORCE=1: a 1-rank communicator still takes the multi-rank path
bool comm_forced() {
    const char* e = std::getenv("EK_COMM_FORCE");
    return e && e[0] && e[0] != '0';
}

}  // namespace

extern "C" {

int ek_device_count(int* count) {
    EK_TRY
    int c = 0;
    const hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    if (count) *count = c;
    return EK_OK;
    EK_CATCH
}

int ek_init(int device, ek_ctx** out) {
    EK_TRY
    if (!out) ek::fail(EK_EINVAL, "ek_init: null out");
    int cnt = 0;
    ek::cold_stamp("hip_first_call");
    if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= 0) ek::fail(EK_EHIP, "no HIP device available (no CPU fallback)");
    ek::cold_stamp("hip_device_count");
    if (device < 0 || device >= cnt) ek::fail(EK_EINVAL, "device %d out of range [0,%d)", device, cnt);
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    ek::cold_stamp("hip_props");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        ek::fail(EK_EHIP, "device %d is %s; this build targets gfx950 (MI355X)", device, prop.gcnArchName);
    auto c = std::make_unique<ek_ctx>();
    c->device = device;
    c->num_cu = std::max(1, prop.multiProcessorCount);
    HIPCHK(hipSetDevice(device));
    ek::cold_stamp("hip_set_device");
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    ek::cold_stamp("hip_stream0");
    HIPCHK(hipStreamCreateWithFlags(&c->kstream, hipStreamNonBlocking));
    ek::cold_stamp("hip_streams");
    *out = c.release();
    return EK_OK;
    EK_CATCH
}

void ek_destroy(ek_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    // drain every stream before anything it may still copy from is freed
    // (an error exit can leave async copies of the pinned buffers queued)
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->kstream);
    if (c->cstream) (void)hipStreamSynchronize(c->cstream);
    if (c->comm) ncclCommDestroy(c->comm);
    for (auto e : c->spmv_ev) (void)hipEventDestroy(e);
    for (auto e : c->cm_ev) (void)hipEventDestroy(e);
    for (int i = 0; i < 2; ++i) {
        if (i == 0 && c->fin_ev) (void)hipEventDestroy(c->fin_ev);
        if (c->chk_done[i]) (void)hipEventDestroy(c->chk_done[i]);
        if (c->chk_copied[i]) (void)hipEventDestroy(c->chk_copied[i]);
    }
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    if (c->gstream) {
        (void)hipStreamSynchronize(c->gstream);
        (void)hipStreamDestroy(c->gstream);
    }
    for (auto e : c->ag_ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& g : c->lz_graphs) (void)hipGraphExecDestroy(g.second);
    (void)hipStreamDestroy(c->kstream);
    (void)hipStreamDestroy(c->stream);
    if (c->chk_pin) (void)hipHostFree(c->chk_pin);
    if (c->chk_word) (void)hipHostFree(c->chk_word);
    if (c->q_pin) (void)hipHostFree(c->q_pin);
    if (c->pin) (void)hipHostFree(c->pin);
    if (c->stage) (void)hipHostFree(c->stage);
    if (c->up) (void)hipHostFree(c->up);
    if (c->kup) (void)hipHostFree(c->kup);
    delete c;
}

int ek_get_stream(ek_ctx* c, void** s) {
    EK_TRY
    check_ctx(c);
    if (s) *s = c->stream;
    return EK_OK;
    EK_CATCH
}

int ek_synchronize(ek_ctx* c) {
    EK_TRY
    check_ctx(c);
    HIPCHK(hipStreamSynchronize(c->stream));
    return EK_OK;
    EK_CATCH
}

int ek_comm_unique_id(void* id128) {
    EK_TRY
    if (!id128) ek::fail(EK_EINVAL, "null id buffer");
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    std::memcpy(id128, &id, sizeof id);
    return EK_OK;
    EK_CATCH
}

int ek_comm_init(ek_ctx* c, int nranks, int rank, const void* id128) {
    EK_TRY
    check_ctx(c);
    if (nranks < 1 || rank < 0 || rank >= nranks || !id128) ek::fail(EK_EINVAL, "ek_comm_init: bad argument");
    comm_reset(c);
    const bool mr = nranks > 1 || comm_forced();
    if (mr) {  // (nranks 1 under EK_COMM_FORCE: a real one-rank RCCL communicator)
        ncclUniqueId id;
        std::memcpy(&id, id128, sizeof id);
        NCCLCHK(ncclCommInitRank(&c->comm, nranks, id, rank));
    }
    c->nranks = nranks;
    c->rank = rank;
    c->mr = mr;
    c->n = 0;  // the shard map changed: ek_spmv_setup again
    return EK_OK;
    EK_CATCH
}

int ek_comm_init_host(ek_ctx* c, int nranks, int rank, ek_allgather_fn ag, ek_allreduce_fn ar, void* user) {
    EK_TRY
    check_ctx(c);
    const bool mr = nranks > 1 || comm_forced();
    if (nranks < 1 || rank < 0 || rank >= nranks || (mr && (!ag || !ar)))
        ek::fail(EK_EINVAL, "ek_comm_init_host: bad argument");
    comm_reset(c);
    c->nranks = nranks;
    c->rank = rank;
    c->mr = mr;
    c->host_ag = ag;
    c->host_ar = ar;
    c->host_user = user;
    c->n = 0;
    return EK_OK;
    EK_CATCH
}

}  // extern "C"

namespace {

inline int64_t gt_round(int64_t x) { return round_up(std::max<int64_t>(x, 1), ek::dev::GT_ROWS); }

// The shard map `off` (nranks + 1 offsets tiling [0, n)) becomes the
// context's: its rows, the largest slice (nloc) and the all-gather slot.
void set_shard(ek_ctx* c, int64_t n, const std::vector<int64_t>& off) {
    if (int(off.size()) != c->nranks + 1 || off[0] != 0 || off.back() != n)
        ek::fail(EK_EINVAL, "shard map does not tile [0, %lld)", (long long)n);
    int64_t mx = 0;
    for (int r = 0; r < c->nranks; ++r) {
        if (off[size_t(r) + 1] < off[size_t(r)]) ek::fail(EK_EINVAL, "shard map not monotone");
        mx = std::max(mx, off[size_t(r) + 1] - off[size_t(r)]);
    }
    c->shard_off = off;
    c->halo = false;
    c->halo_calls = 0;
    c->hx_exchanges = c->hx_sends = c->hx_recvs = 0;
    c->x_ms = c->ar_ms = 0.0;
    c->x_timed = c->ar_timed = 0;
    c->row0 = off[size_t(c->rank)];
    c->nrows = off[size_t(c->rank) + 1] - c->row0;
    c->nloc = c->mr ? mx : n;
    // sharded: the Lanczos vectors' rows (ldv) + 64, the rank's ||f||^2 at [ldv]
    c->slot = c->mr ? gt_round(mx) + 64 : n;
    if (c->mr && c->slot * c->nranks > INT32_MAX) ek::fail(EK_EINVAL, "sharded vector layout exceeds int32");
    // (allocated here, not inside ek_spmv: a reallocation there could free
    // memory that work queued earlier still reads)
    if (c->mr) c->spx.ensure(size_t(c->slot * c->nranks) * 8);
}

// The column space the SpMV reads: global ids, the padded all-gather layout,
// or the compact halo layout
int64_t x_extent(const ek_ctx* c) { return c->halo ? c->hx_base.back() : c->mr ? c->slot * c->nranks : c->n; }

// The halo layout from this rank's columns in the slot layout (col, host, nnz
// entries; remapped in place when the halo exchange is taken).  One
// all-gather of the request counts (every rank then takes the same decision)
// and one of the request lists: setup only.  Collective: every rank of a
// sharded context calls it exactly once per setup, after set_shard (the host
// rows of spmv_setup_rows, or the device build's, whichever the rank took).
bool halo_build(ek_ctx* c, int32_t* col, int64_t nnz) {
    c->halo = false;
    if (c->mr && ++c->halo_calls != 1)
        ek::fail(EK_ESTATE, "halo_build called %d times in one setup (a collective: once per rank)", c->halo_calls);
    if (!c->mr || c->nranks > ek::dev::MAX_HALO_RANKS) return false;
    const char* env = std::getenv("EK_MR_HALO");
    if (env && env[0] == '0') return false;
    const int R = c->nranks, me = c->rank;
    const int64_t S = c->slot;
    const auto& off = c->shard_off;
    // which rows of each other rank this rank's columns read
    std::vector<std::vector<int32_t>> pos(static_cast<size_t>(R));
    for (int q = 0; q < R; ++q)
        if (q != me) pos[size_t(q)].assign(size_t(off[size_t(q) + 1] - off[size_t(q)]), -1);
    for (int64_t p = 0; p < nnz; ++p) {
        const int q = int(col[p] / S);
        if (q != me) pos[size_t(q)][size_t(col[p] - q * S)] = 0;
    }
    std::vector<std::vector<int32_t>> req(static_cast<size_t>(R));
    for (int q = 0; q < R; ++q) {
        auto& pq = pos[size_t(q)];
        for (size_t l = 0; l < pq.size(); ++l)
            if (pq[l] == 0) {
                pq[l] = int32_t(req[size_t(q)].size());
                req[size_t(q)].push_back(int32_t(l));
            }
    }
    // C[r * R + q] = rows rank r reads from rank q
    c->scal.ensure(64);
    DBuf cnt_d, all_d;
    cnt_d.ensure(size_t(R) * 8);
    all_d.ensure(size_t(R) * size_t(R) * 8);
    std::vector<double> mine(static_cast<size_t>(R), 0.0), C(size_t(R) * size_t(R));
    for (int q = 0; q < R; ++q) mine[size_t(q)] = double(req[size_t(q)].size());
    HIPCHK(hipMemcpyAsync(cnt_d.p, mine.data(), size_t(R) * 8, hipMemcpyHostToDevice, c->stream));
    allgather(c, cnt_d.as<double>(), size_t(R), all_d.as<double>());
    HIPCHK(hipMemcpyAsync(C.data(), all_d.p, C.size() * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    auto Cat = [&](int r, int q) { return int64_t(C[size_t(r) * size_t(R) + size_t(q)]); };
    int64_t tot_halo = 0, lmax = 0;
    for (int r = 0; r < R; ++r) {
        int64_t lr = 0;
        for (int q = 0; q < R; ++q)
            if (q != r) {
                tot_halo += Cat(r, q) + 1;
                lr += Cat(r, q);
            }
        lmax = std::max(lmax, lr);
    }
    const int64_t full = int64_t(R) * int64_t(R - 1) * S;
    // (one forced rank: nothing to exchange either way; the slot layout)
    const bool use = env && env[0] ? env[0] != '0' : R > 1 && double(tot_halo) <= 0.75 * double(full);
    if (!use) return false;
    // the request lists, padded to the longest: rank r's request from this
    // rank starts at sum_{q < me, q != r} C[r][q] of r's list
    std::vector<double> lst(size_t(std::max<int64_t>(lmax, 1)), 0.0), lall(size_t(std::max<int64_t>(lmax, 1)) * R);
    {
        size_t o = 0;
        for (int q = 0; q < R; ++q)
            for (int32_t l : req[size_t(q)]) lst[o++] = double(l);
        DBuf ld, la;
        ld.ensure(lst.size() * 8);
        la.ensure(lall.size() * 8);
        HIPCHK(hipMemcpyAsync(ld.p, lst.data(), lst.size() * 8, hipMemcpyHostToDevice, c->stream));
        allgather(c, ld.as<double>(), lst.size(), la.as<double>());
        HIPCHK(hipMemcpyAsync(lall.data(), la.p, lall.size() * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    const int32_t ldv = int32_t(S - 64);  // f[ldv]: the rank's ||f||^2 partial (the Lanczos vectors' ld)
    std::vector<int32_t> sidx;
    c->hx_scnt.assign(size_t(R), 0);
    c->hx_soff.assign(size_t(R), 0);
    for (int r = 0; r < R; ++r) {
        if (r == me) continue;
        int64_t o = 0;
        for (int q = 0; q < me; ++q)
            if (q != r) o += Cat(r, q);
        c->hx_soff[size_t(r)] = int64_t(sidx.size());
        c->hx_scnt[size_t(r)] = Cat(r, me);
        for (int64_t k = 0; k < Cat(r, me); ++k) sidx.push_back(int32_t(lall[size_t(r) * size_t(lst.size()) + size_t(o + k)]));
        sidx.push_back(ldv);
    }
    c->hx_nsend = int64_t(sidx.size());
    c->hx_rcnt.assign(size_t(R), 0);
    c->hx_base.assign(size_t(R) + 1, 0);
    std::vector<int32_t> pidx(static_cast<size_t>(R));
    for (int q = 0; q < R; ++q) {
        c->hx_rcnt[size_t(q)] = q == me ? c->nrows : Cat(me, q);
        pidx[size_t(q)] = int32_t(c->hx_base[size_t(q)] + c->hx_rcnt[size_t(q)]);  // q's partial: the block end
        c->hx_base[size_t(q) + 1] = c->hx_base[size_t(q)] + c->hx_rcnt[size_t(q)] + 1;
    }
    // host-staged exchange: q's sbuf lists its messages to r = 0, 1, ... (r != q)
    c->hx_src.assign(size_t(R), 0);
    c->hx_smax = 1;
    for (int q = 0; q < R; ++q) {
        int64_t o = 0;
        for (int r = 0; r < R; ++r) {
            if (r == q) continue;
            if (r == me) c->hx_src[size_t(q)] = o;
            o += Cat(r, q) + 1;
        }
        c->hx_smax = std::max(c->hx_smax, o);
    }
    // the columns, remapped (monotone: rows stay sorted)
    const int64_t base_me = c->hx_base[size_t(me)];
    for (int64_t p = 0; p < nnz; ++p) {
        const int q = int(col[p] / S);
        const int64_t l = col[p] - q * S;
        col[p] = int32_t(q == me ? base_me + l : c->hx_base[size_t(q)] + pos[size_t(q)][size_t(l)]);
    }
    // X's global rows (ek_spmv with a global x)
    c->hx_gidx_h.assign(size_t(c->hx_base.back()), -1);
    for (int q = 0; q < R; ++q) {
        const int64_t b = c->hx_base[size_t(q)];
        if (q == me)
            for (int64_t k = 0; k < c->nrows; ++k) c->hx_gidx_h[size_t(b + k)] = int32_t(c->row0 + k);
        else
            for (size_t k = 0; k < req[size_t(q)].size(); ++k)
                c->hx_gidx_h[size_t(b) + k] = int32_t(off[size_t(q)] + req[size_t(q)][k]);
    }
    if (sidx.empty()) sidx.push_back(0);  // (one forced rank: no messages; a valid upload)
    upload(c->hx_sidx, sidx.data(), sidx.size(), c->stream);
    upload(c->hx_gidx, c->hx_gidx_h.data(), c->hx_gidx_h.size(), c->stream);
    upload(c->hx_pidx, pidx.data(), pidx.size(), c->stream);
    c->hx_sbuf.ensure(size_t(std::max(c->hx_smax, c->hx_nsend)) * 8);
    c->hx_X.ensure(size_t(std::max<int64_t>(c->hx_base.back(), 1)) * 8);
    if (!c->comm) c->hx_gbuf.ensure(size_t(c->hx_smax) * size_t(R) * 8);
    HIPCHK(hipMemsetAsync(c->hx_sbuf.p, 0, c->hx_sbuf.bytes, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->halo = true;
    return true;
}

// One halo exchange of src (this rank's rows, its ||f||^2 partial at
// src[ldv]) into the compact x (c->hx_X), on stream st: the pack (each
// peer's message in sbuf: the rows it reads, closed by this rank's partial;
// the own block and partial straight into X), then ONE RCCL message to and
// one from every peer in one group — block q of X is exactly q's message,
// rows then partial — or, staged through the host, an all-gather of every
// rank's (padded) messages of which this rank copies its one piece per peer
// into the same block.  Counted as the step's one all-gather.
void halo_exchange(ek_ctx* c, const double* src, hipStream_t st) {
    const int R = c->nranks, me = c->rank;
    double* X = c->hx_X.as<double>();
    double* sb = c->hx_sbuf.as<double>();
    const int64_t bme = c->hx_base[size_t(me)];
    ek::dev::halo_pack(st, src, int(c->slot - 64), c->hx_sidx.as<int>(), c->hx_nsend, sb, X, bme, c->nrows,
                       X + bme + c->nrows);
    ++c->hx_exchanges;
    if (c->comm) {
        ++c->n_ag;
        if (R == 1) return;
        const int e = comm_mark(c, st);
        NCCLCHK(ncclGroupStart());
        for (int q = 0; q < R; ++q) {
            if (q == me) continue;
            const int64_t sc = c->hx_scnt[size_t(q)], rc = c->hx_rcnt[size_t(q)];
            NCCLCHK(ncclSend(sb + c->hx_soff[size_t(q)], size_t(sc + 1), ncclDouble, q, c->comm, st));
            NCCLCHK(ncclRecv(X + c->hx_base[size_t(q)], size_t(rc + 1), ncclDouble, q, c->comm, st));
            ++c->hx_sends;
            ++c->hx_recvs;
        }
        NCCLCHK(ncclGroupEnd());
        comm_done(c, e, 0, st);
        return;
    }
    if (R == 1) {
        ++c->n_ag;
        return;
    }
    double* g = c->hx_gbuf.as<double>();
    allgather(c, sb, size_t(c->hx_smax), g, st);
    c->hx_sends += R - 1;  // (this rank's messages ride in its all-gather block)
    for (int q = 0; q < R; ++q)
        if (q != me) {
            const double* m = g + size_t(q) * size_t(c->hx_smax) + c->hx_src[size_t(q)];
            HIPCHK(hipMemcpyAsync(X + c->hx_base[size_t(q)], m, size_t(c->hx_rcnt[size_t(q)] + 1) * 8,
                                  hipMemcpyDeviceToDevice, st));
            ++c->hx_recvs;
        }
}

// The column-panel form when x outgrows an XCD's L2 (EK_SPMV_PANEL=0/1 forces
// it off/on; default: x > 8 MB, the 10x synthetic.  At 2x (3.2 MB) the two
// forms took the same time inside the solve, 29 vs 30 us, and the 1x x
// stays in every L2: tools/panel_lab.py)
bool want_panels(const ek_ctx* c) {
    if (const char* e = std::getenv("EK_SPMV_PANEL"); e && e[0]) return e[0] != '0';
    return x_extent(c) * 8 > (int64_t(8) << 20);
}

// Build the panel layout from this rank's coded CSR on the device (rowptr_d,
// pk_d: (code << colbits) | col words); rowptr_h is the host copy.  False
// when the codes do not fit beside the panel column bits.
bool build_panels(ek_ctx* c, hipStream_t s, const int32_t* rowptr_h, const int32_t* rowptr_d, const uint32_t* pk_d,
                  int colbits, int64_t ncodes) {
    const int64_t X = x_extent(c);
    int pb = 17;  // 1 MB of x per panel (EK_PANEL_PB: lab override)
    if (const char* e = std::getenv("EK_PANEL_PB"); e && std::atoi(e) >= 10 && std::atoi(e) <= 24) pb = std::atoi(e);
    while (((X + (int64_t(1) << pb) - 1) >> pb) > ek::dev::MAX_PANELS) ++pb;
    if (pb >= 32 || ncodes > (int64_t(1) << (32 - pb))) return false;
    const int P = int((X + (int64_t(1) << pb) - 1) >> pb);
    const int64_t nnz = rowptr_h[c->nrows];
    // The most workgroups (<= 8 per CU) that are all resident at once, so they
    // walk the panels together (a straggling second round of workgroups
    // measured 90 -> 124 us at 10x): each holds its rows' accumulators in LDS.
    std::vector<int32_t> wr;
    int G = 0, max_rows = 1;
    for (int per_cu = 8; per_cu >= 1; --per_cu) {
        wr = ek::dev::panel_row_ranges(rowptr_h, c->nrows, per_cu * c->num_cu);
        G = int(wr.size()) - 1;
        max_rows = 1;
        for (int w = 0; w < G; ++w) max_rows = std::max(max_rows, wr[size_t(w) + 1] - wr[size_t(w)]);
        const int fit = int(std::min<size_t>(8, (160 * 1024) / (ek::dev::panel_lds_bytes(max_rows, int(ncodes)) + 1024)));
        if (G <= fit * c->num_cu) break;
    }
    upload(c->pn_wrow, wr.data(), wr.size(), s);
    DBuf cnt, tiles;
    cnt.ensure(size_t(G) * P * 4 + 4);
    tiles.ensure((size_t(G) * P / 1024 + 4) * 8);
    c->pn_start.ensure((size_t(G) * P + 1) * 8);
    c->pn_word.ensure(size_t(std::max<int64_t>(nnz, 1)) * 4);
    c->pn_rid.ensure(size_t(std::max<int64_t>(nnz, 1)) * 2);
    ek::dev::panel_count(s, G, rowptr_d, pk_d, colbits, c->pn_wrow.as<int32_t>(), pb, P, cnt.as<int>());
    ek::dev::exclusive_scan(s, cnt.as<int>(), (long long)G * P, c->pn_start.as<long long>(), tiles.as<long long>());
    ek::dev::panel_fill(s, G, rowptr_d, pk_d, colbits, c->pn_wrow.as<int32_t>(), pb, P, c->pn_start.as<long long>(),
                        c->pn_word.as<uint32_t>(), c->pn_rid.as<uint16_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));  // the temporaries and the host row ranges go out of scope
    c->pn_G = G;
    c->pn_P = P;
    c->pn_pb = pb;
    c->pn_max_rows = max_rows;
    c->pn_ndict = int(ncodes);
    c->nrb_spmv = G;  // the alpha partials: one per workgroup
    c->mat_bytes = nnz * 6 + int64_t(G) * P * 8 + int64_t(wr.size()) * 4 + ncodes * 8;
    return true;
}

// Global column -> the all-gather layout (host copy of k_remap_cols)
void remap_cols_host(const ek_ctx* c, const int32_t* col, int64_t nnz, std::vector<int32_t>& out) {
    out.resize(size_t(nnz));
    const auto& off = c->shard_off;
    ek::parallel_for(nnz, [&](int64_t lo, int64_t hi) {
        for (int64_t p = lo; p < hi; ++p) {
            const int64_t g = col[p];
            const int r = int(std::upper_bound(off.begin() + 1, off.end() - 1, g) - (off.begin() + 1));
            out[size_t(p)] = int32_t(r * c->slot + (g - off[size_t(r)]));
        }
    });
}

// The owned-slot rows of a sharded context (factorize_mr overlaps their SpMV
// with the all-gather): row blocks over the local CSR own_rowptr_h, the
// stream and events of the overlapped step.
void own_finish(ek_ctx* c, const std::vector<int32_t>& orp) {
    auto rbv = ek::dev::spmv_row_blocks(orp.data(), c->nrows, 512);
    c->own_nrb = int(rbv.size() / 4);
    upload(c->own_rb, rbv.data(), rbv.size(), c->stream);
    c->yown.ensure(size_t(std::max<int64_t>(c->nrows, 1)) * 8);
    if (!c->gstream) HIPCHK(hipStreamCreateWithFlags(&c->gstream, hipStreamNonBlocking));
    for (auto& e : c->ag_ev)
        if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->own_ready = true;
}

// ... from the host rows (columns already in the slot layout)
void own_build_host(ek_ctx* c, const int32_t* rowptr, const int32_t* col, const double* val) {
    c->own_ready = false;
    const int64_t lo = c->rank * c->slot, hi = lo + c->nrows;
    std::vector<int32_t> orp(size_t(c->nrows) + 1, 0), oc;
    std::vector<double> ov;
    for (int64_t r = 0; r < c->nrows; ++r) {
        for (int32_t p = rowptr[r]; p < rowptr[r + 1]; ++p)
            if (col[p] >= lo && col[p] < hi) {
                oc.push_back(int32_t(col[p] - lo));
                ov.push_back(val[p]);
            }
        orp[size_t(r) + 1] = int32_t(oc.size());
    }
    c->own_nnz = int64_t(oc.size());
    upload(c->own_rowptr, orp.data(), orp.size(), c->stream);
    upload(c->own_col, oc.data(), std::max<size_t>(oc.size(), 1), c->stream);
    upload(c->own_val, ov.data(), std::max<size_t>(ov.size(), 1), c->stream);
    own_finish(c, orp);
}

// ... from the device rows (ek_spmv_setup_pins: c->rowptr / col / val, columns remapped)
void own_build_dev(ek_ctx* c, hipStream_t s, long long* tiles) {
    c->own_ready = false;
    const int lo = int(c->rank * c->slot), hi = int(lo + c->nrows);
    const size_t nr = size_t(c->nrows);
    DBuf cnt, offs;
    cnt.ensure((nr + 1) * 4);
    offs.ensure((nr + 1) * 8);
    const long long tot = ek::dev::own_split(s, (long long)nr, c->rowptr.as<int>(), c->col.as<int>(),
                                             c->val.as<double>(), lo, hi, cnt.as<int>(), offs.as<long long>(), tiles,
                                             nullptr, nullptr, nullptr);
    c->own_nnz = tot;
    c->own_rowptr.ensure((nr + 1) * 4);
    c->own_col.ensure(size_t(std::max<long long>(tot, 1)) * 4);
    c->own_val.ensure(size_t(std::max<long long>(tot, 1)) * 8);
    ek::dev::own_split(s, (long long)nr, c->rowptr.as<int>(), c->col.as<int>(), c->val.as<double>(), lo, hi,
                       cnt.as<int>(), offs.as<long long>(), tiles, c->own_rowptr.as<int>(), c->own_col.as<int>(),
                       c->own_val.as<double>());
    std::vector<int32_t> orp(nr + 1);
    HIPCHK(hipMemcpyAsync(orp.data(), c->own_rowptr.p, (nr + 1) * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    own_finish(c, orp);
}

// ek_spmv_setup's body, the shard map given; also the device build's host
// fallback, which one rank may take alone.  Sharded, it makes halo_build's
// collectives: a rank that takes the fallback returns before the device
// path's own halo_build, so every rank still makes exactly one call (checked
// there).  A rank that fails before that call leaves its peers in the
// setup's all-gather, as any collective setup does.
void spmv_setup_rows(ek_ctx* c, int64_t n, const std::vector<int64_t>& off, const int32_t* rowptr, const int32_t* col,
                     const double* val) {
    set_shard(c, n, off);
    const int64_t nrows = c->nrows;
    if (rowptr[0] != 0) ek::fail(EK_EINVAL, "ek_spmv_setup: rowptr[0] must be 0 (local rows)");
    ek::PhaseTimer pt("spmv_setup");
    const int64_t nnz = rowptr[nrows];
    for (int64_t r = 0; r < nrows; ++r)
        if (rowptr[r + 1] < rowptr[r]) ek::fail(EK_EINVAL, "ek_spmv_setup: rowptr not monotone");
    for (int64_t p = 0; p < nnz; ++p)
        if (col[p] < 0 || col[p] >= n) ek::fail(EK_EINVAL, "ek_spmv_setup: column %d out of range", col[p]);
    std::vector<int32_t> colx;  // sharded: the columns in the all-gather layout
    c->own_ready = false;
    if (c->mr) {
        remap_cols_host(c, col, nnz, colx);
        col = colx.data();
        own_build_host(c, rowptr, col, val);
        halo_build(c, colx.data(), nnz);  // (the owned rows were taken in the slot layout)
    }
    c->n = n;
    c->nnz = nnz;
    // dictionary-coded entries unless EK_SPMV_PLAIN is set or the values do not fit
    std::vector<uint32_t> pkv;
    std::vector<double> dictv;
    int colbits = 0;
    const char* plain = std::getenv("EK_SPMV_PLAIN");
    pt.mark("validate");
    const bool packed = !(plain && plain[0] && plain[0] != '0') &&
                        ek::dev::spmv_pack(x_extent(c), nnz, col, val, pkv, dictv, colbits);
    pt.mark("pack");
    // 512-nnz blocks (tools/spmv_lab.hip for plain CSR; for the coded form,
    // 1024-nnz segments measured 14.3 against 12.7 us inside the solve)
    c->pn_G = 0;
    if (packed && want_panels(c)) {
        DBuf rp_d, pk_d;
        upload(c->dict, dictv.data(), dictv.size(), c->stream);
        upload(rp_d, rowptr, size_t(nrows) + 1, c->stream);
        upload(pk_d, pkv.data(), pkv.size(), c->stream);
        if (build_panels(c, c->stream, rowptr, rp_d.as<int32_t>(), pk_d.as<uint32_t>(), colbits, int64_t(dictv.size()))) {
            c->colbits = colbits;
            c->pk.reset();
            c->rel.reset();
            c->col.reset();
            c->val.reset();
            c->rowptr.reset();
            c->rb.reset();
            pt.mark("panels");
            return;
        }
    }
    c->block_nnz = ek::dev::SPMV_SEG_NNZ;  // (coded or plain: the same row blocks, so the same sums)
    auto rbv = ek::dev::spmv_row_blocks(rowptr, nrows, c->block_nnz);
    c->nrb_spmv = int(rbv.size() / 4);
    c->spmv_long = false;
    for (size_t bk = 0; bk < rbv.size() / 4; ++bk) c->spmv_long = c->spmv_long || rbv[4 * bk + 3] > c->block_nnz;
    c->colbits = packed ? colbits : 0;
    if (packed) {
        std::vector<uint32_t> segv;
        std::vector<uint16_t> relv;
        pt.mark("row blocks");
        ek::dev::spmv_segment(rbv, rowptr, pkv, c->block_nnz, segv, relv);  // long rows: desc nnz0 -> overflow area
        pt.mark("segments");
        upload(c->pk, segv.data(), segv.size(), c->stream);
        upload(c->rel, relv.data(), relv.size(), c->stream);
        upload(c->dict, dictv.data(), dictv.size(), c->stream);
        c->mat_bytes = int64_t(segv.size() * 4 + relv.size() * 2 + dictv.size() * 8 + rbv.size() * 4);
        c->col.reset();
        c->val.reset();
        c->rowptr.reset();
    } else {
        upload(c->rowptr, rowptr, size_t(nrows) + 1, c->stream);
        upload(c->col, col, size_t(nnz), c->stream);
        upload(c->val, val, size_t(nnz), c->stream);
        c->mat_bytes = 12 * nnz + 4 * (nrows + 1);
        c->pk.reset();
        c->rel.reset();
        c->dict.reset();
    }
    upload(c->rb, rbv.data(), rbv.size(), c->stream);
    HIPCHK(hipStreamSynchronize(c->stream));
    pt.mark("upload");
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------------------
// SpMV seam (SparseSymMatProd::perform_op, cEIG.cpp:194)
// Sharded: the ranks' row ranges are learned with one all-gather of
// (row0, nrows) over the comm seam and must tile [0, n) in rank order (equal
// blocks from ek_shard_rows or the nnz-balanced ek_shard_map alike).
int ek_spmv_setup(ek_ctx* c, int64_t n, int64_t row0, int64_t nrows, const int32_t* rowptr, const int32_t* col,
                  const double* val) {
    EK_TRY
    check_ctx(c);
    if (n <= 0 || row0 < 0 || nrows < 0 || row0 + nrows > n || !rowptr || (nrows && (!col || !val)))
        ek::fail(EK_EINVAL, "ek_spmv_setup: bad argument");
    std::vector<int64_t> off{0, n};
    if (c->mr) {
        c->scal.ensure(64);
        c->xexp.ensure(size_t(2 * c->nranks) * 8);
        const double mine[2] = {double(row0), double(nrows)};
        HIPCHK(hipMemcpyAsync(c->scal.p, mine, 16, hipMemcpyHostToDevice, c->stream));
        allgather(c, c->scal.as<double>(), 2, c->xexp.as<double>());
        std::vector<double> all(size_t(2 * c->nranks));
        HIPCHK(hipMemcpyAsync(all.data(), c->xexp.p, all.size() * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        off.assign(size_t(c->nranks) + 1, 0);
        for (int r = 0; r < c->nranks; ++r) {
            if (int64_t(all[size_t(2 * r)]) != off[size_t(r)])
                ek::fail(EK_EINVAL, "ek_spmv_setup: rank %d's rows start at %lld, not where rank %d's end (%lld)", r,
                         (long long)all[size_t(2 * r)], r - 1, (long long)off[size_t(r)]);
            off[size_t(r) + 1] = off[size_t(r)] + int64_t(all[size_t(2 * r) + 1]);
        }
        if (off.back() != n) ek::fail(EK_EINVAL, "ek_spmv_setup: the ranks' rows cover %lld of %lld", (long long)off.back(), (long long)n);
    } else if (row0 != 0 || nrows != n) {
        ek::fail(EK_EINVAL, "ek_spmv_setup: a single context owns all %lld rows", (long long)n);
    }
    spmv_setup_rows(c, n, off, rowptr, col, val);
    return EK_OK;
    EK_CATCH
}

int ek_spmv_dims(ek_ctx* c, int64_t* n, int64_t* row0, int64_t* nrows) {
    EK_TRY
    check_ctx(c);
    if (n) *n = c->n;
    if (row0) *row0 = c->row0;
    if (nrows) *nrows = c->nrows;
    return EK_OK;
    EK_CATCH
}

// the body of ek_spmv_setup_pins; trusted_raw >= 0: the pins come from an
// ek_hgr (every constructor validates them: ranges, monotone offsets) whose
// reader counted the raw entries, so the two input scans (~0.25 ms at the
// headline, bound by reading 4.3 MB) are skipped
static int spmv_setup_pins_impl(ek_ctx* c, int64_t n, int64_t nets, const int64_t* net_ptr, const int32_t* pins,
                                int32_t* on_device, int64_t trusted_raw) {
    EK_TRY
    check_ctx(c);
    if (n <= 0 || n > INT32_MAX || nets < 0 || !net_ptr || (net_ptr[nets] > 0 && !pins) || net_ptr[0] != 0)
        ek::fail(EK_EINVAL, "ek_spmv_setup_pins: bad argument");
    const int64_t npins = net_ptr[nets];
    if (npins > INT32_MAX) ek::fail(EK_EINVAL, "ek_spmv_setup_pins: too many pins");
    ek::PhaseTimer pt("spmv_setup_pins");
    // (both scans branch-free; the error paths re-scan)
    int64_t raw_bound = trusted_raw;  // raw entries: every pin of a net of k >= 2 pins sees k - 1 others
    if (trusted_raw < 0) {
        raw_bound = 0;
        bool non_monotone = false;
        for (int64_t e = 0; e < nets; ++e) {
            const int64_t k = net_ptr[e + 1] - net_ptr[e];
            non_monotone |= k < 0;
            raw_bound += k >= 2 ? k * (k - 1) : 0;
        }
        if (non_monotone) ek::fail(EK_EINVAL, "ek_spmv_setup_pins: net_ptr not monotone");
    }
    // this rank's rows: the nnz-balanced shard map, computed from the pins
    // identically on every rank (no collective)
    std::vector<int64_t> off(size_t(c->nranks) + 1, 0);
    off[1] = n;
    if (c->mr) {
        const int rc = ek_shard_map(n, nets, net_ptr, pins, c->nranks, off.data());
        if (rc != EK_OK) throw ek::Error{rc};
    }
    const int64_t row0 = off[size_t(c->rank)], nrows = off[size_t(c->rank) + 1] - row0;
    pt.mark("raw bound, shard map");
    hipStream_t s = c->stream;
    auto host_fallback = [&](const char* why) {
        if (std::getenv("EK_TRACE")) std::fprintf(stderr, "[spmv_setup_pins] host build: %s\n", why);
        ek_hgr h;
        h.nets = nets;
        h.nodes = n;
        h.net_ptr.assign(net_ptr, net_ptr + nets + 1);
        h.pins.assign(pins, pins + npins);
        ek_csr L;
        ek::build_laplacian_rows(h, row0, row0 + nrows, L);
        spmv_setup_rows(c, n, off, L.rowptr.data(), L.col.data(), L.val64.data());
        if (on_device) *on_device = 0;
    };
    if (std::getenv("EK_HOST_LAPLACIAN")) {
        host_fallback("EK_HOST_LAPLACIAN");
        return EK_OK;
    }
    if (trusted_raw < 0) {
        int32_t lo = INT32_MAX, hi = INT32_MIN;
        for (int64_t p = 0; p < npins; ++p) {
            lo = std::min(lo, pins[p]);
            hi = std::max(hi, pins[p]);
        }
        if (npins > 0 && (lo < 0 || int64_t(hi) >= n))
            for (int64_t p = 0; p < npins; ++p)  // the first offender, for the message
                if (pins[p] < 0 || pins[p] >= n) ek::fail(EK_EINVAL, "ek_spmv_setup_pins: pin %d out of range", pins[p]);
    }
    pt.mark("input checks");
    {
        Uploader up(c, s, (size_t(nets) + 1) * 8 + size_t(std::max<int64_t>(npins, 1)) * 4);
        up.put(c->lb_netptr, net_ptr, size_t(nets) + 1);
        up.put(c->lb_pins, pins, size_t(std::max<int64_t>(npins, 1)));
    }
    pt.mark("pins staged");
    const size_t nr = size_t(nrows);
    ek::dev::LapBuild b;
    b.nets = nets;
    b.r0 = row0;
    b.r1 = row0 + nrows;
    b.net_ptr = c->lb_netptr.as<int64_t>();
    b.pins = c->lb_pins.as<int32_t>();
    c->lb_icnt.ensure((nr + 1) * 4);
    c->lb_rcnt.ensure((nr + 1) * 4);
    c->lb_cur.ensure((nr + 1) * 4);
    c->lb_cnt.ensure(16);
    HIPCHK(hipMemsetAsync(c->lb_icnt.p, 0, (nr + 1) * 4, s));
    HIPCHK(hipMemsetAsync(c->lb_rcnt.p, 0, (nr + 1) * 4, s));
    HIPCHK(hipMemsetAsync(c->lb_cur.p, 0, (nr + 1) * 4, s));
    HIPCHK(hipMemsetAsync(c->lb_cnt.p, 0, 16, s));
    c->lb_ip.ensure((nr + 1) * 8);
    c->lb_rp.ensure((nr + 1) * 8);
    c->lb_off.ensure((nr + 1) * 8);
    constexpr int TSIZE = 1 << 16;  // dictionary table slots (power of two)
    c->lb_tiles.ensure((std::max<size_t>(nr, TSIZE) / 1024 + 2) * 8);
    c->lb_inc.ensure(size_t(std::max<int64_t>(npins, 1)) * 8);
    const size_t raw = size_t(std::max<int64_t>(raw_bound, 1));
    c->lb_scol.ensure(raw * 4);
    c->lb_sval.ensure(raw * 8);
    c->lb_tval.ensure(raw * 8);
    c->lb_ulen.ensure((nr + 1) * 4);
    c->lb_len.ensure((nr + 1) * 4);
    c->lb_diag.ensure((nr + 1) * 8);
    c->lb_long.ensure((nr + 1) * 4);
    b.icnt = c->lb_icnt.as<int>();
    b.rcnt = c->lb_rcnt.as<int>();
    b.cur = c->lb_cur.as<int>();
    b.ip = c->lb_ip.as<long long>();
    b.rp = c->lb_rp.as<long long>();
    b.inc = c->lb_inc.as<int32_t>();
    b.scol = c->lb_scol.as<int>();
    b.sval = c->lb_sval.as<double>();
    b.tval = c->lb_tval.as<double>();
    b.ulen = c->lb_ulen.as<int>();
    b.len = c->lb_len.as<int>();
    b.diag = c->lb_diag.as<double>();
    b.long_rows = c->lb_long.as<int>();
    b.counters = c->lb_cnt.as<int>();
    long long* tiles = c->lb_tiles.as<long long>();
    ek::dev::lap_count(s, b);
    ek::dev::exclusive_scan(s, b.icnt, int64_t(nr), b.ip, tiles);
    ek::dev::exclusive_scan(s, b.rcnt, int64_t(nr), b.rp, tiles);
    ek::dev::lap_fill_rows(s, b);
    int cnt_h[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(cnt_h, b.counters, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    ek::dev::lap_long_rows(s, b, cnt_h[0]);
    ek::dev::exclusive_scan(s, b.len, int64_t(nr), c->lb_off.as<long long>(), tiles);
    // CSR on the device: rowptr (local), col, val; at most raw + nrows entries
    c->rowptr.ensure((nr + 1) * 4);
    c->col.ensure((raw + nr) * 4);
    c->val.ensure((raw + nr) * 8);
    ek::dev::lap_write(s, b, c->lb_off.as<long long>(), c->rowptr.as<int>(), c->col.as<int>(), c->val.as<double>());
    std::vector<int32_t> rowptr(nr + 1);
    HIPCHK(hipMemcpyAsync(rowptr.data(), c->rowptr.p, (nr + 1) * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(cnt_h, b.counters, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    pt.mark("rows on device");
    if (cnt_h[1] > 0) {
        host_fallback("a row longer than the LDS sort");
        return EK_OK;
    }
    const int64_t nnz = rowptr[nr];
    set_shard(c, n, off);
    c->n = n;
    c->nnz = nnz;
    const std::vector<long long> offll(off.begin(), off.end());  // (alive until the stream is drained below)
    c->own_ready = false;
    if (c->mr) {  // global columns -> the all-gather layout (monotone: rows stay sorted)
        upload(c->off_d, offll.data(), offll.size(), s);
        ek::dev::remap_cols(s, nnz, c->col.as<int>(), c->off_d.as<long long>(), c->nranks, c->slot);
        own_build_dev(c, s, tiles);
        // the halo layout is worked out on the host from this rank's columns
        std::vector<int32_t> ch(size_t(std::max<int64_t>(nnz, 1)));
        if (nnz) HIPCHK(hipMemcpyAsync(ch.data(), c->col.p, size_t(nnz) * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (halo_build(c, ch.data(), nnz) && nnz)
            HIPCHK(hipMemcpyAsync(c->col.p, ch.data(), size_t(nnz) * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
        pt.mark("halo layout");
    }
    // the same greedy row blocks as the host path (ek_spmv_setup)
    int colbits = 1;
    while (colbits < 31 && (int64_t(1) << colbits) < x_extent(c)) ++colbits;
    const char* plain_env = std::getenv("EK_SPMV_PLAIN");
    bool packed = !(plain_env && plain_env[0] && plain_env[0] != '0') && colbits <= 28;
    int64_t ncodes = 0;
    if (packed) {
        c->lb_table.ensure(size_t(TSIZE) * 8);
        c->lb_flags.ensure(size_t(TSIZE) * 4);
        c->lb_codes.ensure((size_t(TSIZE) + 1) * 8);
        ek::dev::dict_build(s, nnz, c->val.as<double>(), c->lb_table.as<unsigned long long>(), TSIZE,
                            b.counters + 1, c->lb_flags.as<int>(), c->lb_codes.as<long long>(), tiles);
        long long nd = 0;
        HIPCHK(hipMemcpyAsync(&nd, c->lb_codes.as<long long>() + TSIZE, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(cnt_h, b.counters, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        ncodes = nd;
        packed = cnt_h[1] == 0 && nd <= TSIZE / 2 && nd <= (int64_t(1) << (32 - colbits));
    }
    c->pn_G = 0;
    if (packed && want_panels(c)) {
        DBuf pk_d;
        c->dict.ensure(size_t(std::max<int64_t>(ncodes, 1)) * 8);
        ek::dev::dict_values(s, c->lb_table.as<unsigned long long>(), TSIZE, c->lb_codes.as<long long>(),
                             c->dict.as<double>());
        pk_d.ensure(size_t(std::max<int64_t>(nnz, 1)) * 4);
        ek::dev::encode_words(s, nnz, c->col.as<int>(), c->val.as<double>(), c->lb_table.as<unsigned long long>(), TSIZE,
                              c->lb_codes.as<long long>(), colbits, pk_d.as<uint32_t>());
        if (build_panels(c, s, rowptr.data(), c->rowptr.as<int32_t>(), pk_d.as<uint32_t>(), colbits, ncodes)) {
            c->colbits = colbits;
            pt.mark("panels");
            if (on_device) *on_device = 1;
            return EK_OK;
        }
    }
    c->block_nnz = ek::dev::SPMV_SEG_NNZ;  // (coded or plain: the same row blocks, so the same sums)
    auto rbv = ek::dev::spmv_row_blocks(rowptr.data(), nrows, c->block_nnz);
    c->nrb_spmv = int(rbv.size() / 4);
    c->spmv_long = false;
    for (size_t bk = 0; bk < rbv.size() / 4; ++bk) c->spmv_long = c->spmv_long || rbv[4 * bk + 3] > c->block_nnz;
    if (packed) {
        const size_t nb = size_t(c->nrb_spmv), SEG = size_t(ek::dev::SPMV_SEG_NNZ);
        size_t over = 0;  // long rows: overflow area after the segments (spmv_segment's layout)
        for (size_t bk = 0; bk < nb; ++bk)
            if (size_t(rbv[4 * bk + 3]) > SEG) {
                rbv[4 * bk + 2] = int32_t(nb * SEG + over);
                over += size_t(rbv[4 * bk + 3]);
            }
        c->pk.ensure((nb * SEG + over) * 4);
        c->rel.ensure(nb * ek::dev::SPMV_REL_STRIDE * 2);
        c->dict.ensure(size_t(std::max<int64_t>(ncodes, 1)) * 8);
        upload(c->rb, rbv.data(), rbv.size(), s);
        ek::dev::dict_values(s, c->lb_table.as<unsigned long long>(), TSIZE, c->lb_codes.as<long long>(),
                             c->dict.as<double>());
        ek::dev::encode_segments(s, int(nb), c->rb.as<int32_t>(), c->rowptr.as<int>(), c->col.as<int>(),
                                 c->val.as<double>(), c->lb_table.as<unsigned long long>(), TSIZE,
                                 c->lb_codes.as<long long>(), colbits, c->pk.as<uint32_t>(), c->rel.as<uint16_t>());
        c->colbits = colbits;
        c->mat_bytes = int64_t((nb * SEG + over) * 4 + nb * ek::dev::SPMV_REL_STRIDE * 2 + size_t(ncodes) * 8 +
                               rbv.size() * 4);
    } else {
        upload(c->rb, rbv.data(), rbv.size(), s);
        c->colbits = 0;
        c->mat_bytes = 12 * nnz + 4 * (nrows + 1);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    pt.mark("blocks + coding");
    if (on_device) *on_device = 1;
    return EK_OK;
    EK_CATCH
}

int ek_spmv_setup_pins(ek_ctx* c, int64_t n, int64_t nets, const int64_t* net_ptr, const int32_t* pins,
                       int32_t* on_device) {
    return spmv_setup_pins_impl(c, n, nets, net_ptr, pins, on_device, -1);
}

// x is the global n-vector; a sharded context reads it through its padded
// all-gather layout, so the ranks' slices are copied into that first (into a
// buffer of its own, not the solve's scratch: one ek_spmv at a time per
// sharded context, on any stream)
int ek_spmv(ek_ctx* c, const double* x, double* y, void* stream) {
    EK_TRY
    check_ctx(c);
    if (!c->n) ek::fail(EK_ESTATE, "ek_spmv before ek_spmv_setup");
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
    const double* xs = x;
    if (c->halo) {  // the compact halo layout, gathered from the global x
        if (c->spx.bytes < size_t(x_extent(c)) * 8) ek::fail(EK_ESTATE, "ek_spmv: shard layout not set up");
        ek::dev::gather_idx(s, x, c->hx_gidx.as<int>(), (long long)x_extent(c), c->spx.as<double>());
        xs = c->spx.as<double>();
    } else if (c->mr) {
        if (c->spx.bytes < size_t(x_extent(c)) * 8) ek::fail(EK_ESTATE, "ek_spmv: shard layout not set up");
        for (int r = 0; r < c->nranks; ++r) {
            const int64_t a = c->shard_off[size_t(r)], b = c->shard_off[size_t(r) + 1];
            if (b > a)
                HIPCHK(hipMemcpyAsync(c->spx.as<double>() + r * c->slot, x + a, size_t(b - a) * 8,
                                      hipMemcpyDeviceToDevice, s));
        }
        xs = c->spx.as<double>();
    }
    ek::dev::spmv(s, spmv_mat(c), xs, y, nullptr, nullptr, nullptr, nullptr);
    HIPCHK(hipGetLastError());
    return EK_OK;
    EK_CATCH
}

int ek_spmv_host(ek_ctx* c, const double* x, double* y) {
    EK_TRY
    check_ctx(c);
    if (!c->n) ek::fail(EK_ESTATE, "ek_spmv_host before ek_spmv_setup");
    DBuf dx, dy;
    std::vector<double> xp;  // sharded: the padded all-gather layout (or the halo layout)
    if (c->halo) {
        xp.assign(size_t(x_extent(c)), 0.0);
        for (size_t t = 0; t < xp.size(); ++t)
            if (c->hx_gidx_h[t] >= 0) xp[t] = x[c->hx_gidx_h[t]];
        x = xp.data();
    } else if (c->mr) {
        xp.assign(size_t(x_extent(c)), 0.0);
        for (int r = 0; r < c->nranks; ++r)
            std::copy(x + c->shard_off[size_t(r)], x + c->shard_off[size_t(r) + 1], xp.begin() + r * c->slot);
        x = xp.data();
    }
    upload(dx, x, size_t(x_extent(c)), c->stream);
    dy.ensure(size_t(std::max<int64_t>(c->nrows, 1)) * 8);
    ek::dev::spmv(c->stream, spmv_mat(c), dx.as<double>(), dy.as<double>(), nullptr, nullptr, nullptr, nullptr);
    HIPCHK(hipGetLastError());
    if (c->nrows) HIPCHK(hipMemcpyAsync(y, dy.p, size_t(c->nrows) * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return EK_OK;
    EK_CATCH
}

int ek_spmv_gather_bench(ek_ctx* c, int iters, double* avg_us) {
    EK_TRY
    check_ctx(c);
    if (!c->n) ek::fail(EK_ESTATE, "ek_spmv_gather_bench before ek_spmv_setup");
    if (iters <= 0 || !avg_us) ek::fail(EK_EINVAL, "ek_spmv_gather_bench: bad argument");
    hipStream_t s = c->stream;
    const size_t X = size_t(x_extent(c));
    DBuf x, sink;
    x.ensure(X * 8);
    sink.ensure(size_t(std::max(std::max(c->nrb_spmv, c->pn_G), 1)) * 8);
    std::vector<double> h(X);
    for (size_t i = 0; i < X; ++i) h[i] = double((i * 2654435761u) % 1000u) / 1000.0 - 0.5;
    HIPCHK(hipMemcpyAsync(x.p, h.data(), X * 8, hipMemcpyHostToDevice, s));
    const auto m = spmv_mat(c);
    // EK_GATHER_MODE (lab, kernels_spmv.hip k_lab_gather_step): 1 the gather +
    // a skipped step's update as two launches, 2 as one grid with an in-launch
    // wait, 3 the update alone; 0 (default) the gather-only ceiling
    const char* gm = std::getenv("EK_GATHER_MODE");
    const int mode = gm ? std::atoi(gm) : 0;
    DBuf part, ctr, wv, fv, fpart;
    const int R = int(std::max<int64_t>(c->nrows, 1));
    if (mode) {
        if (mode < 0 || mode > 3 || !m.pk || m.panel.G > 0 || c->mr)
            ek::fail(EK_EINVAL, "EK_GATHER_MODE %d: the single-context coded CSR form only", mode);
        if (mode == 2 && m.nblocks > ek::dev::lab_step_capacity())
            ek::fail(EK_EINVAL, "EK_GATHER_MODE 2: %d blocks exceed the %d resident at once", m.nblocks,
                     ek::dev::lab_step_capacity());
        part.ensure(size_t(m.nblocks) * 8);
        ctr.ensure(66 * 64 * 4);
        wv.ensure(size_t(R) * 3 * 8);
        fv.ensure(size_t(R) * 8);
        fpart.ensure(size_t(m.nblocks) * 8);
        HIPCHK(hipMemsetAsync(part.p, 0, part.bytes, s));
        HIPCHK(hipMemsetAsync(ctr.p, 0, ctr.bytes, s));
        HIPCHK(hipMemsetAsync(wv.p, 0, wv.bytes, s));
    }
    unsigned gen = 0;
    auto launch = [&] {
        if (!mode) return ek::dev::spmv_gather_only(s, m, x.as<double>(), sink.as<double>());
        ++gen;
        const double* w = wv.as<double>();
        ek::dev::lab_gather_step(s, m, mode, x.as<double>(), part.as<double>(), ctr.as<unsigned>(),
                                 gen, R, w, w + R, w + 2 * size_t(R), fv.as<double>(),
                                 fpart.as<double>());
    };
    for (int i = 0; i < 10; ++i) launch();
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, s));
    for (int i = 0; i < iters; ++i) launch();
    HIPCHK(hipEventRecord(e1, s));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    HIPCHK(hipGetLastError());
    *avg_us = 1e3 * double(ms) / iters;
    return EK_OK;
    EK_CATCH
}

int ek_spmv_bench(ek_ctx* c, int iters, int fused, double* avg_us) {
    EK_TRY
    check_ctx(c);
    if (!c->n) ek::fail(EK_ESTATE, "ek_spmv_bench before ek_spmv_setup");
    if (iters <= 0 || !avg_us) ek::fail(EK_EINVAL, "ek_spmv_bench: bad argument");
    // (a sharded context: this rank's rows over the padded all-gather layout,
    // x synthetic in every slot; no collective — bench.py's per-shard leg)
    hipStream_t s = c->stream;
    const size_t X = size_t(x_extent(c)), R = size_t(std::max<int64_t>(c->nrows, 1));
    DBuf x, y, vcol, apart, fn2;
    x.ensure(X * 8);
    y.ensure(R * 8);
    vcol.ensure(R * 8);
    apart.ensure(size_t(std::max(c->nrb_spmv, 1)) * 8);
    fn2.ensure(8);
    std::vector<double> h(X);
    for (size_t i = 0; i < X; ++i) h[i] = double((i * 2654435761u) % 1000u) / 1000.0 - 0.5;
    double nrm = 0.0;
    for (double v : h) nrm += v * v;
    HIPCHK(hipMemcpyAsync(x.p, h.data(), X * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(fn2.p, &nrm, 8, hipMemcpyHostToDevice, s));
    // this rank's rows of x
    const double* fsrc = x.as<double>() + (c->halo ? size_t(c->hx_base[size_t(c->rank)]) : c->mr ? size_t(c->rank * c->slot) : 0);
    // fused == 2: also the Lanczos step's finalize folded into the prologue
    // (||f||^2 from the update's one value, block 0 publishing alpha / offd)
    // and the ||w||^2 partials of partial reorthogonalisation: the SpMV exactly
    // as the solve launches it
    DBuf scratch, wp;
    ek::dev::StepFin fin;
    if (fused == 2) {
        scratch.ensure(64 * 8);
        wp.ensure(size_t(std::max(c->nrb_spmv, 1)) * 8);
        std::vector<double> sv(64, 0.0);
        sv[0] = nrm;   // fast: ||f||^2
        sv[1] = nrm;   // fn2_i
        sv[2] = 0.5;   // a3
        sv[3] = std::nan("");  // bov (no override)
        HIPCHK(hipMemcpyAsync(scratch.p, sv.data(), 64 * 8, hipMemcpyHostToDevice, s));
        double* sc = scratch.as<double>();
        fin.npart = sc + 40;
        fin.nb = 1;
        fin.fast = sc;
        fin.fn2_out = sc + 8;
        fin.h2 = sc + 16;
        fin.step = 1;
        fin.alpha = sc + 24;
        fin.offd = sc + 32;
        fin.a3 = sc + 2;
        fin.fn2_i = sc + 1;
        fin.bov_i = sc + 3;
        fin.wpart = wp.as<double>();
    }
    auto launch = [&] {
        if (fused)
            ek::dev::spmv(s, spmv_mat(c), x.as<double>(), y.as<double>(), fn2.as<double>(), fsrc,
                          vcol.as<double>(), apart.as<double>(), fused == 2 ? &fin : nullptr);
        else
            ek::dev::spmv(s, spmv_mat(c), x.as<double>(), y.as<double>(), nullptr, nullptr, nullptr, nullptr);
    };
    for (int i = 0; i < 10; ++i) launch();
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, s));
    for (int i = 0; i < iters; ++i) launch();
    HIPCHK(hipEventRecord(e1, s));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    HIPCHK(hipGetLastError());
    *avg_us = 1e3 * double(ms) / iters;
    return EK_OK;
    EK_CATCH
}

int64_t ek_spmv_bytes(ek_ctx* c) {
    if (!c) return 0;
    return 12 * c->nnz + 4 * (c->nrows + 1) + 8 * c->n + 8 * c->nrows;
}

int ek_spmv_format(ek_ctx* c, int32_t* packed, int64_t* stored_bytes) {
    EK_TRY
    check_ctx(c);
    if (!c->n) ek::fail(EK_ESTATE, "ek_spmv_format before ek_spmv_setup");
    // coded: segments (padding included) + row starts + table + descriptors; plain: CSR
    const int64_t mat = c->mat_bytes;
    if (packed) *packed = c->colbits > 0 ? 1 : 0;
    if (stored_bytes) *stored_bytes = mat + 8 * c->n + 8 * c->nrows;
    return EK_OK;
    EK_CATCH
}

int ek_comm_stats(ek_ctx* c, int64_t* exchanges, int64_t* sends, int64_t* recvs, double* exchange_ms,
                  int64_t* exchanges_timed, double* allreduce_ms, int64_t* allreduces_timed) {
    EK_TRY
    check_ctx(c);
    if (exchanges) *exchanges = c->hx_exchanges;
    if (sends) *sends = c->hx_sends;
    if (recvs) *recvs = c->hx_recvs;
    if (exchange_ms) *exchange_ms = c->x_ms;
    if (exchanges_timed) *exchanges_timed = c->x_timed;
    if (allreduce_ms) *allreduce_ms = c->ar_ms;
    if (allreduces_timed) *allreduces_timed = c->ar_timed;
    return EK_OK;
    EK_CATCH
}

int ek_spmv_exchange(ek_ctx* c, int32_t* halo, int64_t* recv_doubles, int64_t* send_doubles) {
    EK_TRY
    check_ctx(c);
    if (!c->n) ek::fail(EK_ESTATE, "ek_spmv_exchange before ek_spmv_setup");
    int64_t rv = 0, sd = 0;
    if (c->halo) {
        for (int q = 0; q < c->nranks; ++q)
            if (q != c->rank) {
                rv += c->hx_rcnt[size_t(q)] + 1;
                sd += c->hx_scnt[size_t(q)] + 1;
            }
    } else if (c->mr) {
        rv = (c->nranks - 1) * c->slot;
        sd = (c->nranks - 1) * c->slot;
    }
    if (halo) *halo = c->halo ? 1 : 0;
    if (recv_doubles) *recv_doubles = rv;
    if (send_doubles) *send_doubles = sd;
    return EK_OK;
    EK_CATCH
}

// ---------------------------------------------------------------------------
// Lanczos (Spectra SymEigsSolver restated, cEIG.cpp:194-207)
void ek_lanczos_default_opts(ek_lanczos_opts* o) {
    if (!o) return;
    o->ncv = 0;
    o->maxit = 1000;
    o->tol = 1e-10;
    o->deflate = 1;
    o->time_spmv = 0;
    o->reorth = 3;
    o->check_every = 8;
    o->basis32 = 1;
    o->alpha_last = 0;
    o->keep_min = -1;
    o->reorth_thresh = 0.0;
}

}  // extern "C"

namespace ek {
// ek_spmv_setup_pins for an ek_hgr's pins (valid by construction), with the
// raw-entry count its reader made when known
int spmv_setup_hgr(ek_ctx* c, const ek_hgr& h, int32_t* on_device) {
    return spmv_setup_pins_impl(c, h.nodes, h.nets, h.net_ptr.data(), h.pins.data(), on_device, h.raw_pairs);
}
}  // namespace ek

namespace {

// Spectra SymEigsBase::nev_adjusted (ARPACK dsaup2's count of converged
// unwanted values).  "Converged" = |last component| < machine epsilon: with
// the 10 x DBL_MIN bound (an exact-zero test) the restarts kept 50 vectors
// and ibm10 took 11,006 matvecs instead of 1,201, the 1x synthetic 2,683
// instead of 507 (tools/lanczos_trace.py)
// arpack_half: ARPACK's (and Spectra's) jump to ncv/2 kept vectors when
// nothing else counts (false: the caller's floor decides instead)
int nev_adjusted(int nev, int ncv, int nconv, const std::vector<double>& est, bool arpack_half = true) {
    const double eps = std::numeric_limits<double>::epsilon();
    int nev_new = nev;
    for (int i = nev; i < ncv; ++i)
        if (std::fabs(est[size_t(i)]) < eps) ++nev_new;
    nev_new += std::min(nconv, (ncv - nev_new) / 2);
    if (arpack_half && nev_new == 1 && ncv >= 6) nev_new = ncv / 2;
    else if (arpack_half && nev_new == 1 && ncv > 2) nev_new = 2;
    if (nev_new > ncv - 1) nev_new = ncv - 1;
    return nev_new;
}

struct Lanczos {
    ek_ctx* c;
    hipStream_t s;
    int m, ldv, nrb, nub, has_u0, nreal;
    double u0val;
    bool time_spmv;
    std::vector<hipEvent_t> ev;
    double spmv_ms = 0.0;
    int spmv_timed = 0, matvecs = 0;

    double* V() { return c->V.as<double>(); }
    double* col(int j) { return V() + size_t(j) * ldv; }

    // x for the matvec: the full vector (gathered when sharded, in the padded
    // slot layout the matrix's columns were remapped to)
    const double* gather_f() {
        if (!c->mr) return c->f.as<double>();
        if (c->halo) {
            halo_exchange(c, c->f.as<double>(), s);
            return c->hx_X.as<double>();
        }
        allgather(c, c->f.as<double>(), size_t(c->slot), c->xfull.as<double>());
        return c->xfull.as<double>();
    }

    void reduce_scalar(double* dst) {  // dst = allreduce(sum npart[0:nub])
        ek::dev::finalize_step(s, c->npart.as<double>(), nub, dst, nullptr, nullptr, -1, nullptr, nullptr);
        allreduce(c, dst, 1);
    }

    // Lanczos steps i = k .. m-1 (Spectra Lanczos::factorize_from), with the
    // deflated constant vector u0 in every projection.
    //   reorth 1: three-term recurrence f' = w - alpha v_i - beta_i v_{i-1}
    //             (alpha from the SpMV's fused partials), then ONE classical
    //             Gram-Schmidt pass f = f' - V (V^T f'): 2 passes over V;
    //   reorth 2: CGS2 from w (twice is enough): 4 passes over V.
    // H(i,i) / H(i-1,i) take the projections as corrections (Spectra's
    // H += V^T f after its re-orthogonalisation).
    int reorth = 1;
    // the update reads the fp32 shadow V32 (single-context fused step; k_update B32)
    bool b32 = false;
    // alpha reduced by the SpMV's last workgroup (else by every projection workgroup)
    bool alpha_last = true;
    // the basis passes read V (and V32) non-temporally: a basis larger than
    // the MALL would otherwise evict the matrix and x every pass
    bool nt = false;
    int u32_steps = 0;
    // partial reorthogonalisation (reorth 3, single context): k_pro decides
    // per step whether the projection and the update run (Simon's omega
    // recurrence against thresh; eps1 = eps sqrt(n), its rounding term)
    bool pro = false;
    double pro_thresh = 0.0, pro_eps1 = 0.0;
    int pro_cgw = 0;  // ProLaunch::cgw (EK_PRO_CGW)
    bool pro_cgw_env = false;  // EK_PRO_CGW set: no fitting to the resident grid
    // the decision inside the projection launch (no k_pro launch; needs the
    // projection's hand-off, upd_red 2).  EK_PRO_INLAUNCH=0: the k_pro launch
    bool proi = false;
    // ... and the update's workgroups in the projection launch (no update
    // launch: a skipped step is two launches).  EK_PRO_MERGE=0: its own launch
    bool pro_merge = false;
    unsigned* pro_pub() { return reinterpret_cast<unsigned*>(c->pflags.as<char>() + pro_pub_off()); }
    size_t pro_pub_off() const { return (size_t(m + 2) * 4 + 255) / 256 * 256; }
    float* V32() { return b32 ? c->V32.as<float>() : nullptr; }
    float* col32(int j) { return b32 ? c->V32.as<float>() + size_t(j) * ldv : nullptr; }
    int seg0 = 0;  // first step of the current run of steps (cycle start or injected vector)
    // a mid-cycle check wanted at the end of the next factorize() chunk
    // (chk_dst != null): factorize_fused folds its copy into the chunk's last
    // SpMV (StepFin::chk_*) and sets chk_folded; other forms leave it to the
    // k_chk_gather launch
    double* chk_dst = nullptr;
    unsigned* chk_word = nullptr;
    const unsigned* chk_seq_src = nullptr;
    int chk_b = 0;
    bool chk_folded = false;
    // steps [k, kend) of a run that started at seg0 (the driver enqueues a
    // cycle in chunks to check convergence between them)
    void factorize(int k, int kend) {
        // EK_LANCZOS_UNFUSED: run the sharded step sequence on one GPU (tests)
        static const bool unfused = std::getenv("EK_LANCZOS_UNFUSED") != nullptr;
        if (reorth == 1) {
            if (!c->mr && !unfused) return graphs && !time_spmv ? factorize_graph(k, kend) : factorize_fused(k, kend);
            if (pro) return factorize_mr_pro(k, kend);
            return factorize_mr(k, kend);
        }
        double* fn2 = c->fn2.as<double>();
        for (int i = k; i < kend; ++i) {  // reorth 2: CGS2 from the matvec
            const double* x = gather_f();
            const bool timed = spmv_timed_step(i);
            ek::dev::spmv(s, spmv_mat(c), x, c->w.as<double>(), fn2 + i, c->f.as<double>(), col(i), nullptr, nullptr,
                          timed ? ev[size_t(2 * (i - seg0))] : nullptr, timed ? ev[size_t(2 * (i - seg0) + 1)] : nullptr);
            ++matvecs;
            const int nc = i + 1, tot = nc + has_u0;
            ek::dev::gemvt(s, ldv, nrb, V(), nc, has_u0, u0val, nreal, c->w.as<double>(), c->part.as<double>());
            ek::dev::reduce_cols(s, c->part.as<double>(), nrb, tot, c->h1.as<double>());
            allreduce(c, c->h1.as<double>(), size_t(tot));
            ek::dev::update(s, ldv, V(), nc, has_u0, u0val, nreal, c->h1.as<double>(), c->w.as<double>(),
                            c->f.as<double>(), nullptr);
            ek::dev::gemvt(s, ldv, nrb, V(), nc, has_u0, u0val, nreal, c->f.as<double>(), c->part.as<double>());
            ek::dev::reduce_cols(s, c->part.as<double>(), nrb, tot, c->h2.as<double>());
            allreduce(c, c->h2.as<double>(), size_t(tot));
            ek::dev::update(s, ldv, V(), nc, has_u0, u0val, nreal, c->h2.as<double>(), c->f.as<double>(),
                            c->f.as<double>(), c->npart.as<double>());
            ek::dev::finalize_step(s, c->npart.as<double>(), nub, fn2 + i + 1, c->h1.as<double>(),
                                   c->h2.as<double>(), i, c->alpha.as<double>(), c->offd.as<double>());
            allreduce(c, fn2 + i + 1, 1);
        }
        HIPCHK(hipGetLastError());
    }

    // The sharded step (reorth 1), ONE all-gather and ONE all-reduce:
    //  1. the rank's ||f||^2 partial goes into its all-gather slot (f[ldv]);
    //  2. all-gather f -> x (every rank's rows + every rank's ||f||^2);
    //  3. SpMV on the owned rows; its prologue sums the ranks' ||f||^2 in rank
    //     order (the same bits on every rank): w = L f/||f||, v_i = f/||f||;
    //  4. gemvt3: V^T w, V^T v_i, V^T v_{i-1} in one sweep of V;
    //  5. ONE all-reduce of the three column-sum vectors;
    //  6. update_mr: alpha = (V^T w)_i, f' = w - alpha v_i - beta v_{i-1},
    //     h = V^T w - alpha V^T v_i - beta V^T v_{i-1} (= V^T f'),
    //     f = f' - V h, and H's alpha[i], offd[i].
    // The single-GPU step reduces alpha before forming f' and projects f'
    // itself (two dependent reductions); here V^T f' comes from the linearity
    // of the projection, computed from the same sweep, so its error is
    // eps ||w|| instead of eps ||f'|| (the orthogonality of f to V is then a
    // few ulps x ||w||/||f||; it does not compound, because f' is still formed
    // by direct subtraction).  Not bit-identical to the single-GPU step; within
    // the Fiedler tolerances on every golden (tests).
    // overlap (sharded): the owned-slot SpMV runs on the context stream while
    // the all-gather runs on gstream; the halo SpMV then starts from its sums
    bool overlap = false;
    // The exchange of one sharded step: this rank's ||f||^2 partial (from the
    // update's npart) into its slot, f to every rank, and the SpMV's
    // prologue operands in fin (the ranks' partials, in rank order; with the
    // overlap, the owned slot's rows summed while the all-gather runs).
    // Returns the x the SpMV reads.
    const double* exchange_f(int i, ek::dev::StepFin& fin) {
        double* f = c->f.as<double>();
        ek::dev::finalize_step(s, c->npart.as<double>(), nub, f + ldv, nullptr, nullptr, -1, nullptr, nullptr);
        const double* x = f;
        if (c->halo) {  // only the rows each rank reads, into the compact x (its partials inside)
            if (overlap) {
                HIPCHK(hipEventRecord(c->ag_ev[0], s));
                HIPCHK(hipStreamWaitEvent(c->gstream, c->ag_ev[0], 0));
                ek::dev::spmv(s, own_mat(c), f, c->yown.as<double>(), nullptr, nullptr, nullptr, nullptr);
                halo_exchange(c, f, c->gstream);
                HIPCHK(hipEventRecord(c->ag_ev[1], c->gstream));
                HIPCHK(hipStreamWaitEvent(s, c->ag_ev[1], 0));
                fin.own_lo = int(c->hx_base[size_t(c->rank)]);
                fin.own_hi = int(c->hx_base[size_t(c->rank)] + c->nrows);
                fin.ybase = c->yown.as<double>();
            } else {
                halo_exchange(c, f, s);
            }
            x = c->hx_X.as<double>();
            fin.npart = x;  // the ranks' partials at their block ends
            fin.nidx = c->hx_pidx.as<int>();
            fin.nb = c->nranks;
            fin.nstride = 1;
            fin.fn2_out = c->fn2.as<double>() + i;
            return x;
        }
        if (c->mr && overlap) {
            // f (with this rank's ||f||^2 partial at f[ldv]) is final: the
            // all-gather goes out on gstream, and the owned slot's rows are
            // summed meanwhile (unscaled: ||f|| comes with the all-gather)
            HIPCHK(hipEventRecord(c->ag_ev[0], s));
            HIPCHK(hipStreamWaitEvent(c->gstream, c->ag_ev[0], 0));
            ek::dev::spmv(s, own_mat(c), f, c->yown.as<double>(), nullptr, nullptr, nullptr, nullptr);
            allgather(c, f, size_t(c->slot), c->xfull.as<double>(), c->gstream);
            HIPCHK(hipEventRecord(c->ag_ev[1], c->gstream));
            HIPCHK(hipStreamWaitEvent(s, c->ag_ev[1], 0));
            x = c->xfull.as<double>();
            fin.own_lo = int(c->rank * c->slot);
            fin.own_hi = int(c->rank * c->slot + c->nrows);
            fin.ybase = c->yown.as<double>();
        } else if (c->mr) {
            allgather(c, f, size_t(c->slot), c->xfull.as<double>());
            x = c->xfull.as<double>();
        }
        fin.npart = x + ldv;
        fin.nb = c->nranks;
        fin.nstride = int(c->slot);
        fin.fn2_out = c->fn2.as<double>() + i;
        return x;
    }

    void factorize_mr(int k, int kend) {
        double* fn2 = c->fn2.as<double>();
        double* f = c->f.as<double>();
        for (int i = k; i < kend; ++i) {
            ek::dev::StepFin fin;
            const double* x = exchange_f(i, fin);
            const bool timed = spmv_timed_step(i);
            ek::dev::spmv(s, spmv_mat(c), x, c->w.as<double>(), nullptr, f, col(i), nullptr, &fin,
                          timed ? ev[size_t(2 * (i - seg0))] : nullptr, timed ? ev[size_t(2 * (i - seg0) + 1)] : nullptr);
            ++matvecs;
            const int nc = i + 1, tot = nc + has_u0;
            ek::dev::gemvt3(s, ldv, nrb, V(), nc, has_u0, u0val, nreal, c->w.as<double>(), col(i),
                            i > 0 ? col(i - 1) : col(i), c->part.as<double>());
            // (+ ||w||^2: the cancellation test of update_mr)
            ek::dev::reduce_cols(s, c->part.as<double>(), nrb, 3 * tot + 1, c->h2.as<double>());
            allreduce(c, c->h2.as<double>(), size_t(3 * tot + 1));
            ek::dev::update_mr(s, ldv, V(), nc, has_u0, u0val, nreal, c->h2.as<double>(), c->w.as<double>(), col(i),
                               i > 0 ? col(i - 1) : nullptr, fn2 + i, c->bov.as<double>() + i, f,
                               c->npart.as<double>(), c->alpha.as<double>(), c->offd.as<double>(),
                               c->cflag.as<double>(), mr_cancel);
        }
        if (kend == m) reduce_scalar(fn2 + m);  // the cycle's last residual norm
        HIPCHK(hipGetLastError());
    }

    // The sharded step under partial reorthogonalisation (reorth 3; VERDICT
    // r4 next-3).  The single-context PRO step needs alpha_i and ||w||^2
    // before it decides, and the decision before it projects, so the step has
    // two reductions:
    //  1. exchange_f: the all-gather of f (every rank's ||f||^2 partial with it);
    //  2. SpMV: w = L f/||f||, v_i, and per-block partials of alpha and ||w||^2;
    //  3. this rank's (alpha, ||w||^2) -> ONE all-reduce of 2 doubles;
    //  4. k_pro on the global sums: Simon's omega recurrence runs replicated on
    //     every rank (the same alpha, T and state everywhere: the same decision);
    //  5. the projection of f' = w - alpha v_i - beta v_{i-1} (f' formed per row
    //     and stored to f; on a skipped step only that, and ||f'||^2);
    //  6. ONE all-reduce of the column sums h (+ ||f'||^2): issued on every step,
    //     since the host cannot see the device's decision without waiting for
    //     it; a skipped step's kernels have no basis pass and its h entries
    //     the finalize reads are exact zeros;
    //  7. the update f = f' - V h (a skipped step: nothing; ||f||^2 = ||f'||^2
    //     reaches the next SpMV as one global value).
    // A skipped step is the all-gather, the SpMV, two small all-reduces and no
    // pass over V; a projecting one adds the two basis passes (the sharded
    // reorth-1 step always made them, through k_gemvt3 / k_update_mr).  f' is
    // projected directly (not by linearity as in factorize_mr), so there is no
    // cancellation to repair.  H's alpha[i] / offd[i] are written by step i+1's
    // SpMV prologue (the single-context lag) or the cycle's closing finalize.
    void factorize_mr_pro(int k, int kend) {
        double* fn2 = c->fn2.as<double>();
        double* f = c->f.as<double>();
        double* a3 = c->scal.as<double>() + 2;
        double* fast = c->scal.as<double>() + 4;  // ||f||^2 of a skipped step for the next SpMV (NaN: the partials)
        double* aw = c->scal.as<double>() + 6;    // (alpha, ||w||^2): this rank's, then all-reduced
        const double* bov = c->bov.as<double>();
        double* h2 = c->h2.as<double>();
        for (int i = k; i < kend; ++i) {
            ek::dev::StepFin fin;
            const double* x = exchange_f(i, fin);
            fin.wpart = c->wpart.as<double>();
            if (i > seg0) {  // step i-1's finalize in this SpMV's prologue; ||f||^2 from its update when not NaN
                fin.fast = fast;
                fin.h2 = h2;
                fin.step = i - 1;
                fin.alpha = c->alpha.as<double>();
                fin.offd = c->offd.as<double>();
                fin.a3 = a3;
                fin.fn2_i = fn2 + i - 1;
                fin.bov_i = bov + i - 1;
            }
            const bool timed = spmv_timed_step(i);
            ek::dev::spmv(s, spmv_mat(c), x, c->w.as<double>(), nullptr, f, col(i), c->apart.as<double>(), &fin,
                          timed ? ev[size_t(2 * (i - seg0))] : nullptr, timed ? ev[size_t(2 * (i - seg0) + 1)] : nullptr);
            ++matvecs;
            ek::dev::sum_pair(s, c->apart.as<double>(), c->wpart.as<double>(), c->nrb_spmv, aw);
            allreduce(c, aw, 2);
            ek::dev::pro_step(s, aw, aw + 1, 1, a3, fn2 + i, bov + i, c->alpha.as<double>(), c->offd.as<double>(),
                              c->omega.as<double>(), c->prost.as<ek::dev::ProState>(), c->pflags.as<int>(), i, seg0, m,
                              pro_thresh, pro_eps1);
            const int* flag = c->pflags.as<int>() + i;
            const int nc = i + 1, tot = nc + has_u0;
            ek::dev::gemvt_tt(s, ldv, nrb, V(), nc, has_u0, u0val, nreal, c->w.as<double>(), a3, col(i),
                              i > 0 ? col(i - 1) : nullptr, fn2 + i, bov + i, f, c->part.as<double>(), nullptr, nullptr,
                              0, nullptr, nullptr, nt, flag, nullptr, nullptr);
            ek::dev::reduce_cols(s, c->part.as<double>(), nrb, tot + 1, h2);  // (+ ||f'||^2)
            allreduce(c, h2, size_t(tot + 1));
            ek::dev::update(s, ldv, V(), nc, has_u0, u0val, nreal, h2, f, f, c->npart.as<double>(), nullptr, nullptr,
                            fast, nt, flag);
        }
        if (kend == m) {  // the cycle's last step (always projected): its finalize and residual norm
            ek::dev::finalize_step(s, c->npart.as<double>(), nub, fn2 + m, nullptr, h2, m - 1, c->alpha.as<double>(),
                                   c->offd.as<double>(), a3, fn2 + m - 1, bov + m - 1);
            allreduce(c, fn2 + m, 1);
        }
        HIPCHK(hipGetLastError());
    }

    // Single GPU, reorth 1: four launches per step.  The SpMV also runs the
    // previous step's finalize (||f||^2, alpha, beta) and the update reduces
    // the projection partials itself (same column-sum order as k_reduce_cols,
    // so the fused and unfused paths give identical bits).  Folding the
    // three-term recurrence into the projection was measured slower: every
    // column tile re-reads w, v_i and v_{i-1}.  Step i > seg0 finalizes step
    // i - 1 in its SpMV, also across chunks; the last step of the cycle is
    // finalized by its own launch.
    // Who sums the projection partials (nrb row blocks per column): every
    // update workgroup itself (k_update<true>: no launch, but each of the
    // ldv/512 workgroups reads all tot x nrb partials, quadratic in n) or one
    // k_reduce_cols launch ahead of k_update<false> (same col_sum2 order, the
    // same bits).  EK_UPD_RED=0/1 forces either (A/B).
    // 0: a k_reduce_cols launch; 1: every update workgroup; 2: the
    // projection's last workgroup per column group (k_gemvt hand-off, the
    // default up to 256 row blocks).  EK_UPD_RED=0/1/2 forces one (A/B; all
    // three give the same bits).
    static int upd_reduces(int nrb) {
        const char* e = std::getenv("EK_UPD_RED");
        if (e && e[0]) return e[0] - '0';
        return nrb <= EK_UPD_RED_MAX_NRB ? 2 : 0;
    }
    void factorize_fused(int k, int kend) {
        // EK_LANCZOS_TT=0: the separate three-term launch (A/B; the same bits)
        static const bool tt_fused = [] {
            const char* e = std::getenv("EK_LANCZOS_TT");
            return !(e && e[0] == '0');
        }();
        double* fn2 = c->fn2.as<double>();
        double* a3 = c->scal.as<double>() + 2;
        const double* bov = c->bov.as<double>();
        // (partial reorthogonalisation: a skipped step has no partials for
        // every update workgroup to reduce, so the update_r form is not used)
        const int upd_red = pro && upd_reduces(nrb) == 1 ? 0 : upd_reduces(nrb);
        // ||f||^2 for the next SpMV from the update (or, on a skipped step, ||f'||^2)
        double* fast = (b32 || pro) ? c->scal.as<double>() + 4 : nullptr;
        const bool tt = tt_fused || pro;
        unsigned* gctr = upd_red == 2 ? c->gctr.as<unsigned>() : nullptr;
        double* hoff = upd_red == 2 ? c->h2.as<double>() : nullptr;
        const bool inl = pro && proi && upd_red == 2;
        static const bool pro_apart = std::getenv("EK_PRO_APART") != nullptr;  // (lab: k_pro + alpha re-reduced in the projection)
        ek::dev::ProLaunch pl;
        if (inl) {
            pl.wpart = c->wpart.as<double>();
            pl.alpha = c->alpha.as<double>();
            pl.offd = c->offd.as<double>();
            pl.omega = c->omega.as<double>();
            pl.st = c->prost.as<ek::dev::ProState>();
            pl.flags = c->pflags.as<int>();
            pl.pub = pro_pub();
            pl.a3 = a3;
            pl.seg0 = seg0;
            pl.m = m;
            pl.thresh = pro_thresh;
            pl.eps1 = pro_eps1;
            pl.cgw = pro_cgw;
            // tickets (dispatch-order independence): a launch whose grid is
            // not all resident at once takes them (pl.cap); EK_PRO_TICKETS=1
            // on every launch, =0 on none (logical index = blockIdx: A/B)
            static const int tickets = [] {
                const char* e = std::getenv("EK_PRO_TICKETS");
                return e && e[0] ? (e[0] == '0' ? 0 : 2) : 1;
            }();
            if (tickets) pl.tix = pro_pub() + size_t(ek::dev::PRO_PUB_WORDS) * ek::dev::PRO_PUB_STRIDE;
            if (tickets == 1) {
                pl.cap = ek::dev::gemvt_pro_capacity(nt, c->nrb_spmv > 12 * 256, pro_merge, pro_merge && b32,
                                                     c->num_cu);
                // the most workgroups per row block (<= pro_cgw) with which the
                // cycle's widest launch is still resident at once: its launches
                // then need no tickets (the headline: 8 -> 2, +0.2 ms a solve,
                // against +1.0 ms for tickets on every launch;
                // profiles/r06/dispatch_order_ab.txt)
                const int ncg_max = (m + has_u0 + ek::dev::GT_COLS - 1) / ek::dev::GT_COLS;
                auto grid = [&](int cg) { return ek::dev::gemvt_pro_grid(nrb, std::min(ncg_max, cg), ldv, pro_merge); };
                int cg = pl.cgw;  // (0: one workgroup per tile, left as it is; EK_PRO_CGW: as set)
                while (!pro_cgw_env && cg > 1 && grid(cg) > pl.cap) --cg;
                if (!pro_cgw_env && cg > 0 && grid(cg) <= pl.cap) pl.cgw = cg;
            }
            pl.rev = std::getenv("EK_DISPATCH_REVERSE") ? 1 : 0;
            if (pro_merge) {
                pl.merged = 1;
                pl.npart = c->npart.as<double>();
                pl.V32 = V32();
                pl.fb = b32 ? c->fbk.as<unsigned>() : nullptr;
            }
        }
        const bool mrg = inl && pro_merge;
        for (int i = k; i < kend; ++i) {
            ek::dev::StepFin fin;
            if (i > seg0) {
                fin.npart = c->npart.as<double>();
                fin.nb = nub;
                fin.fn2_out = fn2 + i;
                fin.h2 = c->h2.as<double>();
                fin.step = i - 1;
                fin.alpha = c->alpha.as<double>();
                fin.offd = c->offd.as<double>();
                fin.a3 = a3;
                fin.fn2_i = fn2 + i - 1;
                fin.bov_i = bov + i - 1;
                fin.fast = fast;  // the update's ||f||^2 (or NaN)
            }
            if (pro) fin.wpart = c->wpart.as<double>();  // ||w||^2 partials for k_pro (also at i == seg0)
            if (mrg) fin.pub_rearm = pro_pub();  // (the merged update's words and done counter)
            if (chk_dst && i == kend - 1 && i > seg0) {  // the check's copy, in this SpMV's block 0
                fin.chk_dst = chk_dst;
                fin.chk_word = chk_word;
                fin.chk_seq_src = chk_seq_src;
                fin.chk_b = chk_b;
                fin.chk_m = m;
                fin.chk_fn2 = fn2;
                chk_folded = true;
            }
            const bool timed = spmv_timed_step(i);
            // the SpMV's last block also reduces alpha into a3 (k_three_term's bits)
            ek::dev::spmv(s, spmv_mat(c), c->f.as<double>(), c->w.as<double>(), fn2 + i, c->f.as<double>(), col(i),
                          c->apart.as<double>(), (i > seg0 || pro) ? &fin : nullptr,
                          timed ? ev[size_t(2 * (i - seg0))] : nullptr, timed ? ev[size_t(2 * (i - seg0) + 1)] : nullptr,
                          !pro && tt_fused && alpha_last ? a3 : nullptr, c->actr.as<unsigned>());
            ++matvecs;
            const int nc = i + 1;
            // partial reorthogonalisation: alpha, and whether this step projects
            const int* flag = pro ? c->pflags.as<int>() + i : nullptr;
            if (pro && !inl)
                ek::dev::pro_step(s, c->apart.as<double>(), c->wpart.as<double>(), c->nrb_spmv, a3, fn2 + i, bov + i,
                                  c->alpha.as<double>(), c->offd.as<double>(), c->omega.as<double>(),
                                  c->prost.as<ek::dev::ProState>(), c->pflags.as<int>(), i, seg0, m, pro_thresh, pro_eps1);
            if (tt) {  // the projection of f' = w - alpha v_i - beta v_{i-1}, formed per row (and stored to f)
                ek::dev::gemvt_tt(s, ldv, nrb, V(), nc, has_u0, u0val, nreal, c->w.as<double>(), a3, col(i),
                                  i > 0 ? col(i - 1) : nullptr, fn2 + i, bov + i, c->f.as<double>(), c->part.as<double>(),
                                  col32(i),
                                  inl || pro_apart || !(alpha_last || pro) ? c->apart.as<double>() : nullptr, c->nrb_spmv,
                                  gctr, hoff, nt, flag, pro ? fast : nullptr, inl ? &pl : nullptr);
            } else {
                ek::dev::three_term(s, ldv, c->apart.as<double>(), c->nrb_spmv, a3, c->w.as<double>(), col(i),
                                    i > 0 ? col(i - 1) : nullptr, fn2 + i, bov + i, c->f.as<double>(), col32(i));
                ek::dev::gemvt(s, ldv, nrb, V(), nc, has_u0, u0val, nreal, c->f.as<double>(), c->part.as<double>(),
                               b32 ? 1 : 0, gctr, hoff, nt);
            }
            // (b32: ||f'||^2 rides along as one more column of the partials)
            unsigned* fb = b32 ? c->fbk.as<unsigned>() : nullptr;
            // (b32: the update also leaves ||f||^2 = ||f'||^2 - ||h||^2 for the next SpMV)
            if (mrg) {
                // (the update ran inside the projection launch)
            } else if (upd_red == 2) {  // h (and ||f'||^2) reduced by the projection
                ek::dev::update(s, ldv, V(), nc, has_u0, u0val, nreal, c->h2.as<double>(), c->f.as<double>(),
                                c->f.as<double>(), c->npart.as<double>(), V32(), fb, fast, nt, flag,
                                inl ? pro_pub() : nullptr);
            } else if (upd_red == 1) {
                ek::dev::update_r(s, ldv, V(), nc, has_u0, u0val, nreal, c->part.as<double>(), nrb, c->h2.as<double>(),
                                  c->f.as<double>(), c->f.as<double>(), c->npart.as<double>(), V32(), fb, fast, nt);
            } else {
                ek::dev::reduce_cols(s, c->part.as<double>(), nrb, nc + has_u0 + ((b32 || pro) ? 1 : 0),
                                     c->h2.as<double>());
                ek::dev::update(s, ldv, V(), nc, has_u0, u0val, nreal, c->h2.as<double>(), c->f.as<double>(),
                                c->f.as<double>(), c->npart.as<double>(), V32(), fb, fast, nt, flag);
            }
            if (b32) ++u32_steps;
        }
        if (kend == m)
            ek::dev::finalize_step(s, c->npart.as<double>(), nub, fn2 + m, nullptr, c->h2.as<double>(), m - 1,
                                   c->alpha.as<double>(), c->offd.as<double>(), a3, fn2 + m - 1, bov + m - 1);
        HIPCHK(hipGetLastError());
    }

    // The sharded step projects f' by linearity (V^T f' = V^T w - alpha V^T v_i
    // - beta V^T v_{i-1}), exact to eps ||w||.  When f' cancelled (update_mr's
    // cflag: ||f'||^2 < mr_cancel ||w||^2, near an invariant subspace) that is
    // not small against ||f'||, and v_{j1} = f_{j1}/||f_{j1}|| would carry a
    // loss of orthogonality of eps ||w|| / beta_{j1}.  The driver sees the flag
    // at its next check and re-projects: f = v_{j1} (unit; or f_m itself at
    // the cycle's end, j1 == m) against V[:, :j1] and u0 — one more CGS pass,
    // the CGS2 path's second pass — with Spectra's H += V^T f correction
    // (scaled by beta_{j1}: f_{j1} = beta_{j1} v_{j1}) and T(j1, j1-1) =
    // beta_{j1} ||f|| through the beta override; the cycle continues at j1.
    // beta_j1: sqrt(fn2[j1]) as the run left it (host copy); returns the
    // corrections (h[j1-1], h[j1-2]) to add to the host's T.
    std::pair<double, double> repair(int j1, double beta_j1) {
        double* f = c->f.as<double>();
        double* fn2 = c->fn2.as<double>();
        const double sc = j1 < m ? beta_j1 : 1.0;
        if (j1 < m) HIPCHK(hipMemcpyAsync(f, col(j1), size_t(ldv) * 8, hipMemcpyDeviceToDevice, s));
        ek::dev::gemvt(s, ldv, nrb, V(), j1, has_u0, u0val, nreal, f, c->part.as<double>());
        ek::dev::reduce_cols(s, c->part.as<double>(), nrb, j1 + has_u0, c->h1.as<double>());
        allreduce(c, c->h1.as<double>(), size_t(j1 + has_u0));
        ek::dev::update(s, ldv, V(), j1, has_u0, u0val, nreal, c->h1.as<double>(), f, f, c->npart.as<double>());
        reduce_scalar(fn2 + j1);
        double hh[2] = {0.0, 0.0}, n2 = 0.0;
        HIPCHK(hipMemcpyAsync(hh, c->h1.as<double>() + std::max(j1 - 2, 0), size_t(std::min(j1, 2)) * 8,
                              hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(&n2, fn2 + j1, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        const double h1 = sc * (j1 >= 2 ? hh[1] : hh[0]), h2 = j1 >= 2 ? sc * hh[0] : 0.0;  // h[j1-1], h[j1-2]
        // device T entries (the host's are corrected by the caller)
        double a = 0.0, o = 0.0;
        HIPCHK(hipMemcpyAsync(&a, c->alpha.as<double>() + j1 - 1, 8, hipMemcpyDeviceToHost, s));
        if (j1 >= 2) HIPCHK(hipMemcpyAsync(&o, c->offd.as<double>() + j1 - 1, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        a += h1;
        o += h2;
        HIPCHK(hipMemcpyAsync(c->alpha.as<double>() + j1 - 1, &a, 8, hipMemcpyHostToDevice, s));
        if (j1 >= 2) HIPCHK(hipMemcpyAsync(c->offd.as<double>() + j1 - 1, &o, 8, hipMemcpyHostToDevice, s));
        if (j1 < m) {
            const double bo = beta_j1 * std::sqrt(std::max(0.0, n2));
            HIPCHK(hipMemcpyAsync(c->bov.as<double>() + j1, &bo, 8, hipMemcpyHostToDevice, s));
        }
        HIPCHK(hipStreamSynchronize(s));  // (host operands)
        ++repairs;
        return {h1, h2};
    }
    int repairs = 0;
    double mr_cancel = 0x1p-20;

    // The single-context step chunk as a HIP graph.  Eager, the host spends
    // ~10 us per kernel launch, so a partially reorthogonalised step (four
    // launches, ~26 us of kernels when it skips the basis passes) waited for
    // its launches (tools/trace_gaps.py: the GPU idle between kernels).  A
    // chunk's launches depend only on (k, kend, seg0) and the context's
    // buffers, so its graph is captured the second time the chunk is run and
    // replayed from then on: the restart cycles repeat the same chunks, and a
    // service's solves all of them.  (The first time it runs eagerly: a
    // one-shot process does not pay for captures it never replays.)
    bool graphs = false;
    void factorize_graph(int k, int kend) {
        const auto key = std::make_tuple(k, kend, seg0, static_cast<const void*>(V()), static_cast<const void*>(V32()));
        auto it = c->lz_graphs.find(key);
        if (it == c->lz_graphs.end()) {
            if (++c->lz_seen[key] < 2) return factorize_fused(k, kend);
            hipGraph_t g = nullptr;
            HIPCHK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
            try {
                factorize_fused(k, kend);  // (recorded, not run; its host counters advance here)
            } catch (...) {
                (void)hipStreamEndCapture(s, &g);
                if (g) (void)hipGraphDestroy(g);
                throw;
            }
            HIPCHK(hipStreamEndCapture(s, &g));
            hipGraphExec_t ex = nullptr;
            const hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            HIPCHK(e);
            it = c->lz_graphs.emplace(key, ex).first;
        } else {
            matvecs += kend - k;
            if (b32) u32_steps += kend - k;
            // (the replayed launches carry the check's fold exactly when the
            // captured ones did: factorize_fused's condition, constant per chunk)
            if (chk_dst && kend - 1 > seg0) chk_folded = true;
        }
        HIPCHK(hipGraphLaunch(it->second, s));
    }

    // Invariant subspace found at step j1-1 (||f|| collapsed, as on a graph
    // with several components): continue the sequence from a fresh random
    // vector orthogonal to V[:, :j1] and u0, with H(j1, j1-1) = 0 — Spectra's
    // Lanczos::factorize_from restart-on-breakdown.  The vector is generated
    // over GLOBAL indices so every rank builds the same one.
    // The sequence is the Lehmer generator st <- 48271 st mod (2^31 - 1) from
    // st0; the device kernel jumps ahead to each global row (a host loop over
    // the rows, plus the copy, took ~0.6 ms of GPU idle per injection).
    void inject(int j1, int tag) {
        const uint64_t st0 = 2654435761ull * uint64_t(tag) % 2147483647ull + 1;
        double* f = c->f.as<double>();
        ek::dev::inject_random(s, f, ldv, c->row0, c->nrows, st0);
        for (int pass = 0; pass < 2; ++pass) {
            ek::dev::gemvt(s, ldv, nrb, V(), j1, has_u0, u0val, nreal, f, c->part.as<double>());
            ek::dev::reduce_cols(s, c->part.as<double>(), nrb, j1 + has_u0, c->h1.as<double>());
            allreduce(c, c->h1.as<double>(), size_t(j1 + has_u0));
            ek::dev::update(s, ldv, V(), j1, has_u0, u0val, nreal, c->h1.as<double>(), f, f,
                            pass == 1 ? c->npart.as<double>() : nullptr);
        }
        reduce_scalar(c->fn2.as<double>() + j1);
        HIPCHK(hipMemsetAsync(c->bov.as<double>() + j1, 0, 8, s));  // beta_j1 = +0.0
    }

    // pinned slot i of the mid-cycle checks: alpha[m], offd[m], fn2[m]
    // (four regions: alpha, offd, fn2 at m-based offsets; the sharded step's
    // cancellation flags at CHK_FLAGS)
    static constexpr size_t CHK_FLAGS = 3 * size_t(ek::dev::MAX_NCV + 2);
    double* chk_slot(int i) { return c->chk_pin + size_t(i) * 4 * size_t(ek::dev::MAX_NCV + 2); }

    // The SpMV's kernel timestamps are taken on every 4th step of a cycle: a
    // launch with timing events costs the host ~7 us more, which the timed
    // solve would otherwise carry on every step.  The sample starts at the
    // cycle's second step: the first SpMV after a restart (1 in 100 of the
    // launches) follows the V <- VQ stream and would be 1 in 25 of the sample.
    static constexpr int SPMV_SAMPLE = 4;
    bool spmv_timed_step(int i) const {
        return time_spmv && (i - seg0) % SPMV_SAMPLE == 1 && size_t(2 * (i - seg0) + 1) < ev.size();
    }

    // the timed SpMVs of steps [seg0, kend) (the steps launched in this run)
    void collect_spmv_times(int kend) {
        if (!time_spmv) return;
        HIPCHK(hipStreamSynchronize(s));
        for (int i = seg0; i < kend && size_t(2 * (i - seg0) + 1) < ev.size(); ++i) {
            if (!spmv_timed_step(i)) continue;
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, ev[size_t(2 * (i - seg0))], ev[size_t(2 * (i - seg0) + 1)]));
            spmv_ms += ms;
            ++spmv_timed;
        }
    }
};

}  // namespace

extern "C" int ek_lanczos_fiedler(ek_ctx* c, const ek_lanczos_opts* opts, double* lambda_out, double* v_out,
                                  ek_lanczos_stats* stats) {
    EK_TRY
    check_ctx(c);
    if (!c->n) ek::fail(EK_ESTATE, "ek_lanczos_fiedler before ek_spmv_setup");
    ek_lanczos_opts o;
    ek_lanczos_default_opts(&o);
    if (opts) o = *opts;
    const auto t0 = std::chrono::steady_clock::now();
    c->comm_ms = 0.0;
    c->n_ag = c->n_ar = 0;
    c->comm_time = opts && opts->time_spmv && c->mr;
    c->cm_rec.clear();
    c->cm_used = 0;
    if (c->comm_time) c->x_ms = c->ar_ms = 0.0, c->x_timed = c->ar_timed = 0;
    c->fied_n = 0;  // any earlier vector is void once a solve starts; set again only on success
    const int64_t n = c->n;
    const bool deflate = o.deflate != 0;
    const int nev = deflate ? 1 : 2;
    // ncv: the reference's min(100, n/2) (cEIG.cpp:195) for the full and CGS2
    // passes.  Under partial reorthogonalisation (reorth 3, the default) a
    // step costs ~ncv only when it projects, and a restart's host QL and QR
    // shifts cost ~ncv^2 with the GPU idle, so below a million rows, where a
    // restart weighs most against the steps, a smaller basis pays: min(80,
    // n/2) (round 5, tools/ncv_ab.py, profiles/r05/ncv_ab_r05*.txt: headline
    // 17.6 -> 16.7 ms, ibm10 38.7 -> 37.7, the 2x LCC 36.8 -> 35.2, the 5x
    // LCC 54.0 -> 51.2, ibm01 7.6 -> 6.9; 64-72 lose on ibm10).  Above it
    // the steps dominate and the basis's convergence decides: the 10x
    // synthetic (disconnected: its null space) took 838 matvecs at 80 against
    // 394 at 100 (tools/ncv10_lab.py, profiles/r05/ncv10.txt)
    // reorth 3: partial reorthogonalisation, on the single-context step and
    // on the sharded one (factorize_mr_pro; the CGS2 step always projects).
    // EK_REORTH=1|3 overrides (A/B).
    int reorth_mode = o.reorth;
    if (const char* e = std::getenv("EK_REORTH"); e && e[0]) reorth_mode = std::atoi(e);
    const int ncv_dflt = reorth_mode == 3 && n < 1000000 ? 80 : 100;
    int m = o.ncv > 0 ? o.ncv : int(std::min<int64_t>(ncv_dflt, n / 2));
    m = int(std::min<int64_t>(m, n - (deflate ? 1 : 0)));
    if (m > ek::dev::MAX_NCV) ek::fail(EK_EINVAL, "ncv %d exceeds %d", m, ek::dev::MAX_NCV);
    if (m <= nev) ek::fail(EK_EINVAL, "graph too small for ncv=%d (n=%lld)", m, (long long)n);
    const double tol = o.tol > 0 ? o.tol : 1e-10;
    const int maxit = o.maxit > 0 ? o.maxit : 1000;
    const double eps23 = std::pow(std::numeric_limits<double>::epsilon(), 2.0 / 3.0);
    const bool trace = std::getenv("EK_LANCZOS_TRACE") != nullptr;
    const bool ortho_check = std::getenv("EK_LANCZOS_ORTHO") != nullptr;
    double ortho_max = 0.0;

    Lanczos L{};
    L.c = c;
    L.s = c->stream;
    L.m = m;
    L.ldv = int(round_up(std::max<int64_t>(c->nloc, 1), ek::dev::GT_ROWS));
    L.nrb = L.ldv / ek::dev::GT_ROWS;
    L.nub = L.ldv / ek::dev::UPD_ROWS;
    L.has_u0 = deflate ? 1 : 0;
    L.nreal = int(c->nrows);
    L.u0val = 1.0 / std::sqrt(double(n));
    L.time_spmv = o.time_spmv != 0;
    L.reorth = o.reorth == 2 ? 2 : 1;
    hipStream_t s = c->stream;
    L.pro = reorth_mode == 3 && L.reorth == 1 && std::getenv("EK_LANCZOS_UNFUSED") == nullptr;
    // threshold 1e-10, not Simon's sqrt(eps): across implicit restarts the
    // kept Ritz block carries the basis's loss of orthogonality into the next
    // cycle, and the dropped projection coefficients (O(threshold) beta) stay
    // in the Lanczos relation.  tools/pro_model.py on ibm10 (15 restarts):
    // sqrt(eps) -> max|V^T V - I| 1e-7, residual 2e-9, lambda off by 5e-10;
    // 1e-9 -> 3e-8, 1.4e-9; 1e-10 -> 1.4e-10, 1.9e-10 (full: 5e-14, 1e-12),
    // 44 % of the steps projected; the headline LCC 32 %, residual unchanged
    L.pro_thresh = o.reorth_thresh > 0 ? o.reorth_thresh : 1e-10;
    L.pro_eps1 = std::numeric_limits<double>::epsilon() * std::sqrt(double(n));
    // (the in-launch decision and merged update: single context only; the
    // sharded step all-reduces alpha and ||w||^2 before its k_pro launch.
    // Their spin-waits assume workgroups are dispatched in index order, which
    // HIP does not promise: every wait is bounded, the first to give up aborts
    // the launch's other waiters (kernels_lanczos.hip pro_poll), and the solve
    // fails with EK_EHIP.  EK_PRO_INLAUNCH=0 runs the step with no in-launch
    // wait at all.)
    if (const char* e = std::getenv("EK_PRO_INLAUNCH"); L.pro && !c->mr) L.proi = !(e && e[0] == '0');
    if (const char* e = std::getenv("EK_PRO_MERGE"); L.proi) L.pro_merge = !(e && e[0] == '0');
    // column groups walked per projection workgroup: about 850 projection
    // workgroups, at least 3 per row block (the 1.15x LCC, 207 row blocks:
    // 4; ibm01 / ibm10: one workgroup per tile as before).  A skipped step
    // then dispatches ~850 + 422 workgroups instead of up to ~3,100 (headline
    // Lanczos 20.4 -> 19.4 ms; ibm10 and ibm01 lost 3-10 % at 3-4 per row
    // block: too few workgroups for the projecting steps;
    // profiles/r04/cgw/).  Round 5: with column group 0 dispatched first the
    // other groups' workgroups cost a skipped step little (they read the
    // decision and return), so more of them, which a projecting step uses,
    // pay: at least 8 per row block (headline Lanczos 17.93-18.05 ms at 4,
    // 17.67-17.72 at 6, 17.53-17.61 at 8, 17.66-17.70 at one per tile;
    // profiles/r05/pro/cgw_ab*.txt).  EK_PRO_CGW overrides (0: one workgroup
    // per tile)
    L.pro_cgw = std::max(8, 850 / std::max(1, L.nrb));
    if (const char* e = std::getenv("EK_PRO_CGW"); e && e[0]) {
        L.pro_cgw = std::atoi(e);
        L.pro_cgw_env = true;
    }

    const size_t ldv = size_t(L.ldv);
    c->V.ensure(ldv * size_t(m + 1) * 8);
    c->Vn.ensure(ldv * size_t(m + 1) * 8);
    // the fp32 shadow: single-context three-term steps (the sharded and CGS2
    // steps project w itself, where h is not small)
    // (EK_BASIS32=0|1 / EK_ALPHA_LAST=0|1 override the options: A/B runs)
    auto env_or = [](const char* k, bool dflt) {
        const char* e = std::getenv(k);
        return e && e[0] ? e[0] != '0' : dflt;
    };
    L.b32 = env_or("EK_BASIS32", o.basis32 != 0) && !c->mr && L.reorth == 1 &&
            std::getenv("EK_LANCZOS_UNFUSED") == nullptr;
    L.alpha_last = env_or("EK_ALPHA_LAST", o.alpha_last != 0);
    // non-temporal basis passes once the fp64 basis exceeds 768 MB (3x the
    // 256 MB MALL): it cannot stay there, and sweeping it through evicts the
    // matrix and x between SpMVs.  10x synthetic (1.6 GB): 404 -> 380 us per
    // matvec; at 300 MB (the 2x synthetics) the basis still profits from the
    // MALL (LCC 59.3 -> 61.2 ms with them).  EK_V_NT=0/1 forces either.
    L.nt = env_or("EK_V_NT", ldv * size_t(m + 1) * 8 > (size_t(768) << 20));
    if (L.b32) {
        c->V32.ensure(ldv * size_t(m + 1) * 4);
        c->Vn32.ensure(ldv * size_t(m + 1) * 4);
        c->fbk.ensure(64);
        HIPCHK(hipMemsetAsync(c->fbk.p, 0, 4, c->stream));
    }
    // f: + 64 (the sharded step's all-gather slot carries the rank's ||f||^2 at [ldv])
    if (c->mr && c->slot != int64_t(ldv) + 64) ek::fail(EK_ESTATE, "shard slot %lld != ldv + 64", (long long)c->slot);
    c->f.ensure((ldv + 64) * 8);
    c->w.ensure(ldv * 8);
    if (c->mr) c->xfull.ensure(size_t(c->slot) * size_t(c->nranks) * 8);
    c->part.ensure(3 * size_t(m + 2) * size_t(L.nrb) * 8);  // x 3: gemvt3 (sharded step)
    c->h1.ensure(size_t(m + 2) * 8);
    c->h2.ensure(3 * size_t(m + 2) * 8);
    c->alpha.ensure(size_t(m + 1) * 8);
    c->offd.ensure(size_t(m + 1) * 8);
    c->fn2.ensure(size_t(m + 2) * 8);
    c->bov.ensure(size_t(m + 2) * 8);
    c->npart.ensure(size_t(L.nub) * 8);
    c->apart.ensure(size_t(std::max(c->nrb_spmv, 1)) * 8);
    c->Qd.ensure(size_t(m) * size_t(m + 1) * 8);
    c->scal.ensure(64);
    // the hand-off counters are zero between launches; re-armed here too, so a
    // launch that died part-way cannot leave them out of step for this solve
    c->actr.ensure((ek::dev::ALPHA_SUB + 1) * 256);
    HIPCHK(hipMemsetAsync(c->actr.p, 0, c->actr.bytes, s));
    c->gctr.ensure(size_t(ek::dev::GT_HANDOFF_UINTS) * 4);
    HIPCHK(hipMemsetAsync(c->gctr.p, 0, c->gctr.bytes, s));
    if (L.pro) {
        c->wpart.ensure(size_t(std::max(c->nrb_spmv, 1)) * 8);
        c->omega.ensure(3 * size_t(ek::dev::OMEGA_LD) * 8);
        c->prost.ensure(sizeof(ek::dev::ProState));
        // + the in-launch decision's words (PRO_PUB lines of 256 B), zero between launches
        // + the tickets of the in-launch jobs (8 lines of 256 B after them)
        c->pflags.ensure(L.pro_pub_off() + size_t(ek::dev::PRO_PUB_WORDS + 8) * 256);
        HIPCHK(hipMemsetAsync(c->prost.p, 0, sizeof(ek::dev::ProState), s));
        HIPCHK(hipMemsetAsync(L.pro_pub(), 0, size_t(ek::dev::PRO_PUB_WORDS + 8) * 256, s));
    }
    // the step chunks' graphs (EK_LANCZOS_GRAPH=0: eager launches, A/B), kept
    // while every buffer and parameter their launches carry is unchanged
    L.graphs = env_or("EK_LANCZOS_GRAPH", true) && !c->mr && L.reorth == 1;
    if (L.graphs) {
        const int tt_env = std::getenv("EK_LANCZOS_TT") ? 1 : 0;
        auto pv = [](const void* p) { return uint64_t(reinterpret_cast<uintptr_t>(p)); };
        auto db = [](double x) {
            uint64_t u;
            std::memcpy(&u, &x, 8);
            return u;
        };
        // (V / Vn and V32 / Vn32 swap at every restart: the pairs, not their order)
        std::vector<uint64_t> sig{std::min(pv(c->V.p), pv(c->Vn.p)), std::max(pv(c->V.p), pv(c->Vn.p)),
                                  std::min(pv(c->V32.p), pv(c->Vn32.p)), std::max(pv(c->V32.p), pv(c->Vn32.p)),
                                  pv(c->f.p), pv(c->w.p),
                                  pv(c->part.p), pv(c->h1.p), pv(c->h2.p), pv(c->alpha.p), pv(c->offd.p), pv(c->fn2.p),
                                  pv(c->bov.p), pv(c->npart.p), pv(c->apart.p), pv(c->scal.p), pv(c->fbk.p),
                                  pv(c->actr.p), pv(c->gctr.p), pv(c->wpart.p), pv(c->omega.p), pv(c->prost.p),
                                  pv(c->pflags.p), pv(c->rb.p), pv(c->pk.p), pv(c->rel.p), pv(c->dict.p), pv(c->col.p),
                                  pv(c->val.p), pv(c->rowptr.p), pv(c->pn_wrow.p), pv(c->pn_start.p), pv(c->pn_word.p),
                                  pv(c->pn_rid.p), uint64_t(m), uint64_t(L.ldv), uint64_t(L.nreal), uint64_t(c->n),
                                  uint64_t(c->nrb_spmv), uint64_t(c->pn_G), uint64_t(c->colbits), uint64_t(L.has_u0),
                                  uint64_t(L.b32), uint64_t(L.pro), uint64_t(L.proi), uint64_t(L.pro_merge), uint64_t(L.nt), uint64_t(L.alpha_last),
                                  uint64_t(tt_env), db(L.pro_thresh),
                                  db(L.pro_eps1), db(L.u0val)};
        if (sig != c->lz_sig) {
            for (auto& g : c->lz_graphs) HIPCHK(hipGraphExecDestroy(g.second));
            c->lz_graphs.clear();
            c->lz_seen.clear();
            c->lz_sig = std::move(sig);
        }
    }
    // padded rows must be exactly 0 (only those: every kernel writes real
    // rows before it reads them, and no kernel writes a padded row nonzero)
    ek::dev::zero_pad_rows(s, c->V.as<double>(), L.ldv, L.nreal, m + 1);
    ek::dev::zero_pad_rows(s, c->Vn.as<double>(), L.ldv, L.nreal, m + 1);
    HIPCHK(hipMemsetAsync(c->w.p, 0, c->w.bytes, s));
    HIPCHK(hipMemsetAsync(c->f.p, 0, c->f.bytes, s));
    if (c->mr) HIPCHK(hipMemsetAsync(c->xfull.p, 0, c->xfull.bytes, s));
    if (!c->cstream) {  // mid-cycle check resources, created once per context
        HIPCHK(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
        // chk_done orders the check's copy (cstream, same device) after a
        // chunk: a device-scope release is all it needs.  With the default
        // system-scope fence every chunk boundary left the compute queue idle
        // for the fence's L2 write-back (6-15 us at each of ~58 boundaries a
        // solve, kernel trace).  EK_CHK_FENCE: 0 system (the HIP default), 1
        // device-scope release (default), 2 no fence
        static const int chk_fence = [] {
            const char* e = std::getenv("EK_CHK_FENCE");
            return e && e[0] ? std::atoi(e) : 1;
        }();
        const unsigned done_flags = hipEventDisableTiming | (chk_fence == 1   ? hipEventReleaseToDevice
                                                             : chk_fence == 2 ? hipEventDisableSystemFence
                                                                              : 0u);
        for (int i = 0; i < 2; ++i) {
            HIPCHK(hipEventCreateWithFlags(&c->chk_done[i], done_flags));
            HIPCHK(hipEventCreateWithFlags(&c->chk_copied[i], hipEventDisableTiming));
        }
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->chk_pin), 2 * 4 * size_t(ek::dev::MAX_NCV + 2) * 8,
                             hipHostMallocDefault));
        // [slot * 64]: the completion words; [128 + slot * 64]: the sequence
        // numbers the folded copy stores (written by the host before the chunk)
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->chk_word), 4 * 256, hipHostMallocCoherent));
        std::memset(c->chk_word, 0, 4 * 256);
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->q_pin),
                             (size_t(ek::dev::MAX_NCV) * size_t(ek::dev::MAX_NCV + 1) + 2 * size_t(ek::dev::MAX_NCV + 2)) * 8,
                             hipHostMallocDefault));
    }
    if (L.time_spmv) {  // created once per context: ~200 creations per solve cost milliseconds
        while (c->spmv_ev.size() < size_t(2 * m)) {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            c->spmv_ev.push_back(e);
        }
        L.ev.assign(c->spmv_ev.begin(), c->spmv_ev.begin() + 2 * m);
    }

    // start vector: Park-Miller LCG over GLOBAL indices (identical on every
    // rank), values in [-0.5, 0.5) like Spectra's SimpleRandom; deflated.
    // Generated on the device (jump-ahead per element, the same doubles as
    // the sequential host loop it replaces, without its ~1 ms and the upload).
    {
        ek::dev::start_vector(s, L.ldv, (long long)c->row0, int(c->nrows), c->f.as<double>());
        double* sc = c->scal.as<double>();
        if (deflate) {
            ek::dev::sum_partial(s, L.ldv, c->f.as<double>(), L.nreal, c->npart.as<double>(), 0);
            L.reduce_scalar(sc);
            ek::dev::scale_sub_mean(s, L.ldv, c->f.as<double>(), L.nreal, sc, 1.0 / double(n));
        }
        ek::dev::sum_partial(s, L.ldv, c->f.as<double>(), L.nreal, c->npart.as<double>(), 1);
        L.reduce_scalar(c->fn2.as<double>());
    }

    std::vector<double> d(size_t(m), 0.0), e(size_t(m), 0.0), theta(static_cast<size_t>(m)), zl(static_cast<size_t>(m));
    std::vector<double> alpha_h(size_t(m + 1)), offd_h(size_t(m + 1)), fn2_h(size_t(m + 2));
    std::vector<ek::QRot> rots;
    std::vector<double> qscratch;
    // the restart's floor on the kept vectors (EK_KEEP_MIN overrides: A/B)
    const int keep_min = std::getenv("EK_KEEP_MIN") ? std::atoi(std::getenv("EK_KEEP_MIN"))
                         : o.keep_min < 0                ? m / 5
                                                         : o.keep_min;
    int k = 0, restarts = 0, nconv = 0, injected = 0;
    double fn2_k = 1.0;  // ||f_k||^2 entering a cycle (after an implicit restart: the restart's residual)
    bool converged = false;
    int mf = m;  // steps the returned Ritz pair is taken from (< m: converged at a mid-cycle check)
    const double beta_eps = std::numeric_limits<double>::epsilon() * std::sqrt(double(n));
    double host_restart_ms = 0.0, device_cycle_ms = 0.0, host_qr_ms = 0.0;  // EK_LANCZOS_TRACE diagnostics
    double host_ql_ms = 0.0, restart_sync_ms = 0.0;
    auto anorm_of = [&] {
        double a = 1.0;
        for (int i = 0; i < m; ++i) a = std::max(a, std::fabs(d[size_t(i)]) + (i > 0 ? std::fabs(e[size_t(i - 1)]) : 0.0));
        return a;
    };
    // the sharded step's re-projection of a cancelled f' (Lanczos::repair);
    // EK_LANCZOS_UNFUSED runs that step (and its flags) on a single context too
    const bool mr_step = (c->mr || std::getenv("EK_LANCZOS_UNFUSED") != nullptr) && L.reorth == 1 && !L.pro;
    // the owned-slot / halo split of the sharded SpMV (EK_MR_OVERLAP=0: one
    // SpMV after the all-gather, the round-3 step; A/B and tests)
    {
        const char* e = std::getenv("EK_MR_OVERLAP");
        L.overlap = c->mr && c->own_ready && !(e && e[0] == '0');
    }
    if (mr_step) {
        c->cflag.ensure(size_t(m + 2) * 8);  // (update_mr writes one flag per step)
        if (const char* e = std::getenv("EK_MR_CANCEL"); e && e[0]) L.mr_cancel = std::atof(e);  // (tests)
    }
    const bool chk_kernel = [] {
        const char* e = std::getenv("EK_CHK_KERNEL");
        return !(e && e[0] == '0');
    }();
    // The mid-cycle check's gather on the compute stream itself, followed by
    // a completion word the host polls (EK_CHK_POLL=0: the event on the
    // compute stream, the gather on the copy stream, an event the host waits
    // on).  The event was a barrier packet that drained the compute queue at
    // every chunk boundary (~12 us each, ~57 a solve); a kernel in the stream
    // is not.  The word is the gather's last store, made after every store of
    // the slot is released to the system (k_chk_gather).
    const bool chk_poll = chk_kernel && [] {
        const char* e = std::getenv("EK_CHK_POLL");
        return !(e && e[0] == '0');
    }();
    // the host's wait for a slot's completion word (bounded: a kernel that
    // never ran must fail the solve, not hang the host)
    auto chk_wait = [&](int sl, unsigned seq) {
        volatile unsigned* w = c->chk_word + size_t(sl) * 64;
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned spin = 0; *w != seq; ++spin) {
            if ((spin & 1023u) == 1023u) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(20))
                    ek::fail(EK_EHIP, "Lanczos: a mid-cycle check's completion word never arrived");
                const hipError_t qe = hipStreamQuery(s);  // (a faulted stream ends the wait)
                if (qe != hipSuccess && qe != hipErrorNotReady) HIPCHK(qe);
                if (qe == hipSuccess && *w != seq)  // (the stream drained: the word can no longer arrive)
                    ek::fail(EK_EHIP, "Lanczos: the stream finished without a mid-cycle check's completion word "
                                      "(slot %d: %u, expected %u)", sl, *w, seq);
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    };
    unsigned chk_seq_of[2] = {0u, 0u};
    bool cycle_reset = false;  // the restart already queued the resets below
    for (;;) {
        if (!cycle_reset) {
            HIPCHK(hipMemsetAsync(c->bov.p, 0xFF, c->bov.bytes, s));  // NaN: no beta override
            if (mr_step) HIPCHK(hipMemsetAsync(c->cflag.p, 0, c->cflag.bytes, s));
        }
        cycle_reset = false;
        const auto tc = std::chrono::steady_clock::now();
        int cycle_breakdowns = 0;  // bounded per cycle: each one moves the factorisation forward
        int from = k;
        // After an implicit restart the residual f_k can collapse (the kept
        // Ritz space is invariant, seen on the 2x synthetic): a zero column k
        // would leave a spurious exact-zero Ritz pair whose vector is zero, so
        // the cycle starts from a fresh vector at k instead of running on it.
        if (k > 0 && !(std::sqrt(std::max(0.0, fn2_k)) > beta_eps * anorm_of())) {
            if (trace) std::fprintf(stderr, "[lanczos] restart residual collapsed at %d (|f|^2=%.3e)\n", k, fn2_k);
            ++cycle_breakdowns;
            L.inject(k, ++injected);
        }
        int jconv = -1;  // > 0: converged on the projected matrix of the first jconv steps (mid-cycle check)
        double beta_r = 0.0;  // ||f_jr|| as the run left it (a re-projection's scale)
        for (;;) {
            L.seg0 = from;
            // After the first cycle the cycle is enqueued in chunks; the host
            // tests the projected matrix of each chunk (its {alpha, offd,
            // fn2} copied on a second stream into a pinned slot) while the GPU
            // runs the next one: a converged Ritz pair stops the cycle there,
            // a collapsed residual is injected without running the rest of
            // the cycle on a zero vector.
            // (about 0.5 ms of GPU work per chunk: the host's check of one
            // chunk and its launches of the next must fit in the chunk the GPU
            // is running.  The step time is modelled from n, not measured, so
            // the stopping step and the result bits do not depend on timing:
            // ~12 us + 0.23 ns per row, 15 us at ibm01, 58 us at ibm18 shape.)
            const int chunk = (restarts > 0 && o.check_every > 0)
                                  ? std::max({2, int(o.check_every), int(std::ceil(500.0 / (12.0 + 2.3e-4 * double(n))))})
                                  : m;
            int a = from, launched = from, j1 = -1, jr = -1;  // breakdown / re-projection at
            int pend = -1, pend_slot = 0, slot = 0;
            while (a < m) {
                const int b = std::min(m, a + chunk);
                if (b < m && chk_poll) {  // this chunk ends with a check: its copy rides on the chunk's last SpMV
                    chk_seq_of[slot] = ++c->chk_seq;
                    c->chk_word[128 + size_t(slot) * 64] = chk_seq_of[slot];  // (read by the kernel at run time)
                    L.chk_dst = L.chk_slot(slot);
                    L.chk_word = c->chk_word + size_t(slot) * 64;
                    L.chk_seq_src = c->chk_word + 128 + size_t(slot) * 64;
                    L.chk_b = b;
                    L.chk_folded = false;
                    // EK_CHK_FOLD=1: the copy rides in block 0 of the chunk's last
                    // SpMV instead of its own k_chk_gather launch (opt-in: same
                    // bits, no measurable gain on the headline, r06w A/B)
                    static const bool fold = [] {
                        const char* e = std::getenv("EK_CHK_FOLD");
                        return e && e[0] == '1';
                    }();
                    if (!fold || mr_step) L.chk_dst = nullptr, L.chk_folded = false;
                }
                L.factorize(a, b);
                launched = b;
                int cur = -1;
                if (b < m && chk_poll) {  // the chunk's last SpMV (or a gather after it), then the completion word
                    if (!L.chk_folded) {
                        ek::dev::chk_gather(s, c->alpha.as<double>(), c->offd.as<double>(), c->fn2.as<double>(),
                                            mr_step ? c->cflag.as<double>() : nullptr, b, m, L.CHK_FLAGS,
                                            L.chk_slot(slot), -1, c->chk_word + size_t(slot) * 64, chk_seq_of[slot]);
                    }
                    L.chk_dst = nullptr;
                    L.chk_folded = false;
                    cur = b - 1;
                } else if (b < m) {
                    double* pinned = L.chk_slot(slot);
                    HIPCHK(hipEventRecord(c->chk_done[slot], s));
                    HIPCHK(hipStreamWaitEvent(c->cstream, c->chk_done[slot], 0));
                    if (chk_kernel) {  // one launch writing the pinned slot (device-accessible host memory)
                        ek::dev::chk_gather(c->cstream, c->alpha.as<double>(), c->offd.as<double>(), c->fn2.as<double>(),
                                            mr_step ? c->cflag.as<double>() : nullptr, b, m, L.CHK_FLAGS, pinned);
                    } else {  // (EK_CHK_KERNEL=0: one DMA blit per array)
                        HIPCHK(hipMemcpyAsync(pinned, c->alpha.p, size_t(b) * 8, hipMemcpyDeviceToHost, c->cstream));
                        HIPCHK(hipMemcpyAsync(pinned + m, c->offd.p, size_t(b) * 8, hipMemcpyDeviceToHost, c->cstream));
                        HIPCHK(hipMemcpyAsync(pinned + 2 * m, c->fn2.p, size_t(b) * 8, hipMemcpyDeviceToHost, c->cstream));
                        if (mr_step)
                            HIPCHK(hipMemcpyAsync(pinned + L.CHK_FLAGS, c->cflag.p, size_t(b) * 8, hipMemcpyDeviceToHost,
                                                  c->cstream));
                    }
                    HIPCHK(hipEventRecord(c->chk_copied[slot], c->cstream));
                    cur = b - 1;  // complete: alpha, offd of steps < b - 1 (the fused finalize lags one step), fn2 <= b - 1
                }
                if (pend >= 0) {  // the previous chunk's check, while this chunk runs
                    if (chk_poll) chk_wait(pend_slot, chk_seq_of[pend_slot]);
                    else HIPCHK(hipEventSynchronize(c->chk_copied[pend_slot]));
                    const double* pa = L.chk_slot(pend_slot);
                    const int j = pend;
                    for (int i = from; i < j; ++i) {
                        d[size_t(i)] = pa[i];
                        if (i > 0) e[size_t(i - 1)] = pa[m + i];
                    }
                    double an = 1.0;
                    for (int i = 0; i < j; ++i) an = std::max(an, std::fabs(d[size_t(i)]) + (i > 0 ? std::fabs(e[size_t(i - 1)]) : 0.0));
                    for (int i = std::max(from, 1); i <= j && j1 < 0; ++i)
                        if (!(std::sqrt(std::max(0.0, pa[2 * m + i])) > beta_eps * an)) j1 = i;
                    for (int i = from; mr_step && i < j && jr < 0; ++i)
                        if (pa[L.CHK_FLAGS + size_t(i)] != 0.0) {
                            jr = i + 1;
                            beta_r = std::sqrt(std::max(0.0, pa[2 * m + jr]));
                        }
                    if (j1 >= 0 || jr >= 0) break;
                    // only the nev smallest Ritz values and their last components
                    // (bisection + inverse iteration: ~70 us at j = 100 against
                    // ~370 us for all j by QL; with partial reorthogonalisation a
                    // chunk of steps is shorter than the QL took, and the GPU
                    // waited for the check before the next chunk's launches)
                    if (!ek::tridiag_smallest(j, d.data(), e.data(), std::min(nev, j), theta.data(), zl.data()))
                        ek::fail(EK_ENOCONV, "tridiagonal eigensolver failed");
                    const double fj = std::sqrt(std::max(0.0, pa[2 * m + j]));
                    int nc = 0;
                    for (int i = 0; i < nev && i < j; ++i)
                        if (std::fabs(zl[size_t(i)]) * fj < tol * std::max(eps23, std::fabs(theta[size_t(i)]))) ++nc;
                    if (trace)
                        std::fprintf(stderr, "[lanczos]   check j=%d theta0=%.15g est0=%.3e\n", j, theta[0],
                                     std::fabs(zl[0]) * fj);
                    if (nc >= nev) {
                        jconv = j;
                        break;
                    }
                }
                pend = cur;
                pend_slot = slot;
                slot ^= 1;
                a = b;
            }
            L.collect_spmv_times(launched);
            if (jconv > 0) break;
            if (j1 < 0 && jr < 0) {  // the whole cycle ran: its projected matrix and residuals (pinned slot 0:
                           // no check copy is in flight at the cycle's end)
                double* pin0 = L.chk_slot(0);
                if (chk_kernel) {
                    ek::dev::chk_gather(s, c->alpha.as<double>(), c->offd.as<double>(), c->fn2.as<double>(), nullptr, m,
                                        m, 0, pin0, m + 1);
                } else {
                    HIPCHK(hipMemcpyAsync(pin0, c->alpha.p, size_t(m) * 8, hipMemcpyDeviceToHost, s));
                    HIPCHK(hipMemcpyAsync(pin0 + m, c->offd.p, size_t(m) * 8, hipMemcpyDeviceToHost, s));
                    HIPCHK(hipMemcpyAsync(pin0 + 2 * m, c->fn2.p, size_t(m + 1) * 8, hipMemcpyDeviceToHost, s));
                }
                HIPCHK(hipStreamSynchronize(s));
                std::copy(pin0, pin0 + m, alpha_h.begin());
                std::copy(pin0 + m, pin0 + 2 * m, offd_h.begin());
                std::copy(pin0 + 2 * m, pin0 + 3 * m + 1, fn2_h.begin());
                for (int i = from; i < m; ++i) {
                    d[size_t(i)] = alpha_h[size_t(i)];
                    if (i > 0) e[size_t(i - 1)] = offd_h[size_t(i)];
                }
                const double anorm = anorm_of();
                for (int i = std::max(from, 1); i < m; ++i)
                    if (!(std::sqrt(std::max(0.0, fn2_h[size_t(i)])) > beta_eps * anorm)) {
                        j1 = i;
                        break;
                    }
                if (mr_step && j1 < 0) {
                    std::vector<double> cf(static_cast<size_t>(m));
                    HIPCHK(hipMemcpyAsync(cf.data(), c->cflag.p, size_t(m) * 8, hipMemcpyDeviceToHost, s));
                    HIPCHK(hipStreamSynchronize(s));
                    for (int i = from; i < m && jr < 0; ++i)
                        if (cf[size_t(i)] != 0.0) {
                            jr = i + 1;
                            beta_r = std::sqrt(std::max(0.0, fn2_h[size_t(jr)]));
                        }
                }
                if (j1 < 0 && jr < 0) break;
            } else {
                HIPCHK(hipStreamSynchronize(s));  // the chunk launched beyond the breakdown / cancellation
            }
            if (j1 >= 0 && (jr < 0 || j1 <= jr)) {
                if (trace) std::fprintf(stderr, "[lanczos] breakdown at step %d\n", j1);
                if (++cycle_breakdowns > m) ek::fail(EK_ENOCONV, "Lanczos: repeated breakdown within one cycle");
                L.inject(j1, ++injected);
                from = j1;
            } else {
                if (trace) std::fprintf(stderr, "[lanczos] cancelled f' at step %d: re-projected\n", jr - 1);
                const auto corr = L.repair(jr, beta_r);
                d[size_t(jr - 1)] += corr.first;
                if (jr >= 2) e[size_t(jr - 2)] += corr.second;
                HIPCHK(hipMemsetAsync(c->cflag.as<double>() + jr - 1, 0, 8, s));
                if (jr == m) {  // f_m re-projected in place: the cycle's residual norm again
                    HIPCHK(hipMemcpyAsync(&fn2_h[size_t(m)], c->fn2.as<double>() + m, 8, hipMemcpyDeviceToHost, s));
                    HIPCHK(hipStreamSynchronize(s));
                    break;
                }
                from = jr;
            }
        }
        if (jconv > 0) {
            HIPCHK(hipStreamSynchronize(s));
            device_cycle_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc).count();
            converged = true;
            mf = jconv;
            break;
        }
        const auto th = std::chrono::steady_clock::now();
        device_cycle_ms += std::chrono::duration<double, std::milli>(th - tc).count();
        if (!ek::tridiag_eig(m, d.data(), e.data(), theta.data(), zl.data(), nullptr))
            ek::fail(EK_ENOCONV, "tridiagonal eigensolver failed");
        host_ql_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th).count();
        const double fnorm = std::sqrt(std::max(0.0, fn2_h[size_t(m)]));
        if (!std::isfinite(fnorm)) ek::fail(EK_ENOCONV, "Lanczos breakdown (non-finite residual)");
        nconv = 0;
        for (int i = 0; i < nev; ++i) {  // Spectra num_converged
            const double thresh = tol * std::max(eps23, std::fabs(theta[size_t(i)]));
            if (std::fabs(zl[size_t(i)]) * fnorm < thresh) ++nconv;
        }
        if (trace)
            std::fprintf(stderr, "[lanczos] restart %d k=%d theta0=%.15g est0=%.3e theta1=%.15g fnorm=%.3e\n", restarts,
                         k, theta[0], std::fabs(zl[0]) * fnorm, theta[1], fnorm);
        if (nconv >= nev) {
            converged = true;
            break;
        }
        if (++restarts >= maxit) break;
        // EK_LANCZOS_ORTHO=1 (tests): max |[V u0]^T [V u0] - I| over the
        // cycle's basis at every restart (one projection per column)
        if (ortho_check) {
            std::vector<double> hh(size_t(m + L.has_u0));
            for (int j = 0; j < m; ++j) {
                ek::dev::gemvt(s, L.ldv, L.nrb, L.V(), m, L.has_u0, L.u0val, L.nreal, L.col(j), c->part.as<double>());
                ek::dev::reduce_cols(s, c->part.as<double>(), L.nrb, m + L.has_u0, c->h1.as<double>());
                allreduce(c, c->h1.as<double>(), size_t(m + L.has_u0));  // (sharded: each rank's rows)
                HIPCHK(hipMemcpyAsync(hh.data(), c->h1.p, hh.size() * 8, hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
                for (int q = 0; q < m + L.has_u0; ++q)
                    ortho_max = std::max(ortho_max, std::fabs(hh[size_t(q)] - (q == j ? 1.0 : 0.0)));
            }
        }
        // implicit restart with the m-knew unwanted Ritz values as shifts
        // (a fixed restart size of 8, 12 or 20 kept vectors, or a cap of 10-30,
        // was no better over ibm01 / industry2 / ibm10 / the 1x synthetic and
        // its largest component, and some sizes lost 3-12x on one of them)
        const bool floor_on = keep_min > 0 && std::fabs(theta[size_t(nev - 1)]) > 1e-8 * anorm_of();
        // Where the floor applies, it replaces ARPACK's jump to ncv/2 kept
        // vectors (taken when no unwanted Ritz estimate is below eps): which
        // side of eps those estimates fall on is rounding noise, and the jump
        // turned the headline's 6 restarts into 9 (50 kept instead of 20, the
        // same 527 matvecs: 20.0 -> 18.5 ms, tools/restart_ab.py,
        // profiles/r05/restart_ab_keephalf.txt).  EK_KEEP_HALF=1 keeps it.
        const char* kh_env = std::getenv("EK_KEEP_HALF");
        const bool keep_half = kh_env && kh_env[0] == '1';
        int knew = nev_adjusted(nev, m, nconv, zl, !floor_on || keep_half);
        // a floor on Spectra's count: its rule keeps ncv/2 when no unwanted
        // Ritz value has converged but only 1 + (those with |e_m^T y| < eps)
        // otherwise, 2-4 vectors on these Laplacians, and a restart that
        // keeps 3 of 100 throws the subspace away (the 1.15x LCC: 755
        // matvecs with Spectra's rule, 527 with a floor of 20; tools/restart_ab.py)
        // Not when the wanted Ritz value is numerically zero: a disconnected
        // graph, whose null space is degenerate; there keeping more vectors
        // slowed convergence to a null vector (10x synthetic: 362 matvecs
        // with Spectra's rule, 756 with a floor of 10, 994 with 20; the 1x
        // and 2x synthetics likewise)
        if (floor_on) knew = std::max(knew, std::min(keep_min, m - 1));
        if (trace) std::fprintf(stderr, "[lanczos]   keep %d (matvecs so far %d)\n", knew, L.matvecs);
        std::vector<double> dd(d), ee(e);
        const auto tq0 = std::chrono::steady_clock::now();
        // the unwanted Ritz values as shifts; of Q only the kept columns and
        // the residual's are used: formed right to left from the rotations
        // (ek::accumulate_q).  (A device form that applied the rotations with
        // one workgroup, k_apply_rots, lost: ~9k dependent rotations took 1.36
        // ms per restart against ~0.3 ms on the host for all of Q.)
        rots.clear();
        ek::tridiag_qr_shifts(m, dd.data(), ee.data(), theta.data() + knew, m - knew, rots);
        double* Q = c->q_pin;  // pinned: the upload below is a plain DMA
        ek::accumulate_q(m, rots, knew + 1, Q, qscratch);
        const double sigma = Q[size_t(knew - 1) * m + size_t(m - 1)];  // Q(m-1, knew-1)
        host_qr_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count();
        // the restart's transfers and the next cycle's resets are queued with
        // the GEMM, all through pinned staging, so the one synchronisation
        // below waits for the device work alone (as pageable copies between
        // host wake-ups they left the GPU idle ~30 us a restart): Q, the kept
        // projected matrix and the beta-override reset in one launch that
        // reads the staging directly (three blits and a fill before)
        double* kp = c->q_pin + size_t(ek::dev::MAX_NCV) * size_t(ek::dev::MAX_NCV + 1);
        double* fn2_pin = kp + 2 * (ek::dev::MAX_NCV + 2) - 1;  // (kp uses [0, 2 knew))
        if (L.pro) {  // the kept projected matrix, for k_pro's omega recurrence (alpha[j], offd[j] of j < knew)
            for (int i = 0; i < knew; ++i) kp[i] = dd[size_t(i)];
            for (int i = 1; i < knew; ++i) kp[knew + i] = ee[size_t(i - 1)];
        }
        ek::dev::restart_upload(s, Q, m * (knew + 1), c->Qd.as<double>(), L.pro ? kp : nullptr, knew,
                                c->alpha.as<double>(), c->offd.as<double>(), c->bov.as<double>(),
                                int(c->bov.bytes / 8));
        const double hk = ee[size_t(knew - 1)];  // H(knew, knew-1)
        ek::dev::gemm_vq(s, L.ldv, L.V(), m, c->Qd.as<double>(), knew + 1, c->Vn.as<double>(),
                         L.b32 ? c->Vn32.as<float>() : nullptr);
        ek::dev::axpby_norm(s, L.ldv, c->f.as<double>(), sigma, c->Vn.as<double>() + size_t(knew) * ldv, hk,
                            c->npart.as<double>());
        L.reduce_scalar(c->fn2.as<double>() + knew);
        HIPCHK(hipMemcpyAsync(fn2_pin, c->fn2.as<double>() + knew, 8, hipMemcpyDeviceToHost, s));
        if (mr_step) HIPCHK(hipMemsetAsync(c->cflag.p, 0, c->cflag.bytes, s));  // the next cycle's flags
        cycle_reset = true;
        std::swap(c->V.p, c->Vn.p);
        std::swap(c->V.bytes, c->Vn.bytes);
        if (L.b32) {
            std::swap(c->V32.p, c->Vn32.p);
            std::swap(c->V32.bytes, c->Vn32.bytes);
        }
        const auto tsy = std::chrono::steady_clock::now();
        HIPCHK(hipStreamSynchronize(s));  // Q upload buffer reused next restart; fn2_k read (and k_pro's staging)
        fn2_k = *fn2_pin;
        restart_sync_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tsy).count();
        if (L.pro && std::getenv("EK_PRO_TRACE")) {  // (lab: the cycle's per-step decisions)
            std::vector<int> fl(static_cast<size_t>(m));
            HIPCHK(hipMemcpy(fl.data(), c->pflags.p, size_t(m) * 4, hipMemcpyDeviceToHost));
            std::string row;
            for (int i = k; i < m; ++i) row += fl[size_t(i)] ? '1' : '0';
            std::fprintf(stderr, "[pro] cycle from %d: %s\n", k, row.c_str());
            for (int i = k; i < m; ++i)
                std::fprintf(stderr, "[pro] %d d %a e %a\n", i, d[size_t(i)], i + 1 < m ? e[size_t(i)] : 0.0);
        }
        for (int i = 0; i < knew; ++i) d[size_t(i)] = dd[size_t(i)];
        for (int i = 0; i + 1 < knew; ++i) e[size_t(i)] = ee[size_t(i)];
        k = knew;
        host_restart_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th).count();
    }
    if (trace)
        std::fprintf(stderr, "[lanczos] factorization cycles %.3f ms, restarts %.3f ms (of which QL %.3f ms, QR shifts "
                     "%.3f ms, waiting for the restart's device work %.3f ms)\n",
                     device_cycle_ms, host_restart_ms, host_ql_ms, host_qr_ms, restart_sync_ms);
    if (!converged)
        ek::fail(EK_ENOCONV, "Eigenvalue computation failed: %d of %d Ritz pairs converged after %d restarts", nconv,
                 nev, restarts);
    // Ritz vector of the wanted value (ascending: [0] is the null pair unless deflated)
    const int want = deflate ? 0 : 1;
    std::vector<double> Z(size_t(mf) * mf);
    ek::tridiag_eig(mf, d.data(), e.data(), theta.data(), zl.data(), Z.data());
    const double lambda = theta[size_t(want)];
    HIPCHK(hipMemcpyAsync(c->Qd.p, Z.data() + size_t(want) * mf, size_t(mf) * 8, hipMemcpyHostToDevice, s));
    double* xloc = c->Vn.as<double>();
    ek::dev::gemm_vq(s, L.ldv, L.V(), mf, c->Qd.as<double>(), 1, xloc);
    // full vector on every rank; copied out through pinned staging kept by the
    // context (pageable copies of these 2 x 8n bytes cost ~0.5 ms a solve)
    // (+ tail: the final step's small read-backs, below: one residual partial
    // per 512 rows, then the in-launch waits' state and the fallback count in
    // the last 8 doubles; at least 4,096 so small graphs keep one allocation)
    const size_t tail = std::max<size_t>(4096, (size_t(std::max(L.nub, 0)) + 8 + 63) & ~size_t(63));
    const size_t need = size_t(n) + size_t(std::max<int64_t>(c->nrows, 1)) + tail;
    if (c->pin_doubles < need) {
        if (c->pin) HIPCHK(hipHostFree(c->pin));
        c->pin = nullptr;
        c->pin_doubles = 0;
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->pin), need * 8, hipHostMallocDefault));
        c->pin_doubles = need;
    }
    double* v = c->pin;
    double* y = c->pin + n;
    double* xg = xloc;   // the vector as the SpMV reads it
    double* xc = xloc;   // ... and contiguous over the global rows
    if (c->mr) {  // the padded slot layout, then compacted
        allgather(c, xloc, size_t(c->slot), c->xfull.as<double>());
        xg = c->xfull.as<double>();
        c->xexp.ensure(size_t(n) * 8);
        xc = c->xexp.as<double>();
        for (int r = 0; r < c->nranks; ++r) {
            const int64_t a = c->shard_off[size_t(r)], b = c->shard_off[size_t(r) + 1];
            if (b > a)
                HIPCHK(hipMemcpyAsync(xc + a, xg + r * c->slot, size_t(b - a) * 8, hipMemcpyDeviceToDevice, s));
        }
        if (c->halo) {  // the residual's SpMV reads the compact layout: from the full vector, no collective
            ek::dev::gather_idx(s, xc, c->hx_gidx.as<int>(), (long long)x_extent(c), c->hx_X.as<double>());
            xg = c->hx_X.as<double>();
        }
    }
    HIPCHK(hipMemcpyAsync(v, xc, size_t(n) * 8, hipMemcpyDeviceToHost, s));
    // single context: the residual (a diagnostic) is reduced on the device
    // while the host scales the vector, and the final read-backs (residual
    // partials, the in-launch waits' state, the fp64-fallback count) land with
    // ONE synchronisation after fiedler_scale is queued.  (Reading the
    // 1.7 MB residual vector back, summing it on the host and syncing three
    // times left the GPU idle ~0.35 ms a solve at the headline.)
    const bool fin_fast = !c->mr;
    double* rpart = c->pin + size_t(n) + size_t(std::max<int64_t>(c->nrows, 1));  // nub <= tail - 8
    ek::dev::ProState* ps_pin = reinterpret_cast<ek::dev::ProState*>(rpart + tail - 8);
    unsigned* fb_pin = reinterpret_cast<unsigned*>(rpart + tail - 2);
    static_assert(sizeof(ek::dev::ProState) <= 6 * sizeof(double), "ProState overlaps the fallback count");
    if (fin_fast) {
        if (!c->fin_ev) HIPCHK(hipEventCreateWithFlags(&c->fin_ev, hipEventDisableTiming));
        HIPCHK(hipEventRecord(c->fin_ev, s));
    }
    // residual ||L x - lambda x|| on the owned rows
    ek::dev::spmv(s, spmv_mat(c), xg, c->w.as<double>(), nullptr, nullptr, nullptr, nullptr);
    if (fin_fast) {
        ek::dev::resid_partial(s, L.ldv, c->w.as<double>(), xc, lambda, int(c->nrows), c->npart.as<double>());
        HIPCHK(hipMemcpyAsync(rpart, c->npart.p, size_t(L.nub) * 8, hipMemcpyDeviceToHost, s));
        if (L.pro) HIPCHK(hipMemcpyAsync(ps_pin, c->prost.p, sizeof(ek::dev::ProState), hipMemcpyDeviceToHost, s));
        if (L.b32) HIPCHK(hipMemcpyAsync(fb_pin, c->fbk.p, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipEventSynchronize(c->fin_ev));
        double nx2 = 0.0;
        for (int64_t i = 0; i < n; ++i) nx2 += v[i] * v[i];
        if (!(nx2 > 0.0) || !std::isfinite(nx2)) {
            HIPCHK(hipStreamSynchronize(s));
            ek::fail(EK_ENOCONV, "Lanczos: the Ritz vector is zero or not finite (|x|^2 = %g)", nx2);
        }
        const double inv = 1.0 / std::sqrt(nx2);
        int64_t imax = 0;
        for (int64_t i = 1; i < n; ++i)
            if (std::fabs(v[i]) > std::fabs(v[imax])) imax = i;
        const double sgn = v[imax] < 0 ? -inv : inv;
        c->fied.ensure(size_t(n) * 8);
        c->fied_n = 0;  // set only once the solve is known good (a failed solve leaves no vector)
        ek::dev::fiedler_scale(s, xc, sgn, int(n), c->fied.as<double>());
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(s));
        if (L.proi && ps_pin->timeouts)
            ek::fail(EK_EHIP, "Lanczos: %d in-launch wait(s) of the partially reorthogonalised step gave up "
                              "(EK_PRO_INLAUNCH=0 runs the step without them)", ps_pin->timeouts);
        c->fied_n = n;
        double rs = 0.0;
        for (int b = 0; b < L.nub; ++b) rs += rpart[b];
        const double r2 = rs * inv * inv;
        if (c->comm_time) comm_collect(c);
        c->comm_time = false;
        if (lambda_out) *lambda_out = lambda;
        if (v_out)
            for (int64_t i = 0; i < n; ++i) v_out[i] = v[i] * sgn;
        if (stats) {
            stats->restarts = restarts;
            stats->matvecs = L.matvecs;
            stats->converged = 1;
            stats->residual = std::sqrt(r2);
            stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            stats->spmv_ms = L.spmv_ms;
            stats->spmv_timed = L.spmv_timed;
            stats->comm_ms = c->comm_ms;
            stats->allgathers = int32_t(c->n_ag);
            stats->allreduces = int32_t(c->n_ar);
            stats->update32_steps = L.u32_steps;
            stats->update32_fallbacks = L.b32 ? int32_t(*fb_pin) : 0;
            stats->projected_steps = L.pro ? ps_pin->projected : L.matvecs;
            stats->reprojected = L.repairs;
            stats->ortho_max = ortho_max;
        }
        return EK_OK;
    }
    if (c->nrows) HIPCHK(hipMemcpyAsync(y, c->w.p, size_t(c->nrows) * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    double r2 = 0.0, nx2 = 0.0;
    for (int64_t i = 0; i < n; ++i) nx2 += v[i] * v[i];
    if (!(nx2 > 0.0) || !std::isfinite(nx2))
        ek::fail(EK_ENOCONV, "Lanczos: the Ritz vector is zero or not finite (|x|^2 = %g)", nx2);
    const double inv = 1.0 / std::sqrt(nx2);
    for (int64_t i = 0; i < c->nrows; ++i) {
        const double t = (y[i] - lambda * v[c->row0 + i]) * inv;
        r2 += t * t;
    }
    if (c->mr) {
        double* sc = c->scal.as<double>();
        HIPCHK(hipMemcpyAsync(sc, &r2, 8, hipMemcpyHostToDevice, s));
        allreduce(c, sc, 1);
        HIPCHK(hipMemcpyAsync(&r2, sc, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    if (L.proi) {  // the in-launch hand-offs' waits are bounded: any that gave up fails the solve
        ek::dev::ProState ps{};
        HIPCHK(hipMemcpyAsync(&ps, c->prost.p, sizeof(ps), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (ps.timeouts)
            ek::fail(EK_EHIP, "Lanczos: %d in-launch wait(s) of the partially reorthogonalised step gave up "
                              "(EK_PRO_INLAUNCH=0 runs the step without them)", ps.timeouts);
    }
    // deterministic sign: the entry of largest magnitude (first on ties) is positive
    int64_t imax = 0;
    for (int64_t i = 1; i < n; ++i)
        if (std::fabs(v[i]) > std::fabs(v[imax])) imax = i;
    const double sgn = v[imax] < 0 ? -inv : inv;
    c->fied.ensure(size_t(n) * 8);
    ek::dev::fiedler_scale(s, xc, sgn, int(n), c->fied.as<double>());
    HIPCHK(hipGetLastError());
    c->fied_n = n;
    if (c->comm_time) {
        HIPCHK(hipStreamSynchronize(s));
        comm_collect(c);
    }
    c->comm_time = false;
    if (lambda_out) *lambda_out = lambda;
    if (v_out)
        for (int64_t i = 0; i < n; ++i) v_out[i] = v[i] * sgn;
    if (stats) {
        stats->restarts = restarts;
        stats->matvecs = L.matvecs;
        stats->converged = 1;
        stats->residual = std::sqrt(r2);
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        stats->spmv_ms = L.spmv_ms;
        stats->spmv_timed = L.spmv_timed;
        stats->comm_ms = c->comm_ms;
        stats->allgathers = int32_t(c->n_ag);
        stats->allreduces = int32_t(c->n_ar);
        stats->update32_steps = L.u32_steps;
        stats->update32_fallbacks = 0;
        stats->projected_steps = L.matvecs;  // every step projects unless partial reorthogonalisation ran
        stats->reprojected = L.repairs;
        stats->ortho_max = ortho_max;
        if (L.pro) {
            ek::dev::ProState ps{};
            HIPCHK(hipMemcpyAsync(&ps, c->prost.p, sizeof(ps), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            stats->projected_steps = ps.projected;
        }
        if (L.b32) {
            unsigned fbn = 0;
            HIPCHK(hipMemcpyAsync(&fbn, c->fbk.p, 4, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            stats->update32_fallbacks = int32_t(fbn);
        }
    }
    return EK_OK;
    EK_CATCH
}

// ---------------------------------------------------------------------------
// KL driver (KL(), cKL.cpp:288-406)
extern "C" {

int ek_kl_graph_setup(ek_ctx* c, int64_t n, const int32_t* rowptr, const int32_t* col, const float* w) {
    EK_TRY
    check_ctx(c);
    ek::PhaseTimer pt("kl_graph_setup");
    if (n <= 0 || n > INT32_MAX || !rowptr || !col || !w) ek::fail(EK_EINVAL, "ek_kl_graph_setup: bad argument");
    const int64_t nnz = rowptr[n];
    for (int64_t r = 0; r < n; ++r)
        if (rowptr[r + 1] < rowptr[r]) ek::fail(EK_EINVAL, "ek_kl_graph_setup: rowptr not monotone");
    {
        std::atomic<bool> bad{false};
        ek::parallel_for(nnz, [&](int64_t lo, int64_t hi) {
            for (int64_t p = lo; p < hi; ++p)
                if (col[p] < 0 || col[p] >= n) bad = true;
        });
        if (bad) ek::fail(EK_EINVAL, "ek_kl_graph_setup: column out of range");
    }
    pt.mark("checks");
    hipStream_t s = c->kstream;
    // not ready until this setup has finished: a failure part-way must not
    // leave the previous graph's flags over this one's sizes
    c->kl_graph_ready = false;
    c->kl_part_ready = false;
    c->kl_n = n;
    c->kl_rowptr_h.assign(rowptr, rowptr + n + 1);
    Uploader up(c, s, (size_t(n) + 1) * 4 + size_t(nnz) * 8 + size_t(nnz) * 4);
    up.put(c->kl_rowptr, rowptr, size_t(n) + 1);
    // 16 zero entries of tail padding: the swap loop reads rows 16 at a time unconditionally
    c->kl_col.ensure((size_t(nnz) + 16) * 4);
    c->kl_w.ensure((size_t(nnz) + 16) * 4);
    HIPCHK(hipMemsetAsync(c->kl_col.as<int32_t>() + nnz, 0, 16 * 4, s));
    HIPCHK(hipMemsetAsync(c->kl_w.as<float>() + nnz, 0, 16 * 4, s));
    if (nnz) {
        // (the staging copies on the host threads: ~9 MB at ibm18 shape)
        unsigned char* const dc = up.buf + up.off;
        unsigned char* const dw = dc + size_t(nnz) * 4;
        ek::parallel_for(nnz, [&](int64_t lo, int64_t hi) {
            std::memcpy(dc + size_t(lo) * 4, col + lo, size_t(hi - lo) * 4);
            std::memcpy(dw + size_t(lo) * 4, w + lo, size_t(hi - lo) * 4);
        });
        HIPCHK(hipMemcpyAsync(c->kl_col.p, dc, size_t(nnz) * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(c->kl_w.p, dw, size_t(nnz) * 4, hipMemcpyHostToDevice, s));
        up.off += size_t(nnz) * 8;
    }
    pt.mark("CSR staged");
    // inline neighbour-row segments for the swap loop: weight-coded (128 B per
    // entry) when the distinct weights fit the code bits and the LDS table,
    // else plain (256 B per entry); skipped past 32 GB.  EK_KL_NOSEGC=1 at
    // setup: plain (A/B, tests).
    std::vector<uint32_t> kw;
    std::vector<float> wdict;
    int wcolbits = 0;
    c->kl_segc_ok = !std::getenv("EK_KL_NOSEGC") &&
                    size_t(nnz) * ek::dev::KL_SEGC_PIECES * sizeof(ek::dev::KLInfo) <= (size_t(32) << 30) &&
                    ek::dev::kl_weight_codes(n, nnz, col, w, kw, wdict, wcolbits);
    pt.mark("weight codes");
    c->kl_seg_ok = !c->kl_segc_ok && size_t(nnz) * ek::dev::KL_SEG_LANES * sizeof(ek::dev::KLInfo) <= (size_t(32) << 30);
    if (c->kl_segc_ok) {
        DBuf dkw;
        up.put(dkw, kw.data(), kw.size());
        upload(c->kl_wdict, wdict.data(), wdict.size(), s);
        c->kl_nwd = int(wdict.size());
        c->kl_wcolbits = wcolbits;
        c->kl_seg.reset();
        c->kl_segc.ensure(size_t(std::max<int64_t>(nnz, 1)) * ek::dev::KL_SEGC_PIECES * sizeof(ek::dev::KLInfo));
        ek::dev::kl_build_segc(s, nnz, c->kl_rowptr.as<int32_t>(), c->kl_col.as<int32_t>(), dkw.as<uint32_t>(),
                               c->kl_segc.as<ek::dev::KLInfo>());
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(s));  // dkw is freed at scope end
    }
    if (c->kl_seg_ok) {
        c->kl_segc.reset();
        c->kl_seg.ensure(size_t(std::max<int64_t>(nnz, 1)) * ek::dev::KL_SEG_LANES * sizeof(ek::dev::KLInfo));
        ek::dev::kl_build_seg(s, nnz, c->kl_rowptr.as<int32_t>(), c->kl_col.as<int32_t>(), c->kl_w.as<float>(),
                              c->kl_seg.as<ek::dev::KLInfo>());
        HIPCHK(hipGetLastError());
    }
    c->kl_side.ensure(size_t(n));
    c->kl_side_init.ensure(size_t(n));
    // (also the side / locked bitmaps of the on-chip loop when they exceed
    // its LDS budget: 2 ceil(n/32) words, k_kl_swap_loop<.., GB>)
    c->kl_locked.ensure(std::max(size_t(n), size_t((n + 31) / 32) * 8 + 64));
    c->kl_plist.ensure(size_t(n) * 4);
    c->kl_sides_tmp.ensure(size_t(n));
    c->kl_cutpart.ensure(size_t((n + 255) / 256) * 8);
    c->kl_cut0.ensure(16);
    c->kl_out.ensure(sizeof(ek::dev::KLOut));
    c->kl_count.ensure(64);
    pt.mark("segments queued");
    HIPCHK(hipStreamSynchronize(s));
    pt.mark("synchronised");
    c->kl_graph_ready = true;
    c->kl_part_ready = false;
    return EK_OK;
    EK_CATCH
}

int ek_kl_nets_setup(ek_ctx* c, int64_t nets, const int64_t* net_ptr, const int32_t* pins) {
    EK_TRY
    check_ctx(c);
    if (nets < 0 || !net_ptr || (net_ptr[nets] > 0 && !pins)) ek::fail(EK_EINVAL, "ek_kl_nets_setup: bad argument");
    c->kl_nets = nets;
    Uploader up(c, c->kstream, (size_t(nets) + 1) * 8 + size_t(net_ptr[nets]) * 4);
    up.put(c->kl_netptr, net_ptr, size_t(nets) + 1);
    up.put(c->kl_pins, pins, size_t(net_ptr[nets]));
    c->kl_count.ensure(size_t(3) * size_t(ek::dev::net_cut_blocks(nets)) * sizeof(unsigned));  // ek_kl_run's cut partials
    HIPCHK(hipStreamSynchronize(c->kstream));
    return EK_OK;
    EK_CATCH
}

}  // extern "C"

namespace {
// The rest of the partition setup once remain[] lists, plist and the initial
// sides are on the device (uploaded, or split there from the Fiedler vector)
void partition_on_device(ek_ctx* c, int64_t n0, int64_t n1) {
    hipStream_t s = c->stream;
    const int64_t n = c->kl_n;
    c->kl_n0 = n0;
    c->kl_n1 = n1;
    // row descriptors: by position {node, rowptr, rowlen} and by node {rowptr,
    // rowlen, plist}, built on the device from the lists just uploaded (the
    // by-position arrays are padded to whole chunks with zero descriptors, and
    // the gains with NaN = invalid keys, so the chunk scans load unconditionally)
    {
        c->kl_pinfo0.ensure(size_t(chunk_pad(n0)) * sizeof(ek::dev::KLInfo));
        c->kl_pinfo1.ensure(size_t(chunk_pad(n1)) * sizeof(ek::dev::KLInfo));
        c->kl_nd.ensure(size_t(std::max<int64_t>(n, 1)) * sizeof(ek::dev::KLInfo));
        ek::dev::kl_build_desc(s, int(n), int(n0), int(n1), int(chunk_pad(n0)), int(chunk_pad(n1)),
                               c->kl_order0.as<int32_t>(), c->kl_order1.as<int32_t>(), c->kl_plist.as<uint32_t>(),
                               c->kl_rowptr.as<int32_t>(), c->kl_pinfo0.as<ek::dev::KLInfo>(),
                               c->kl_pinfo1.as<ek::dev::KLInfo>(), c->kl_nd.as<ek::dev::KLInfo>());
        HIPCHK(hipGetLastError());
        const int64_t nnz = c->kl_rowptr_h[size_t(n)];
        c->kl_aux.ensure(size_t(std::max<int64_t>(nnz, 1)) * sizeof(ek::dev::KLInfo));
        ek::dev::kl_build_aux(s, nnz, c->kl_col.as<int32_t>(), c->kl_nd.as<ek::dev::KLInfo>(),
                              c->kl_aux.as<ek::dev::KLInfo>());
        HIPCHK(hipGetLastError());
        c->kl_cinfo0.ensure(size_t((n0 + ek::dev::KL_CHUNK - 1) / ek::dev::KL_CHUNK + 1) * sizeof(ek::dev::KLInfo));
        c->kl_cinfo1.ensure(size_t((n1 + ek::dev::KL_CHUNK - 1) / ek::dev::KL_CHUNK + 1) * sizeof(ek::dev::KLInfo));
    }
    c->kl_gp0.ensure(size_t(chunk_pad(n0)) * 4);
    c->kl_gp1.ensure(size_t(chunk_pad(n1)) * 4);
    HIPCHK(hipMemsetAsync(c->kl_gp0.p, 0xFF, c->kl_gp0.bytes, s));  // NaN padding
    HIPCHK(hipMemsetAsync(c->kl_gp1.p, 0xFF, c->kl_gp1.bytes, s));
    c->kl_ckey0.ensure(size_t((n0 + ek::dev::KL_CHUNK - 1) / ek::dev::KL_CHUNK + 1) * 8);
    c->kl_ckey1.ensure(size_t((n1 + ek::dev::KL_CHUNK - 1) / ek::dev::KL_CHUNK + 1) * 8);
    c->kl_log.ensure(size_t(std::max<int64_t>(1, std::min(n0, n1))) * sizeof(ek_swap));
    HIPCHK(hipStreamSynchronize(s));
    c->kl_part_ready = true;
}

}  // namespace

extern "C" {

int ek_kl_set_partition(ek_ctx* c, const int32_t* order0, int64_t n0, const int32_t* order1, int64_t n1) {
    EK_TRY
    check_ctx(c);
    if (!c->kl_graph_ready) ek::fail(EK_ESTATE, "ek_kl_set_partition before ek_kl_graph_setup");
    const int64_t n = c->kl_n;
    if (n0 < 0 || n1 < 0 || n0 + n1 != n || (n0 && !order0) || (n1 && !order1))
        ek::fail(EK_EINVAL, "ek_kl_set_partition: the two lists must cover all %lld nodes", (long long)n);
    std::vector<uint8_t> side(size_t(n), 2);
    std::vector<uint32_t> plist(size_t(n), 0);
    for (int64_t i = 0; i < n0; ++i) {
        const int32_t u = order0[i];
        if (u < 0 || u >= n || side[size_t(u)] != 2) ek::fail(EK_EINVAL, "ek_kl_set_partition: bad/duplicate node %d", u);
        side[size_t(u)] = 0;
        plist[size_t(u)] = uint32_t(i);
    }
    for (int64_t i = 0; i < n1; ++i) {
        const int32_t u = order1[i];
        if (u < 0 || u >= n || side[size_t(u)] != 2) ek::fail(EK_EINVAL, "ek_kl_set_partition: bad/duplicate node %d", u);
        side[size_t(u)] = 1;
        plist[size_t(u)] = uint32_t(i) | 0x80000000u;
    }
    hipStream_t s = c->stream;
    Uploader up(c, s, size_t(n0) * 4 + size_t(n1) * 4 + size_t(n) + size_t(n) * 4);
    up.put(c->kl_order0, order0, size_t(n0));
    up.put(c->kl_order1, order1, size_t(n1));
    up.put(c->kl_side_init, side.data(), size_t(n));
    up.put(c->kl_plist, plist.data(), size_t(n));
    partition_on_device(c, n0, n1);
    return EK_OK;
    EK_CATCH
}

int ek_kl_set_partition_fiedler(ek_ctx* c, double* median_out, int64_t* n0_out, int64_t* n1_out) {
    EK_TRY
    check_ctx(c);
    if (!c->kl_graph_ready) ek::fail(EK_ESTATE, "ek_kl_set_partition_fiedler before ek_kl_graph_setup");
    const int64_t n = c->kl_n;
    if (c->fied_n != n || n < 1)
        ek::fail(EK_ESTATE, "ek_kl_set_partition_fiedler: no Fiedler vector of %lld entries on this context",
                 (long long)n);
    if (n > INT32_MAX - 1) ek::fail(EK_EINVAL, "ek_kl_set_partition_fiedler: %lld nodes", (long long)n);
    hipStream_t s = c->stream;
    const int ni = int(n);
    const double* v = c->fied.as<double>();
    const size_t tb = ek::dev::split_tmp_bytes(ni);
    c->sp_tmp.ensure(tb);
    c->sp_out.ensure(64);
    // the median: ranks n/2 (and n/2 - 1 for even n, their mean), the values
    // nth_element gives ek_median_split (a radix select on the device)
    const unsigned hi = unsigned(n / 2), lo = n % 2 == 0 ? hi - 1 : hi;
    auto* keys = c->sp_out.as<unsigned long long>();
    ek::dev::split_select(s, c->sp_tmp.p, v, ni, lo, hi, keys);
    unsigned long long kk[2] = {0ull, 0ull};
    HIPCHK(hipMemcpyAsync(kk, keys, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const double mid[2] = {ek::dev::key_value(kk[0]), ek::dev::key_value(kk[1])};
    const double med = n % 2 == 0 ? (mid[0] + mid[1]) / 2.0 : mid[0];
    c->kl_order0.ensure(size_t(n) * 4);
    c->kl_order1.ensure(size_t(n) * 4);
    c->kl_side_init.ensure(size_t(n));
    c->kl_plist.ensure(size_t(n) * 4);
    unsigned* n0_dev = reinterpret_cast<unsigned*>(c->sp_out.as<unsigned long long>() + 2);
    ek::dev::split_partition(s, c->sp_tmp.p, v, ni, med, c->kl_order0.as<int32_t>(), c->kl_order1.as<int32_t>(),
                             c->kl_plist.as<uint32_t>(), c->kl_side_init.as<uint8_t>(), n0_dev);
    HIPCHK(hipGetLastError());
    unsigned n0u = 0;
    HIPCHK(hipMemcpyAsync(&n0u, n0_dev, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const int64_t n0 = int64_t(n0u);
    partition_on_device(c, n0, n - n0);
    if (median_out) *median_out = med;
    if (n0_out) *n0_out = n0;
    if (n1_out) *n1_out = n - n0;
    return EK_OK;
    EK_CATCH
}

int ek_kl_set_partition_bits(ek_ctx* c, int64_t n, const uint8_t* bits) {
    EK_TRY
    if (n < 0 || (n && !bits)) ek::fail(EK_EINVAL, "ek_kl_set_partition_bits: bad argument");
    std::vector<int32_t> o[2];
    o[0].reserve(size_t(n) / 2 + 1);
    o[1].reserve(size_t(n) / 2 + 1);
    for (int64_t i = 0; i < n; ++i) {
        if (bits[i] > 1) ek::fail(EK_EINVAL, "ek_kl_set_partition_bits: bit %d at node %lld", int(bits[i]), (long long)i);
        o[bits[i]].push_back(int32_t(i));
    }
    return ek_kl_set_partition(c, o[0].data(), int64_t(o[0].size()), o[1].data(), int64_t(o[1].size()));
    EK_CATCH
}

}  // extern "C"

namespace {

ek::dev::KLDev kl_dev(ek_ctx* c) {
    ek::dev::KLDev d;
    d.n = int(c->kl_n);
    d.nnz = c->kl_rowptr_h.empty() ? 0 : c->kl_rowptr_h.back();
    d.rowptr = c->kl_rowptr.as<int32_t>();
    d.col = c->kl_col.as<int32_t>();
    d.w = c->kl_w.as<float>();
    d.side = c->kl_side.as<uint8_t>();
    d.side_init = c->kl_side_init.as<uint8_t>();
    d.locked = c->kl_locked.as<uint8_t>();
    d.gp0 = c->kl_gp0.as<float>();
    d.gp1 = c->kl_gp1.as<float>();
    d.order0 = c->kl_order0.as<int32_t>();
    d.order1 = c->kl_order1.as<int32_t>();
    d.plist = c->kl_plist.as<uint32_t>();
    d.pinfo0 = c->kl_pinfo0.as<ek::dev::KLInfo>();
    d.pinfo1 = c->kl_pinfo1.as<ek::dev::KLInfo>();
    d.nd = c->kl_nd.as<ek::dev::KLInfo>();
    d.cinfo0 = c->kl_cinfo0.as<ek::dev::KLInfo>();
    d.cinfo1 = c->kl_cinfo1.as<ek::dev::KLInfo>();
    d.aux = c->kl_aux.as<ek::dev::KLInfo>();
    const bool noseg = std::getenv("EK_KL_NOSEG") != nullptr;  // env: A/B, no inline segments at all
    d.seg = c->kl_seg_ok && !noseg ? c->kl_seg.as<ek::dev::KLInfo>() : nullptr;
    d.segc = c->kl_segc_ok && !noseg ? c->kl_segc.as<ek::dev::KLInfo>() : nullptr;
    d.wdict = c->kl_wdict.as<float>();
    d.nwd = c->kl_nwd;
    d.wcolbits = c->kl_wcolbits;
    d.n0 = int(c->kl_n0);
    d.n1 = int(c->kl_n1);
    d.nck0 = int((c->kl_n0 + ek::dev::KL_CHUNK - 1) / ek::dev::KL_CHUNK);
    d.nck1 = int((c->kl_n1 + ek::dev::KL_CHUNK - 1) / ek::dev::KL_CHUNK);
    d.ckey0 = c->kl_ckey0.as<unsigned long long>();
    d.ckey1 = c->kl_ckey1.as<unsigned long long>();
    d.cut_part = c->kl_cutpart.as<double>();
    d.cut0 = c->kl_cut0.as<float>();
    return d;
}

}  // namespace

extern "C" int ek_kl_run(ek_ctx* c, int32_t limit, ek_swap* log_out, int64_t cap, ek_kl_result* res) {
    EK_TRY
    check_ctx(c);
    if (!c->kl_graph_ready || !c->kl_part_ready) ek::fail(EK_ESTATE, "ek_kl_run before graph/partition setup");
    hipStream_t s = c->stream;
    const int64_t n = c->kl_n;
    const int lim = limit >= 0 ? limit : int(std::log2(double(n))) + 5;  // cKL.cpp:303
    const auto d = kl_dev(c);
    hipEvent_t e0, e1, e2;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventCreate(&e2));
    struct G {
        hipEvent_t a, b, c;
        ~G() {
            (void)hipEventDestroy(a);
            (void)hipEventDestroy(b);
            (void)hipEventDestroy(c);
        }
    } guard{e0, e1, e2};
    const long long dcap = std::max<int64_t>(1, std::min(c->kl_n0, c->kl_n1));
    auto* out = c->kl_out.as<ek::dev::KLOut>();
    HIPCHK(hipEventRecord(e0, s));
    HIPCHK(hipMemcpyAsync(c->kl_side.p, c->kl_side_init.p, size_t(n), hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemsetAsync(c->kl_locked.p, 0, size_t(n), s));
    ek::dev::kl_prepare(s, d);
    HIPCHK(hipEventRecord(e1, s));
    ek::dev::kl_loop(s, d, lim, c->kl_log.as<ek_swap>(), dcap, out);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(e2, s));
    // integer net cuts: initial, best prefix, final
    const bool nets = c->kl_nets > 0;
    const int ncb = nets ? ek::dev::net_cut_blocks(c->kl_nets) : 0;
    std::vector<unsigned> cparts(size_t(3) * size_t(ncb));
    if (nets) {  // one pass over the pins for all three; per-workgroup counts, added here
        ek::dev::kl_replay(s, int(n), c->kl_side_init.as<uint8_t>(), c->kl_log.as<ek_swap>(), &out->best_iter, dcap,
                           c->kl_sides_tmp.as<uint8_t>());
        ek::dev::net_cut(s, c->kl_nets, c->kl_netptr.as<int64_t>(), c->kl_pins.as<int32_t>(),
                         c->kl_side_init.as<uint8_t>(), c->kl_sides_tmp.as<uint8_t>(), c->kl_side.as<uint8_t>(),
                         c->kl_count.as<unsigned>());
    }
    ek::dev::KLOut ho{};
    HIPCHK(hipMemcpyAsync(&ho, out, sizeof ho, hipMemcpyDeviceToHost, s));
    if (nets)
        HIPCHK(hipMemcpyAsync(cparts.data(), c->kl_count.p, cparts.size() * sizeof(unsigned), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (ho.status == 3u)
        ek::fail(EK_EHIP, "KL swap loop: an in-launch wait gave up (EK_KL_PIPE=0 runs the loop without them)");
    unsigned long long hc[3] = {0, 0, 0};
    for (int k = 0; k < 3; ++k)
        for (int b = 0; b < ncb; ++b) hc[k] += cparts[size_t(k) * size_t(ncb) + size_t(b)];
    if (log_out && cap > 0) {
        const int64_t k = std::min<int64_t>(cap, ho.iterations);
        if (k) HIPCHK(hipMemcpy(log_out, c->kl_log.p, size_t(k) * sizeof(ek_swap), hipMemcpyDeviceToHost));
    }
    if (res) {
        float loop_ms = 0.f, prep_ms = 0.f;
        HIPCHK(hipEventElapsedTime(&prep_ms, e0, e1));
        HIPCHK(hipEventElapsedTime(&loop_ms, e1, e2));
        res->iterations = ho.iterations;
        res->initial_cut = ho.initial_cut;
        res->best_cut = ho.best_cut;
        res->final_cut = ho.final_cut;
        res->best_iter = ho.best_iter;
        res->net_cut_initial = nets ? int64_t(hc[0]) : -1;
        res->net_cut_best = nets ? int64_t(hc[1]) : -1;
        res->net_cut_final = nets ? int64_t(hc[2]) : -1;
        res->loop_ms = loop_ms;
        if (std::getenv("EK_KL_PROF") && ho.prof[13] == 0x9199ull) {  // the overlapped loop (k_kl_swap_pipe)
            const double sw = double(std::max<long long>(1, ho.iterations)), gs = double(std::max<unsigned long long>(1, ho.prof[2]));
            std::fprintf(stderr, "[kl-pipe] %lld swaps: speculated %.1f %%, hits %.1f %%; loop %.0f cycles/swap\n",
                         (long long)ho.iterations, 100.0 * double(ho.prof[0]) / sw, 100.0 * double(ho.prof[1]) / gs,
                         double(ho.prof[12]) / sw);
            std::fprintf(stderr, "[kl-pipe] gain wave 0, cycles/swap: pair wait %.0f, P %.0f, speculative rows %.0f (per "
                         "speculation), pair->barrier1 %.0f\n", double(ho.prof[3]) / gs, double(ho.prof[4]) / gs,
                         double(ho.prof[5]) / double(std::max<unsigned long long>(1, ho.prof[0])), double(ho.prof[6]) / gs);
            std::fprintf(stderr, "[kl-pipe] W wave, cycles/swap: barrier-2 wait %.0f, selection %.0f, pair->barrier1 %.0f, "
                         "G2 span %.0f; G2a wave's G2 span %.0f\n", double(ho.prof[7]) / sw, double(ho.prof[8]) / sw,
                         double(ho.prof[9]) / sw, double(ho.prof[10]) / sw, double(ho.prof[11]) / sw);
        } else if (std::getenv("EK_KL_PROF")) {
            static const char* names[12] = {"select", "G1-key", "bar1", "G2a", "G2bc", "bar2", "G1-aux", "G1-sum",
                                            "n_stale", "n_late+tail", "G1-load", "G1-look"};
            std::fprintf(stderr, "[kl] %lld swaps, us/swap:", (long long)ho.iterations);
            for (int i = 0; i < 12; ++i)
                std::fprintf(stderr, " %s %.3f", names[i], ho.prof[i] * 0.01 / std::max<long long>(1, ho.iterations));
            std::fprintf(stderr, "\n");
            if (ho.prof[15])
                std::fprintf(stderr, "[kl] in-loop shader clock %.0f MHz\n", double(ho.prof[14]) / (double(ho.prof[15]) * 0.01));
            if (ho.warr[0] || ho.warr[8]) {
                const double cyc_ns = ho.prof[15] ? double(ho.prof[15]) * 10.0 / double(ho.prof[14]) : 1.0 / 2.4;
                const double f = 1e-3 * cyc_ns / double(std::max<long long>(1, ho.iterations));
                std::fprintf(stderr, "[kl] per wave, us after its loop top: selection done / barrier 1 / G2a done / barrier 2:\n");
                std::fprintf(stderr, "[kl] prefetch predicted node1 in %.1f %%, node2 in %.1f %% of swaps\n",
                             100.0 * double(ho.warr[40]) / double(std::max<long long>(1, ho.iterations)),
                             100.0 * double(ho.warr[41]) / double(std::max<long long>(1, ho.iterations)));
                for (int w = 0; w < 8; ++w)
                    std::fprintf(stderr, "[kl]   w%d %.3f %.3f %.3f %.3f  (G2a reads consumed %.3f)\n", w,
                                 f * double(ho.warr[24 + w]), f * double(ho.warr[w]), f * double(ho.warr[16 + w]),
                                 f * double(ho.warr[8 + w]), f * double(ho.warr[32 + w]));
            }
        }
        res->total_ms = double(loop_ms) + double(prep_ms);
    }
    return EK_OK;
    EK_CATCH
}

extern "C" int ek_kl_sides(ek_ctx* c, int32_t which, uint8_t* sides_out) {
    EK_TRY
    check_ctx(c);
    if (!c->kl_part_ready || !sides_out) ek::fail(EK_ESTATE, "ek_kl_sides: nothing to report");
    hipStream_t s = c->stream;
    const int64_t n = c->kl_n;
    const uint8_t* src = c->kl_side_init.as<uint8_t>();
    if (which == 2) src = c->kl_side.as<uint8_t>();
    if (which == 1) {
        const long long dcap = std::max<int64_t>(1, std::min(c->kl_n0, c->kl_n1));
        ek::dev::kl_replay(s, int(n), c->kl_side_init.as<uint8_t>(), c->kl_log.as<ek_swap>(),
                           &c->kl_out.as<ek::dev::KLOut>()->best_iter, dcap, c->kl_sides_tmp.as<uint8_t>());
        src = c->kl_sides_tmp.as<uint8_t>();
    }
    HIPCHK(hipMemcpyAsync(sides_out, src, size_t(n), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return EK_OK;
    EK_CATCH
}
