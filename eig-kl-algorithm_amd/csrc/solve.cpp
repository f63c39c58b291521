// The whole hot path in-process, .hgr in -> results/ out (ek_solve_file):
// the body the reference splits over two processes and a text file,
//   cEIG <in>    : read, clique Laplacian, Spectra Lanczos, median split
//                  (cEIG.cpp:138-237)
//   cKL <in> -EIG: read, KL adjacency, split from the EIG file, KL loop,
//                  results file (cKL.cpp:288-468)
// with the Fiedler split handed over in memory (gKL2 <in> -EIG, gKL2.cu:989-1033,
// whose "EIG" is replaced by the real Lanczos).  Host phases overlap the GPU:
// the KL adjacency (hash-order emulation) is built on a host thread while the
// GPU runs the Lanczos solve.  Multi-rank contexts shard the Lanczos rows
// (each rank builds and uploads only its rows); the KL loop is rank 0's.
#include <cerrno>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstring>
#include <filesystem>
#include <future>
#include <mutex>
#include <random>
#include <string>
#include <system_error>

#include "ek_internal.hpp"

namespace ek {

namespace {
using clk = std::chrono::steady_clock;
double since(clk::time_point t) { return std::chrono::duration<double>(clk::now() - t).count(); }

void chk(int rc) {
    if (rc != EK_OK) throw Error{rc};  // ek_last_error() already holds the message
}

// The KL adjacency (cKL.cpp:84-149, hash-order emulation) built on host
// threads, then uploaded with the nets (the device-side inline segments and
// weight codes included) on the context's KL stream: all of it while the GPU
// runs the Lanczos solve on the main stream.  A small host copy is freed
// here too, off the solve's path (freeing ~10 MB that several threads
// touched cost the solve's thread ~2.5 ms at the end of a step).  A large
// one goes back to the caller, which frees it on another thread while the
// KL loop runs: the 10x graph's ~100 MB took ~20 ms to unmap, and this
// thread's end is on the path between Lanczos and KL there.
// Its errors come back as {status, message}: the message was written to this
// thread's ek_last_error(), which the caller's thread cannot see.
struct ThreadStatus {
    int code = EK_OK;
    std::string msg;
    std::unique_ptr<ek_csr> host_copy;  // (large graphs) for the caller to free off the path
};
// The host build needs no context: in a fresh process it runs while the HIP
// runtime starts (get_ctx waits for that only before the uploads).
ThreadStatus kl_graph_host(const std::function<ek_ctx*()>* get_ctx, const ek_hgr* h, int threads) {
    ThreadStatus st;
    try {
        PhaseTimer pt("kl_thread");
        ThreadCap cap(threads);
        auto G = std::make_unique<ek_csr>();
        build_kl_graph(*h, *G);
        pt.mark("graph built");
        ek_ctx* ctx = (*get_ctx)();
        chk(ek_kl_graph_setup(ctx, h->nodes, G->rowptr.data(), G->col.data(), G->val32.data()));
        pt.mark("graph set up");
        chk(ek_kl_nets_setup(ctx, h->nets, h->net_ptr.data(), h->pins.data()));
        pt.mark("nets set up");
        if (G->col.size() >= (size_t(1) << 22)) st.host_copy = std::move(G);  // (>= 32 MB of col + val)
    } catch (...) {
        st.code = guard_exceptions();
        st.msg = ek_last_error();
    }
    return st;
}

// the KL adjacency's host threads: beside a Lanczos solve, all but 4 of the
// host's (the solve's thread, the HIP runtime's); EK_KL_GRAPH_THREADS
// overrides (A/B)
int kl_graph_threads(bool beside_solve) {
    if (const char* e = std::getenv("EK_KL_GRAPH_THREADS"); e && std::atoi(e) > 0) return std::atoi(e);
    return beside_solve ? std::max(1, host_threads() - 4) : 0;
}

// the results file's text buffer, kept across calls (one caller at a time)
struct TextCache {
    std::mutex mu;
    dvec<char> buf;
};
TextCache& text_cache() {
    static TextCache c;
    return c;
}

std::string join(const char* dir, const std::string& rel) {
    if (!dir || !dir[0]) return rel;
    return (std::filesystem::path(dir) / rel).string();
}

}  // namespace

// Fiedler vector of this rank's Laplacian rows (cEIG.cpp:86-209): rows built
// on the host, uploaded, Lanczos on the GPU; the full vector on every rank.
void fiedler_vector(ek_ctx* ctx, int rank, int nranks, const ek_hgr& h, const ek_solve_opts& o, double& lambda,
                    std::vector<double>& v, ek_lanczos_stats& st, double* t_laplacian, double* t_lanczos,
                    const std::function<void()>& after_laplacian, double* t_spmv_setup, bool host_v) {
    const int64_t n = h.nodes;
    (void)rank;
    (void)nranks;
    auto t = clk::now();
    // the KL adjacency's host thread starts first: the Laplacian rows are
    // assembled on the GPU, and the adjacency (~3 ms on 12 threads at the
    // headline, ~37 ms at 10x) must finish within the Lanczos solve (~17 ms,
    // ~76 ms) not to stall the KL phase
    if (after_laplacian) after_laplacian();
    // this rank's rows, assembled on the GPU from the pins into the SpMV's
    // coded form (the host build only as ek_spmv_setup_pins' fallback)
    cold_stamp("laplacian_start");
    chk(spmv_setup_hgr(ctx, h, nullptr));
    cold_stamp("laplacian_done");
    if (t_laplacian) *t_laplacian = since(t);
    if (t_spmv_setup) *t_spmv_setup = 0.0;
    t = clk::now();
    // (host_v false: the vector stays on the device for ek_kl_set_partition_fiedler)
    if (host_v) v.assign(size_t(n), 0.0);
    chk(ek_lanczos_fiedler(ctx, &o.lanczos, &lambda, host_v ? v.data() : nullptr, &st));
    cold_stamp("lanczos_done");
    if (host_v && o.sign_ref && o.sign_ref[0]) {
        std::vector<double> ref(static_cast<size_t>(n));
        chk(ek_eig_read(o.sign_ref, n, nullptr, nullptr, nullptr, ref.data(), nullptr, nullptr, nullptr, nullptr));
        chk(ek_align_sign(n, v.data(), ref.data()));
    }
    if (t_lanczos) *t_lanczos = since(t);
}

void solve(const std::function<ek_ctx*()>& get_ctx, int rank, int nranks, const ek_hgr& h, const std::string& base,
           const ek_solve_opts& o, ek_swap* log_out, int64_t cap, ek_solve_result& r) {
    const auto t0 = clk::now();
    const int64_t n = h.nodes;
    r.nets = h.nets;
    r.nodes = n;
    r.pins = int64_t(h.pins.size());
    if (n < 2) fail(EK_EINVAL, "%s: %lld nodes, nothing to partition", base.c_str(), (long long)n);
    // initial partition (shuffleSparceMatrix, cKL.cpp:151-197)
    std::vector<int32_t> order0, order1;
    std::future<ThreadStatus> kg;
    // while the GPU solves, the KL adjacency leaves the solve's host thread
    // (and the HIP runtime's) a few cores
    auto start_kl_graph = [&] {
        if (rank == 0)
            kg = std::async(std::launch::async, kl_graph_host, &get_ctx, &h, kl_graph_threads(o.eig == 1));
    };
    // -EIG without a sign reference: the median split runs on the device,
    // from the Fiedler vector the Lanczos solve left there, once the KL graph
    // is set up (ek_kl_set_partition_fiedler: the same lists, no host round trip)
    const bool dev_split = o.eig == 1 && !(o.sign_ref && o.sign_ref[0]);
    std::vector<double> v;  // (host split only)
    if (o.eig == 1) {
        // the KL adjacency starts on its host thread before the context is
        // asked for (a fresh process: while the HIP runtime starts) and runs
        // while the GPU solves
        start_kl_graph();
        fiedler_vector(get_ctx(), rank, nranks, h, o, r.lambda, v, r.lanczos, &r.t_laplacian, &r.t_lanczos,
                       nullptr, &r.t_spmv_setup, !dev_split);
        if (rank != 0) {
            r.t_total = since(t0);
            return;
        }
    }
    if (o.eig == 1 && !dev_split) {
        const auto t = clk::now();
        std::vector<uint8_t> bits(static_cast<size_t>(n));
        chk(ek_median_split(n, v.data(), &r.median, bits.data()));
        // remain[] lists in node order (cKL.cpp:155-174), built on the host
        // threads: per-chunk counts, then each chunk fills its ranges
        const int T = int(std::min<int64_t>(host_threads(), std::max<int64_t>(1, n / 32768)));
        std::vector<int64_t> z(size_t(T) + 1, 0);
        run_threads(T, [&](int t) {
            int64_t c = 0;
            for (int64_t i = n * t / T; i < n * (t + 1) / T; ++i) c += bits[size_t(i)] == 0;
            z[size_t(t) + 1] = c;
        });
        for (int t = 0; t < T; ++t) z[size_t(t) + 1] += z[size_t(t)];
        order0.resize(size_t(z[size_t(T)]));
        order1.resize(size_t(n - z[size_t(T)]));
        run_threads(T, [&](int t) {
            const int64_t lo = n * t / T;
            int64_t a = z[size_t(t)], b = lo - z[size_t(t)];
            for (int64_t i = lo; i < n * (t + 1) / T; ++i) {
                if (bits[size_t(i)]) order1[size_t(b++)] = int32_t(i);
                else order0[size_t(a++)] = int32_t(i);
            }
        });
        r.t_split = since(t);
    } else if (o.eig != 1) {
        if (rank != 0) {  // the KL loop does not shard: other ranks have nothing to do
            r.t_total = since(t0);
            return;
        }
        const auto t = clk::now();
        if (o.eig == 2) {  // cKL -EIG: pre_saved_EIG/<base>_out.txt (cKL.cpp:442, 155-174)
            const std::string eig_file = join(o.out_dir, "pre_saved_EIG/" + base + "_out.txt");
            order0.resize(size_t(n));
            order1.resize(size_t(n));
            int64_t n0 = 0, n1 = 0;
            if (ek_eig_read(eig_file.c_str(), n, &r.lambda, &r.median, nullptr, nullptr, order0.data(), &n0,
                            order1.data(), &n1) != EK_OK)
                fail(EK_EIO, "Error: EIG file not found (%s)", eig_file.c_str());
            order0.resize(size_t(n0));
            order1.resize(size_t(n1));
        } else {
            order0.resize(size_t(n / 2));
            order1.resize(size_t(n - n / 2));
            chk(ek_random_split(n, o.seed, order0.data(), order1.data()));
        }
        r.t_split = since(t);
        // (after the split: a missing EIG file fails before the GPU is touched)
        start_kl_graph();
    }
    ek_ctx* ctx = get_ctx();
    auto t = clk::now();
    // graph and nets set up on the context (KL stream, synchronised); a
    // failure there is re-raised here with its message
    std::future<void> host_copy_freed;  // (joined when solve returns, long after it is done)
    {
        ThreadStatus st = kg.get();
        if (st.code != EK_OK) fail(st.code, "KL graph setup: %s", st.msg.c_str());
        if (st.host_copy) {
            try {
                host_copy_freed = std::async(std::launch::async, [p = std::move(st.host_copy)]() mutable {
                    PhaseTimer pt("kl_host_copy");
                    p.reset();
                    pt.mark("freed");
                });
            } catch (const std::system_error&) {
                // no thread to spare: the copy was freed here, with the lambda
            }
        }
    }
    r.t_kl_graph_wait = since(t);
    t = clk::now();
    int64_t n0 = int64_t(order0.size()), n1 = int64_t(order1.size());
    if (dev_split) {
        chk(ek_kl_set_partition_fiedler(ctx, &r.median, &n0, &n1));
        r.t_split = since(t);  // (split and partition setup together)
    } else {
        chk(ek_kl_set_partition(ctx, order0.data(), n0, order1.data(), n1));
        r.t_kl_setup = since(t);
    }
    t = clk::now();
    const int64_t lcap = std::min(n0, n1);
    // the swap log goes straight into the caller's buffer when it holds the
    // whole run (no 32-B-per-node zeroed temporary and copy)
    dvec<ek_swap> own;
    ek_swap* log_buf = log_out;
    if (!log_out || cap < lcap) {
        own.resize(size_t(std::max<int64_t>(lcap, 1)));
        log_buf = own.data();
    }
    cold_stamp("kl_start");
    chk(ek_kl_run(ctx, o.limit, log_buf, lcap, &r.kl));
    cold_stamp("kl_done");
    r.t_kl = since(t);
    const int64_t iters = std::min<int64_t>(r.kl.iterations, lcap);
    if (log_out && log_buf != log_out && cap > 0) std::copy(log_buf, log_buf + std::min(iters, cap), log_out);
    const ek_swap* log = log_buf;
    t = clk::now();
    if (o.write_results) {  // results/<base>_KL_CutSize[_EIG]_output.txt (cKL.cpp:438-444, 315, 380)
        std::error_code ec;  // results/ (and out_dir) created as needed, like the reference's createDir
        std::filesystem::create_directories(join(o.out_dir, "results"), ec);
        const std::string path =
            join(o.out_dir, "results/" + base + (o.eig ? "_KL_CutSize_EIG_output.txt" : "_KL_CutSize_output.txt"));
        FILE* f = std::fopen(path.c_str(), "w");
        if (!f) fail(EK_EIO, "Error: Cannot open output file %s (%s)", path.c_str(), std::strerror(errno));
        // rows formatted on the host threads, written in order.  The ostream
        // default format is printf's %g; std::to_chars(general, 6) is specified
        // as that printf conversion and runs ~4x faster than snprintf (equal on
        // 20 M random floats)
        // (~0.1 us a row: 1,024 rows a thread at least)
        const int T = int(std::min<int64_t>(host_threads(), std::max<int64_t>(1, iters / 1024)));
        // one text buffer, each thread's rows in its own 48-B-per-row region
        // (kept across calls like the parse buffers: no zero-fill, no
        // first-touch faults per step)
        constexpr size_t ROW = 48;
        std::unique_lock<std::mutex> lk(text_cache().mu, std::try_to_lock);
        dvec<char> own;
        dvec<char>& text = lk.owns_lock() ? text_cache().buf : own;
        text.resize(size_t(iters + T + 1) * ROW);
        std::vector<size_t> len(static_cast<size_t>(T), 0);
        auto put_g = [](char* p, char* end, float v) {
            return std::to_chars(p, end, double(v), std::chars_format::general, 6).ptr;
        };
        run_threads(T, [&](int t) {
            const int64_t lo = iters * t / T, hi = iters * (t + 1) / T;
            char* const base = text.data() + size_t(lo + t) * ROW;
            char* p = base;
            char* const end = base + size_t(hi - lo + 1) * ROW;
            if (t == 0) {
                *p++ = '0';
                *p++ = '\t';
                p = put_g(p, end, r.kl.initial_cut);
                *p++ = '\t';
                *p++ = '0';
                *p++ = '\n';
            }
            for (int64_t i = lo; i < hi; ++i) {
                const ek_swap& sw = log[i];
                p = std::to_chars(p, end, sw.iter).ptr;
                *p++ = '\t';
                p = put_g(p, end, sw.cut);
                *p++ = '\t';
                p = put_g(p, end, sw.gain);
                *p++ = '\n';
            }
            len[size_t(t)] = size_t(p - base);
        });
        bool ok = true;
        for (int t = 0; t < T; ++t) {
            const char* base = text.data() + size_t(iters * t / T + t) * ROW;
            ok &= std::fwrite(base, 1, len[size_t(t)], f) == len[size_t(t)];
        }
        ok &= std::fclose(f) == 0;
        if (!ok) fail(EK_EIO, "short write to %s", path.c_str());
    }
    r.t_write = since(t);
    r.t_total = since(t0);
}

}  // namespace ek

extern "C" {

void ek_solve_default_opts(ek_solve_opts* o) {
    if (!o) return;
    *o = ek_solve_opts{};
    o->eig = 1;
    o->seed = 0;
    o->write_results = 1;
    o->limit = -1;
    o->out_dir = nullptr;
    o->sign_ref = nullptr;
    ek_lanczos_default_opts(&o->lanczos);
}

int ek_solve_file(ek_ctx* ctx, const char* path, const ek_solve_opts* opts, ek_swap* log_out, int64_t cap,
                  ek_solve_result* res) {
    EK_TRY
    if (!ctx || !path) ek::fail(EK_EINVAL, "ek_solve_file: null argument");
    ek_solve_opts o;
    ek_solve_default_opts(&o);
    if (opts) o = *opts;
    if (o.eig < 0 || o.eig > 2) ek::fail(EK_EINVAL, "ek_solve_file: eig must be 0, 1 or 2");
    int rank = 0, nranks = 1;
    ek::ctx_ranks(ctx, &rank, &nranks);
    ek_solve_result r{};
    const auto t0 = std::chrono::steady_clock::now();
    ek_hgr* h = nullptr;
    if (const int rc = ek_hgr_read(path, &h); rc != EK_OK) throw ek::Error{rc};
    std::unique_ptr<ek_hgr, void (*)(ek_hgr*)> hg(h, ek_hgr_free);
    r.t_read = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    ek::PhaseTimer pt("solve_file");
    ek::solve([ctx] { return ctx; }, rank, nranks, *h, std::filesystem::path(path).filename().string(), o, log_out,
              cap, r);
    pt.mark("solve returned (its locals freed)");
    hg.reset();
    pt.mark("hgr freed");
    r.t_total += r.t_read;
    if (res) *res = r;
    return EK_OK;
    EK_CATCH
}

int ek_random_split(int64_t n, uint32_t seed, int32_t* order0, int32_t* order1) {
    EK_TRY
    if (n < 0 || n > INT32_MAX || (n && (!order1 || (n >= 2 && !order0)))) ek::fail(EK_EINVAL, "ek_random_split: bad argument");
    std::vector<uint32_t> nodes(static_cast<size_t>(n));  // cKL.cpp:176-181
    for (int64_t i = 0; i < n; ++i) nodes[size_t(i)] = uint32_t(i);
    std::mt19937 gen(seed);
    std::shuffle(nodes.begin(), nodes.end(), gen);
    const size_t mid = size_t(n / 2);  // cKL.cpp:183-191
    for (size_t i = 0; i < mid; ++i) order0[i] = int32_t(nodes[i]);
    for (size_t i = mid; i < size_t(n); ++i) order1[i - mid] = int32_t(nodes[i]);
    return EK_OK;
    EK_CATCH
}

}  // extern "C"
