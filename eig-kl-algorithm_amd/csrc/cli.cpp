// Drop-in command-line tools cEIG / cKL / gKL / gKL2 (ek_cli_main).
//
// argv and outputs follow the reference executables, relative to the CWD:
//   cEIG <in.hgr>          -> pre_saved_EIG/<base>_out.txt   (cEIG.cpp:138-237)
//   cKL  <in.hgr> [-EIG]   -> results/<base>_KL_CutSize[_EIG]_output.txt
//                             (-EIG reads pre_saved_EIG/<base>_out.txt; cKL.cpp:424-468)
//   gKL  <in.hgr> [-EIG]   -> same as cKL (gKL.cu:672-713 computes the same
//                             KL on the GPU but with different, racy
//                             semantics; SURVEY §0 finding 3 — this alias
//                             keeps the cKL semantics, the parity target)
//   gKL2 <in.hgr> [-EIG]   -> -EIG computes the Fiedler split in-process on
//                             the GPU (gKL2.cu:989-1033 used a non-Fiedler
//                             power iteration; this uses the Lanczos solver)
// All of them create results/ and pre_saved_EIG/.  Every compute step runs
// on the GPU through the C-ABI; there is no CPU path.  Additive flags:
//   --device D  --seed S (random init)  --sign-ref FILE  --no-deflate
//   --ncv N  --tol T  --quiet
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <cmath>
#include <cstring>
#include <filesystem>
#include <future>
#include <random>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "ek_internal.hpp"

namespace {

struct Opts {
    std::string tool, input;
    bool eig = false, quiet = false, have_seed = false, deflate = true;
    int device = 0, ncv = 0;
    double tol = 0.0;
    uint64_t seed = 0;
    std::string sign_ref;
};

using clk = std::chrono::steady_clock;
double secs(clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); }

void mkdirs() {
    ::mkdir("results", 0755);
    ::mkdir("pre_saved_EIG", 0755);
}

std::string base_name(const std::string& p) { return std::filesystem::path(p).filename().string(); }

struct Fail {
    std::string msg;
};
void check(int rc, const char* what) {
    if (rc != EK_OK) throw Fail{std::string(what) + ": " + ek_last_error()};
}

// Context creation (HIP runtime + device init) is the slowest fixed cost of
// a short run, so it starts on a helper thread at process start and
// overlaps the .hgr parse and the clique expansions.
struct CtxInit {
    std::thread th;
    ek_ctx* ctx = nullptr;
    int rc = EK_OK;
    std::string err;
    explicit CtxInit(int device) {
        th = std::thread([this, device] {
            rc = ek_init(device, &ctx);
            if (rc != EK_OK) err = ek_last_error();
        });
    }
    ek_ctx* get() {
        if (th.joinable()) th.join();
        if (rc != EK_OK) throw Fail{"GPU init: " + err};
        return ctx;
    }
    ~CtxInit() {
        if (th.joinable()) th.join();
        if (ctx) ek_destroy(ctx);
    }
};

struct Phases {  // wall-clock phase log for the non-quiet summary
    std::vector<std::pair<std::string, double>> t;
    clk::time_point last = clk::now();
    void mark(const char* name) {
        t.emplace_back(name, secs(last));
        last = clk::now();
    }
    void print() const {
        std::printf("%-24s:", "Phases (s)");
        for (const auto& p : t) std::printf(" %s %.3f", p.first.c_str(), p.second);
        std::printf("\n");
    }
};

// Fiedler vector of the file's Laplacian on the GPU (cEIG.cpp:188-209).
void fiedler(const Opts& o, ek_hgr* h, CtxInit& ci, double& lambda, std::vector<double>& v, ek_lanczos_stats& st,
             Phases& ph) {
    int64_t nets = 0, nodes = 0;
    ek_hgr_dims(h, &nets, &nodes, nullptr);
    ek_csr* L = nullptr;
    check(ek_laplacian_build(h, &L), "Laplacian");
    int64_t nr = 0, nnz = 0;
    ek_csr_dims(L, &nr, &nnz, nullptr);
    std::vector<int32_t> rowptr(size_t(nr) + 1), col(static_cast<size_t>(nnz));
    std::vector<double> val(static_cast<size_t>(nnz));
    ek_csr_copy(L, rowptr.data(), col.data(), val.data(), nullptr);
    ek_csr_free(L);
    ph.mark("laplacian");
    ek_ctx* ctx = ci.get();
    ph.mark("gpu-init-wait");
    check(ek_spmv_setup(ctx, nodes, 0, nodes, rowptr.data(), col.data(), val.data()), "SpMV setup");
    ek_lanczos_opts lo;
    ek_lanczos_default_opts(&lo);
    lo.deflate = o.deflate ? 1 : 0;
    if (o.ncv > 0) lo.ncv = o.ncv;
    if (o.tol > 0) lo.tol = o.tol;
    v.assign(size_t(nodes), 0.0);
    const int rc = ek_lanczos_fiedler(ctx, &lo, &lambda, v.data(), &st);
    if (rc == EK_ENOCONV) throw Fail{"Eigenvalue computation failed"};
    check(rc, "Lanczos");
    if (!o.sign_ref.empty()) {
        std::vector<double> ref(static_cast<size_t>(nodes));
        double l2 = 0, m2 = 0;
        check(ek_eig_read(o.sign_ref.c_str(), nodes, &l2, &m2, nullptr, ref.data(), nullptr, nullptr, nullptr, nullptr),
              "sign reference");
        ek_align_sign(nodes, v.data(), ref.data());
    }
    ph.mark("lanczos");
}

// KL graph in cKL order, copied out of the library's handle.
struct KLGraph {
    std::vector<int32_t> rowptr, col;
    std::vector<float> w;
};
KLGraph build_kl_graph(ek_hgr* h) {
    ek_csr* G = nullptr;
    check(ek_kl_graph_build(h, &G), "KL graph");
    int64_t nr = 0, nnz = 0;
    ek_csr_dims(G, &nr, &nnz, nullptr);
    KLGraph g;
    g.rowptr.resize(size_t(nr) + 1);
    g.col.resize(static_cast<size_t>(nnz));
    g.w.resize(static_cast<size_t>(nnz));
    ek_csr_copy(G, g.rowptr.data(), g.col.data(), g.w.data(), nullptr);
    ek_csr_free(G);
    return g;
}

int run_eig(const Opts& o) {
    const auto t0 = clk::now();
    CtxInit ci(o.device);
    Phases ph;
    const std::string outfile = "pre_saved_EIG/" + base_name(o.input) + "_out.txt";
    if (!o.quiet) {
        std::printf("\n============= Initialization =============\n");
        std::printf("Device: HIP gfx950 #%d (libeigkl_hip %s)\n", o.device, ek_version());
    }
    ek_hgr* h = nullptr;
    check(ek_hgr_read(o.input.c_str(), &h), "Error opening input file");
    std::unique_ptr<ek_hgr, void (*)(ek_hgr*)> hg(h, ek_hgr_free);
    int64_t nets = 0, nodes = 0;
    ek_hgr_dims(h, &nets, &nodes, nullptr);
    if (!o.quiet) std::printf("\nProblem Size:\n  - Nets: %lld\n  - Nodes: %lld\n", (long long)nets, (long long)nodes);
    double lambda = 0;
    std::vector<double> v;
    ek_lanczos_stats st{};
    if (!o.quiet) std::printf("\nComputing eigenvalues (GPU Lanczos)...\n");
    ph.mark("read");
    fiedler(o, h, ci, lambda, v, st, ph);
    double med = 0;
    std::vector<uint8_t> bits(static_cast<size_t>(nodes));
    check(ek_median_split(nodes, v.data(), &med, bits.data()), "median");
    check(ek_eig_write(outfile.c_str(), nodes, lambda, med, bits.data(), v.data()), "write");
    ph.mark("write");
    if (!o.quiet) {
        ph.print();
        std::printf("  - lambda_1: %.12g  (restarts %d, matvecs %d, residual %.3g, %.3f s on GPU)\n", lambda,
                    st.restarts, st.matvecs, st.residual, st.total_ms / 1000.0);
        std::printf("\n============= Summary =============\n");
        std::printf("Execution time: %.3f seconds\n", secs(t0));
        std::printf("Results written to: %s\n", outfile.c_str());
        std::printf("================================\n\n");
    }
    return 0;
}

int run_kl(const Opts& o) {
    const auto t0 = clk::now();
    CtxInit ci(o.device);
    Phases ph;
    const std::string base = base_name(o.input);
    const std::string fout_name =
        "results/" + base + (o.eig ? "_KL_CutSize_EIG_output.txt" : "_KL_CutSize_output.txt");
    if (!o.quiet) std::printf("\n============= Reading Input File ==============\n");
    ek_hgr* h = nullptr;
    check(ek_hgr_read(o.input.c_str(), &h), "Error opening file");
    std::unique_ptr<ek_hgr, void (*)(ek_hgr*)> hg(h, ek_hgr_free);
    int64_t nets = 0, nodes = 0, pins = 0;
    ek_hgr_dims(h, &nets, &nodes, &pins);
    if (!o.quiet)
        std::printf("Circuit Statistics\n  - Total Nets : %lld\n  - Total Nodes: %lld\n", (long long)nets,
                    (long long)nodes);
    ph.mark("read");
    // the KL graph is built on a host thread while the GPU runs the Lanczos solve
    std::future<KLGraph> kg = std::async(std::launch::async, build_kl_graph, h);
    // initial partition (shuffleSparceMatrix, cKL.cpp:151-197)
    std::vector<int32_t> order0, order1;
    if (o.eig && o.tool == "gKL2") {
        double lambda = 0;
        std::vector<double> v;
        ek_lanczos_stats st{};
        fiedler(o, h, ci, lambda, v, st, ph);
        double med = 0;
        std::vector<uint8_t> bits(static_cast<size_t>(nodes));
        check(ek_median_split(nodes, v.data(), &med, bits.data()), "median");
        for (int64_t i = 0; i < nodes; ++i) (bits[size_t(i)] ? order1 : order0).push_back(int32_t(i));
        if (!o.quiet)
            std::printf("EIG (GPU Lanczos): lambda_1 %.12g, %d matvecs, %.3f s\n", lambda, st.matvecs,
                        st.total_ms / 1000.0);
    } else if (o.eig) {
        const std::string eig_file = "pre_saved_EIG/" + base + "_out.txt";
        order0.resize(size_t(nodes));
        order1.resize(size_t(nodes));
        int64_t n0 = 0, n1 = 0;
        if (ek_eig_read(eig_file.c_str(), nodes, nullptr, nullptr, nullptr, nullptr, order0.data(), &n0,
                        order1.data(), &n1) != EK_OK)
            throw Fail{"Error: EIG file not found"};
        order0.resize(size_t(n0));
        order1.resize(size_t(n1));
    } else {
        std::vector<int32_t> all(static_cast<size_t>(nodes));
        for (int64_t i = 0; i < nodes; ++i) all[size_t(i)] = int32_t(i);
        std::mt19937 gen(o.have_seed ? uint32_t(o.seed) : std::random_device{}());
        std::shuffle(all.begin(), all.end(), gen);
        const size_t mid = size_t(nodes / 2);
        order0.assign(all.begin(), all.begin() + std::ptrdiff_t(mid));
        order1.assign(all.begin() + std::ptrdiff_t(mid), all.end());
    }
    if (!o.quiet) std::printf("Partition sizes - Left: %zu Right: %zu\n", order0.size(), order1.size());
    // KL graph in cKL order (host thread above) -> GPU
    const KLGraph g = kg.get();
    ph.mark("kl-graph-wait");
    std::vector<int64_t> net_ptr(size_t(nets) + 1);
    std::vector<int32_t> pinv(static_cast<size_t>(pins));
    ek_hgr_copy_pins(h, net_ptr.data(), pinv.data());
    ek_ctx* ctx = ci.get();
    check(ek_kl_graph_setup(ctx, nodes, g.rowptr.data(), g.col.data(), g.w.data()), "KL setup");
    check(ek_kl_nets_setup(ctx, nets, net_ptr.data(), pinv.data()), "nets setup");
    check(ek_kl_set_partition(ctx, order0.data(), int64_t(order0.size()), order1.data(), int64_t(order1.size())),
          "partition");
    const int64_t cap = int64_t(std::min(order0.size(), order1.size()));
    std::vector<ek_swap> log(size_t(std::max<int64_t>(cap, 1)));
    ek_kl_result r{};
    if (!o.quiet) std::printf("\n\n=========== Starting KL Algorithm (GPU) =============\n");
    ph.mark("kl-setup");
    check(ek_kl_run(ctx, -1, log.data(), cap, &r), "KL");
    ph.mark("kl");
    // results file (cKL.cpp:315, 380): ostream default format == %g
    FILE* f = std::fopen(fout_name.c_str(), "w");
    if (!f) throw Fail{"Error: Cannot open output file"};
    std::fprintf(f, "0\t%g\t0\n", double(r.initial_cut));
    for (int64_t i = 0; i < r.iterations && i < cap; ++i)
        std::fprintf(f, "%u\t%g\t%g\n", log[size_t(i)].iter, double(log[size_t(i)].cut), double(log[size_t(i)].gain));
    std::fclose(f);
    if (!o.quiet) {
        std::printf("\n=============== Final Results =================\n");
        std::printf("%-24s: %lld\n", "Total iterations", (long long)r.iterations);
        std::printf("%-24s: %.2f\n", "Initial cut size", double(r.initial_cut));
        std::printf("%-24s: %.2f\n", "Best cut size achieved", double(r.best_cut));
        std::printf("%-24s: %.2f%%\n", "Overall improvement", 100.0 * (1.0 - double(r.best_cut) / double(r.initial_cut)));
        std::printf("%-24s: %lld (iteration %lld)\n", "Net cut @ best prefix", (long long)r.net_cut_best,
                    (long long)r.best_iter);
        std::printf("%-24s: %.3f ms (device)\n", "KL loop", r.loop_ms);
        std::printf("%-24s: %.3f seconds\n", "Total runtime", secs(t0));
        ph.print();
    }
    return 0;
}

}  // namespace

extern "C" int ek_cli_main(const char* tool_c, int argc, char** argv) {
    Opts o;
    o.tool = tool_c ? tool_c : "cKL";
    std::vector<std::string> pos;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto need = [&](const char* flag) -> std::string {
            if (i + 1 >= argc) throw Fail{std::string("missing value for ") + flag};
            return argv[++i];
        };
        try {
            if (a == "--device") o.device = std::stoi(need("--device"));
            else if (a == "--seed") {
                o.seed = std::stoull(need("--seed"));
                o.have_seed = true;
            } else if (a == "--sign-ref") o.sign_ref = need("--sign-ref");
            else if (a == "--no-deflate") o.deflate = false;
            else if (a == "--ncv") o.ncv = std::stoi(need("--ncv"));
            else if (a == "--tol") o.tol = std::stod(need("--tol"));
            else if (a == "--quiet") o.quiet = true;
            else pos.push_back(a);
        } catch (const Fail& e) {
            std::fprintf(stderr, "Error: %s\n", e.msg.c_str());
            return 1;
        } catch (...) {
            std::fprintf(stderr, "Error: bad value for %s\n", a.c_str());
            return 1;
        }
    }
    try {
        if (o.tool == "cEIG") {
            mkdirs();  // cEIG.cpp:148-149
            if (pos.size() != 1) throw Fail{"Usage: ./EIG <input_file>"};
            o.input = pos[0];
            return run_eig(o);
        }
        mkdirs();  // cKL.cpp:428-429
        if (pos.empty() || pos.size() > 2) {
            std::printf("Usage: %s <input_file> [-EIG]\n", argc > 0 ? argv[0] : o.tool.c_str());
            return 1;
        }
        o.input = pos[0];
        o.eig = pos.size() == 2 && pos[1] == "-EIG";
        return run_kl(o);
    } catch (const Fail& e) {
        std::fprintf(stderr, "Error: %s\n", e.msg.c_str());
        return 1;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "Error occurred: %s\n", e.what());
        return 1;
    }
}
