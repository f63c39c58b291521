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
//   --spectra            the Lanczos of the reference's Spectra SymEigsSolver
//                        (cEIG.cpp:195-198): a full reorthogonalisation every
//                        step, restarts keeping Spectra's nev_adjusted, fp64
//                        basis reads (ek_lanczos_opts reorth 1, keep_min 0,
//                        basis32 0); default: partial reorthogonalisation, the
//                        ncv/5 restart floor and the fp32 basis shadow
//   --reorth full|partial  only the reorthogonalisation rule
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <mutex>
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
    bool eig = false, quiet = false, have_seed = false, deflate = true, teardown = true;
    int device = 0, ncv = 0;
    bool spectra = false;
    int reorth = 0;  // 0: default (partial)
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
    bool teardown = true;  // false: the context is left to the process exit (EK_CLI_NO_TEARDOWN)
    explicit CtxInit(int device, bool td = true) : teardown(td) {
        th = std::thread([this, device] {
            ek::cold_stamp("ctx_init_start");
            rc = ek_init(device, &ctx);
            ek::cold_stamp("ctx_init_done");
            if (rc != EK_OK) err = ek_last_error();
        });
    }
    std::once_flag joined;  // get() is called from the solve's thread and the KL adjacency's
    ek_ctx* get() {
        std::call_once(joined, [this] {
            if (th.joinable()) th.join();
        });
        if (rc != EK_OK) throw Fail{"GPU init: " + err};
        return ctx;
    }
    ~CtxInit() {
        if (th.joinable()) th.join();
        ek::cold_stamp("ctx_destroy_start");
        if (ctx && teardown) ek_destroy(ctx);
        ek::cold_stamp("ctx_destroy_done");
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

ek_solve_opts solve_opts(const Opts& o) {
    ek_solve_opts so;
    ek_solve_default_opts(&so);
    so.lanczos.deflate = o.deflate ? 1 : 0;
    if (o.ncv > 0) so.lanczos.ncv = o.ncv;
    if (o.tol > 0) so.lanczos.tol = o.tol;
    if (o.spectra) {  // Spectra SymEigsSolver's rule set
        so.lanczos.reorth = 1;
        so.lanczos.keep_min = 0;
        so.lanczos.basis32 = 0;
    }
    if (o.reorth) so.lanczos.reorth = o.reorth;
    so.sign_ref = o.sign_ref.empty() ? nullptr : o.sign_ref.c_str();
    so.seed = o.have_seed ? uint32_t(o.seed) : std::random_device{}();  // cKL.cpp:179-180 when unseeded
    return so;
}

int run_eig(const Opts& o) {
    const auto t0 = clk::now();
    CtxInit ci(o.device, o.teardown);
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
    if (!o.quiet) std::printf("\nComputing eigenvalues (GPU Lanczos)...\n");
    ph.mark("read");
    double lambda = 0, tl = 0, tz = 0;
    std::vector<double> v;
    ek_lanczos_stats st{};
    const ek_solve_opts so = solve_opts(o);
    try {
        // the context initialises on its thread while the Laplacian is built
        ek::fiedler_vector(ci.get(), 0, 1, *h, so, lambda, v, st, &tl, &tz);
    } catch (const ek::Error& e) {
        if (e.code == EK_ENOCONV) throw Fail{"Eigenvalue computation failed"};  // cEIG.cpp:200-202
        throw Fail{std::string("Lanczos: ") + ek_last_error()};
    }
    ph.mark("laplacian+lanczos");
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
    CtxInit ci(o.device, o.teardown);
    const std::string base = base_name(o.input);
    if (!o.quiet) std::printf("\n============= Reading Input File ==============\n");
    ek_hgr* h = nullptr;
    check(ek_hgr_read(o.input.c_str(), &h), "Error opening file");
    std::unique_ptr<ek_hgr, void (*)(ek_hgr*)> hg(h, ek_hgr_free);
    const double t_read = secs(t0);
    ek::cold_stamp("read_done");
    int64_t nets = 0, nodes = 0;
    ek_hgr_dims(h, &nets, &nodes, nullptr);
    if (!o.quiet)
        std::printf("Circuit Statistics\n  - Total Nets : %lld\n  - Total Nodes: %lld\n", (long long)nets,
                    (long long)nodes);
    // initial partition (shuffleSparceMatrix, cKL.cpp:151-197): gKL2 -EIG
    // computes the Fiedler split in-process, cKL/gKL -EIG read the EIG file
    ek_solve_opts so = solve_opts(o);
    so.eig = o.eig ? (o.tool == "gKL2" ? 1 : 2) : 0;
    ek_solve_result r{};
    try {
        ek::solve([&ci] { return ci.get(); }, 0, 1, *h, base, so, nullptr, 0, r);
        ek::cold_stamp("solve_done");
    } catch (const ek::Error& e) {
        if (e.code == EK_ENOCONV) throw Fail{"Eigenvalue computation failed"};
        const std::string msg = ek_last_error();
        throw Fail{msg.rfind("Error", 0) == 0 ? msg : "KL: " + msg};
    }
    if (!o.quiet) {
        if (so.eig == 1)
            std::printf("EIG (GPU Lanczos): lambda_1 %.12g, %d matvecs, %.3f s\n", r.lambda, r.lanczos.matvecs,
                        r.lanczos.total_ms / 1000.0);
        std::printf("\n=============== Final Results =================\n");
        std::printf("%-24s: %lld\n", "Total iterations", (long long)r.kl.iterations);
        std::printf("%-24s: %.2f\n", "Initial cut size", double(r.kl.initial_cut));
        std::printf("%-24s: %.2f\n", "Best cut size achieved", double(r.kl.best_cut));
        std::printf("%-24s: %.2f%%\n", "Overall improvement", 100.0 * (1.0 - double(r.kl.best_cut) / double(r.kl.initial_cut)));
        std::printf("%-24s: %lld (iteration %lld)\n", "Net cut @ best prefix", (long long)r.kl.net_cut_best,
                    (long long)r.kl.best_iter);
        std::printf("%-24s: %.3f ms (device)\n", "KL loop", r.kl.loop_ms);
        std::printf("%-24s: %.3f seconds\n", "Total runtime", secs(t0));
        std::printf("%-24s: read %.3f laplacian %.3f lanczos %.3f split %.3f kl-graph-wait %.3f kl-setup %.3f kl %.3f "
                    "write %.3f\n", "Phases (s)", t_read, r.t_laplacian, r.t_lanczos, r.t_split, r.t_kl_graph_wait,
                    r.t_kl_setup, r.t_kl, r.t_write);
    }
    return 0;
}

}  // namespace

extern "C" int ek_cli_main(const char* tool_c, int argc, char** argv) {
    return ek_cli_main_ex(tool_c, argc, argv, 0);
}

extern "C" int ek_cli_main_ex(const char* tool_c, int argc, char** argv, int flags) {
    ek::cold_stamp("main");
    Opts o;
    o.tool = tool_c ? tool_c : "cKL";
    o.teardown = !(flags & EK_CLI_NO_TEARDOWN);
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
            else if (a == "--spectra") o.spectra = true;
            else if (a == "--reorth") {
                const std::string v = need("--reorth");
                if (v == "full") o.reorth = 1;
                else if (v == "partial") o.reorth = 3;
                else throw Fail{"--reorth takes full or partial"};
            }
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
        std::fprintf(stderr, e.msg.rfind("Error", 0) == 0 ? "%s\n" : "Error: %s\n", e.msg.c_str());
        return 1;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "Error occurred: %s\n", e.what());
        return 1;
    }
}
