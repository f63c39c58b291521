// Error plumbing and host-thread sizing for libeigkl_hip.so.
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <mutex>
#include <thread>
#include <cstdlib>
#include <exception>
#include <new>
#include <stdexcept>

#include "ek_internal.hpp"

namespace ek {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

void fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    throw Error{code};
}

int guard_exceptions() {
    try {
        throw;
    } catch (const Error& e) {
        return e.code;
    } catch (const std::bad_alloc&) {
        set_error("out of host memory");
        return EK_ENOMEM;
    } catch (const std::exception& e) {
        set_error("%s", e.what());
        return EK_EINVAL;
    } catch (...) {
        set_error("unknown exception");
        return EK_EINVAL;
    }
}

static thread_local int g_thread_cap = 0;

ThreadCap::ThreadCap(int cap) : prev(g_thread_cap) { g_thread_cap = cap; }
ThreadCap::~ThreadCap() { g_thread_cap = prev; }

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

PhaseTimer::PhaseTimer(const char* t) : tag(t), t0(0.0), on(std::getenv("EK_TRACE") != nullptr) {
    if (on) t0 = now_ms();
}

void PhaseTimer::mark(const char* what) {
    if (!on) return;
    const double t = now_ms();
    std::fprintf(stderr, "[%s] %s %.3f ms\n", tag, what, t - t0);
    t0 = t;
}

// EK_COLD_TRACE=1: "[cold] <event> <epoch s>" lines on stderr (CLOCK_REALTIME,
// the clock the caller's launch time is read from), so a fresh process's
// wall can be split: library load, HIP init, context, solve phases, exit.
static const bool g_cold = std::getenv("EK_COLD_TRACE") != nullptr;
void cold_stamp(const char* what) {
    if (!g_cold) return;
    const double t = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
    std::fprintf(stderr, "[cold] %s %.6f\n", what, t);
}
namespace {
struct ColdLoad {  // runs when the dynamic loader has mapped libeigkl_hip.so and its dependencies
    ColdLoad() {
        cold_stamp("lib_loaded");
        if (g_cold) std::atexit([] { cold_stamp("atexit"); });
    }
} g_cold_load;
}  // namespace

int host_threads() {
    static const int cached = [] {
        for (const char* var : {"EK_THREADS", "OMP_NUM_THREADS"}) {
            if (const char* s = std::getenv(var)) {
                const int v = std::atoi(s);
                if (v > 0) return std::min(v, 64);
            }
        }
        const unsigned hw = std::thread::hardware_concurrency();
        return int(std::min(16u, std::max(1u, hw)));
    }();
    return g_thread_cap > 0 ? std::max(1, std::min(cached, g_thread_cap)) : cached;
}

// The host worker pool behind run_threads / parallel_for: workers are
// created once and woken per parallel region (spawning 16 threads per region
// cost ~0.3 ms, several times per solve).  Two pools, one caller each: the
// KL graph thread's regions run beside the solve's thread (its Laplacian
// build) on the second pool instead of spawning threads for every region; a
// third concurrent caller gets spawned threads.  Workers run with exceptions
// unhandled, as std::thread's.
namespace {
struct Pool {
    std::mutex run_mu;  // held by the caller of the current region
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::vector<std::thread> th;
    unsigned long long epoch = 0;
    int active = 0, pending = 0;
    void (*fn)(void*, int) = nullptr;
    void* ctx = nullptr;
    void loop(int w) {
        unsigned long long seen = 0;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return epoch != seen; });
            seen = epoch;
            if (w >= active) continue;
            auto f = fn;
            void* c = ctx;
            lk.unlock();
            f(c, w);
            lk.lock();
            if (--pending == 0) done_cv.notify_one();
        }
    }
};
}  // namespace

void pool_run(int T, void (*fn)(void*, int), void* ctx) {
    static Pool* pools = new Pool[2];  // never destroyed: workers stay blocked until the process exits
    Pool* P = &pools[0];
    std::unique_lock<std::mutex> rl(P->run_mu, std::try_to_lock);
    if (!rl.owns_lock()) {
        P = &pools[1];
        rl = std::unique_lock<std::mutex>(P->run_mu, std::try_to_lock);
    }
    if (!rl.owns_lock()) {
        std::vector<std::thread> th;
        th.reserve(size_t(T - 1));
        for (int t = 1; t < T; ++t) th.emplace_back([fn, ctx, t] { fn(ctx, t); });
        fn(ctx, 0);
        for (auto& x : th) x.join();
        return;
    }
    {
        std::lock_guard<std::mutex> lk(P->mu);
        while (int(P->th.size()) < T - 1) {
            const int w = int(P->th.size()) + 1;
            P->th.emplace_back([P, w] { P->loop(w); });
            P->th.back().detach();
        }
        P->fn = fn;
        P->ctx = ctx;
        P->active = T;
        P->pending = T - 1;
        ++P->epoch;
    }
    P->cv.notify_all();
    fn(ctx, 0);
    std::unique_lock<std::mutex> lk(P->mu);
    P->done_cv.wait(lk, [&] { return P->pending == 0; });
}

}  // namespace ek

extern "C" {
const char* ek_last_error(void) { return ek::g_last_error.c_str(); }
const char* ek_version(void) { return "eigkl-mi355x 0.1 (gfx950)"; }
int ek_abi_version(void) { return EIGKL_ABI_VERSION; }
}
