// Error plumbing and host-thread sizing for libeigkl_hip.so.
#include <chrono>
#include <cstdarg>
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

}  // namespace ek

extern "C" {
const char* ek_last_error(void) { return ek::g_last_error.c_str(); }
const char* ek_version(void) { return "eigkl-mi355x 0.1 (gfx950)"; }
}
