// Error plumbing and host-thread sizing for libeigkl_hip.so.
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

int host_threads() {
    static int cached = [] {
        for (const char* var : {"EK_THREADS", "OMP_NUM_THREADS"}) {
            if (const char* s = std::getenv(var)) {
                const int v = std::atoi(s);
                if (v > 0) return std::min(v, 64);
            }
        }
        const unsigned hw = std::thread::hardware_concurrency();
        return int(std::min(16u, std::max(1u, hw)));
    }();
    return cached;
}

}  // namespace ek

extern "C" {
const char* ek_last_error(void) { return ek::g_last_error.c_str(); }
const char* ek_version(void) { return "eigkl-mi355x 0.1 (gfx950)"; }
}
