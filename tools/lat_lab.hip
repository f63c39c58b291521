// Load-latency lab (not part of the product): the dependent round trip one
// wave pays for random 128-B rows of a buffer of a given size, the shape of
// the KL swap loop's per-swap segment fetch (one workgroup, one CU).  Each
// lane chases its own random cycle through the rows (row r holds the next row
// index); a step waits for all active lanes.  The buffer is streamed once
// before timing (MALL-warm where it fits).  Timing: s_memrealtime (100 MHz)
// around the chase inside the kernel, so launch overhead is excluded.
// Build: make -C tools; run: tools/build/lat_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

constexpr int ROW_INTS = 32;  // 128-B rows

__global__ __launch_bounds__(64) void chase(const int* __restrict__ buf, int rows, int steps, int lanes, int start,
                                            unsigned long long* __restrict__ out) {
    // pass 0: first visit of each row (MALL-warm, L2-cold); pass 1: the same
    // rows again (L2-warm while lanes x steps x 128 B fits the XCD's L2)
    const int lane = threadIdx.x;
    int acc = 0;
    for (int pass = 0; pass < 2; ++pass) {
        int r = int((start + size_t(lane) * 7919) % size_t(rows));
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (int s = 0; s < steps; ++s) {
            if (lane < lanes) r = buf[size_t(r) * ROW_INTS];
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) out[pass] = t1 - t0;
        acc ^= r;
    }
    if (acc == -1) out[2] = 1;
}

__global__ void touch(const int4* __restrict__ p, size_t n, int* sink) {
    int4 a = make_int4(0, 0, 0, 0);
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
        const int4 v = p[i];
        a.x ^= v.x;
    }
    if (a.x == 0x7fffffff) *sink = a.x;
}

int main() {
    const size_t sizes_mb[] = {1, 3, 8, 32, 96, 192, 320, 640};
    const int steps = 400;  // x 64 lanes x 128 B = 3.2 MB: the revisit fits one L2
    unsigned long long* out;
    int* sink;
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&sink, 64));
    std::mt19937 rng(12345);
    for (size_t mb : sizes_mb) {
        const size_t rows = mb * 1024 * 1024 / 128;
        // one random cycle over all rows (Sattolo)
        std::vector<int> nxt(rows);
        std::iota(nxt.begin(), nxt.end(), 0);
        for (size_t i = rows - 1; i > 0; --i) {
            const size_t j = rng() % i;
            std::swap(nxt[i], nxt[j]);
        }
        std::vector<int> h(rows * ROW_INTS, 0);
        for (size_t i = 0; i < rows; ++i) h[i * ROW_INTS] = nxt[i];
        int* buf;
        CK(hipMalloc(&buf, h.size() * 4));
        CK(hipMemcpy(buf, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        for (int lanes : {1, 16, 64}) {
            double best = 1e30, best2 = 1e30;
            for (int rep = 0; rep < 3; ++rep) {
                hipLaunchKernelGGL(touch, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const int4*>(buf), h.size() / 4,
                                   sink);
                hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, buf, int(rows), steps, lanes, int((rep * 104729) % rows), out);
                unsigned long long t[2] = {0, 0};
                CK(hipMemcpy(t, out, 16, hipMemcpyDeviceToHost));
                best = std::min(best, double(t[0]) * 10.0 / steps);
                best2 = std::min(best2, double(t[1]) * 10.0 / steps);
            }
            std::printf("buffer %4zu MB  lanes %2d  first visit %7.1f ns  revisit %7.1f ns per dependent step\n", mb,
                        lanes, best, best2);
        }
        CK(hipFree(buf));
    }
    return 0;
}
