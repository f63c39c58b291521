// Gather-ceiling lab (not part of the product): how fast can 13.1 M random
// 8-byte gathers from a 16 MB fp64 vector run on gfx950 — the x reads of the
// 10x synthetic's SpMV (kernels_panel.hip) — with nothing else in the kernel?
//   A  panel order: a persistent grid of G workgroups, each walking its own
//      entries panel by panel (2^17 columns = 1 MB of x per panel, every
//      workgroup in the same panel order), a 4-byte column word streamed per
//      entry, the gathered values summed in registers (no LDS, no barrier);
//   B  the same with the column words in random order over the whole x;
//   C  A plus the panel kernel's per-chunk LDS staging and barrier.
// Each form: average of 20 launches (hipEvents), after 3 warm-up launches.
// Build: make -C tools; run: tools/build/gather_lab [G]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

constexpr int PT = 256, PER = 4;

// start[w * (P + 1) + p]: workgroup w's entries in panel p are [start[..p], start[..p+1])
template <bool STAGE>
__global__ __launch_bounds__(PT) void k_gather(const unsigned* __restrict__ word, const long long* __restrict__ start,
                                               int P, const double* __restrict__ x, double* __restrict__ out) {
    __shared__ double st[PT * PER];
    const int w = blockIdx.x, t = threadIdx.x;
    double acc = 0.0;
    for (int p = 0; p < P; ++p) {
        const long long a = start[size_t(w) * (P + 1) + p], b = start[size_t(w) * (P + 1) + p + 1];
        for (long long c = a; c < b; c += PT * PER) {
            unsigned wd[PER];
            double v[PER];
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const long long i = c + t + u * PT;
                wd[u] = i < b ? word[i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < PER; ++u) v[u] = x[wd[u]];
            if constexpr (STAGE) {
#pragma unroll
                for (int u = 0; u < PER; ++u) st[t + u * PT] = v[u];
                __syncthreads();
                acc += st[(t * 7) % (PT * PER)];
                __syncthreads();
            } else {
#pragma unroll
                for (int u = 0; u < PER; ++u) acc += v[u];
            }
        }
    }
    out[size_t(w) * PT + t] = acc;
}

int main(int argc, char** argv) {
    const int G = argc > 1 ? std::atoi(argv[1]) : 1024;
    const long long n = 2019200, nnz = 13100000;
    const int pb = 17, P = int((n + (1 << pb) - 1) >> pb);
    std::mt19937_64 rng(7);
    std::vector<unsigned> cols(static_cast<size_t>(nnz));
    for (auto& c : cols) c = unsigned(rng() % uint64_t(n));
    // per workgroup an equal share, bucketed by panel (counting sort), random order inside a bucket
    const long long per = (nnz + G - 1) / G;
    std::vector<unsigned> wA(static_cast<size_t>(nnz)), wB(static_cast<size_t>(nnz));
    std::vector<long long> stA(size_t(G) * (P + 1)), stB(size_t(G) * 2);
    for (int w = 0; w < G; ++w) {
        const long long e0 = std::min(nnz, w * per), e1 = std::min(nnz, (w + 1) * per);
        std::vector<long long> cnt(size_t(P) + 1, 0);
        for (long long e = e0; e < e1; ++e) ++cnt[size_t(cols[size_t(e)] >> pb) + 1];
        for (int p = 0; p < P; ++p) cnt[size_t(p) + 1] += cnt[size_t(p)];
        for (int p = 0; p <= P; ++p) {
            stA[size_t(w) * (P + 1) + p] = e0 + cnt[size_t(p)];
            if (p < 2) stB[size_t(w) * 2 + p] = p == 0 ? e0 : e1;  // B: one "panel" holding everything (stride 2)
        }
        std::vector<long long> cur(cnt.begin(), cnt.end() - 1);
        for (long long e = e0; e < e1; ++e) wA[size_t(e0 + cur[size_t(cols[size_t(e)] >> pb)]++)] = cols[size_t(e)];
        for (long long e = e0; e < e1; ++e) wB[size_t(e)] = cols[size_t(e)];
    }
    std::vector<double> xh(static_cast<size_t>(n));
    for (auto& v : xh) v = double(rng() % 1000) / 997.0;
    unsigned *dA, *dB;
    long long *sA, *sB;
    double *dx, *dout;
    CK(hipMalloc(&dA, size_t(nnz) * 4));
    CK(hipMalloc(&dB, size_t(nnz) * 4));
    CK(hipMalloc(&sA, stA.size() * 8));
    CK(hipMalloc(&sB, stB.size() * 8));
    CK(hipMalloc(&dx, size_t(n) * 8));
    CK(hipMalloc(&dout, size_t(G) * PT * 8));
    CK(hipMemcpy(dA, wA.data(), size_t(nnz) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, wB.data(), size_t(nnz) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(sA, stA.data(), stA.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(sB, stB.data(), stB.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dx, xh.data(), size_t(n) * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipEventRecord(e0));
        for (int i = 0; i < 20; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / 20;
        std::printf("%-42s G=%5d  %8.2f us  %.1f G gathers/s  (%.3f of 8 TB/s at 12 B/entry)\n", name, G, us,
                    double(nnz) / us / 1e3, 12.0 * double(nnz) / us / 1e3 / 8000.0);
    };
    run("A panel order, registers", [&] { hipLaunchKernelGGL(k_gather<false>, dim3(G), dim3(PT), 0, 0, dA, sA, P, dx, dout); });
    run("B random over all of x, registers", [&] { hipLaunchKernelGGL(k_gather<false>, dim3(G), dim3(PT), 0, 0, dB, sB, 1, dx, dout); });
    run("C panel order + LDS stage + 2 barriers", [&] { hipLaunchKernelGGL(k_gather<true>, dim3(G), dim3(PT), 0, 0, dA, sA, P, dx, dout); });
    CK(hipGetLastError());
    return 0;
}
