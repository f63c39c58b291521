// SpMV design lab (not part of the product): times candidate layouts of the
// fused Lanczos SpMV (y = L f / |f|, vcol = f / |f|, per-block alpha partials)
// on the ibm18-shape synthetic Laplacian, checks each against a host fp64
// product, and prints the average launch time from back-to-back batches and
// from per-launch event pairs.  Build: make -C tools; run: tools/build/spmv_lab [mult] [iters]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/eigkl.h"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

constexpr int T = 256;

__device__ __forceinline__ double block4(double v, double* wsum) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
    __syncthreads();
    return (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
}

// long row (cnt > BN): one workgroup, strided
__device__ __forceinline__ void long_row(int r0, int p0, int cnt, const int* __restrict__ col,
                                        const double* __restrict__ val, const double* __restrict__ x,
                                        double* __restrict__ y, double scale, const double* __restrict__ f,
                                        double* __restrict__ vcol, double* __restrict__ apart, double* wsum) {
    double s = 0.0;
    for (int i = threadIdx.x; i < cnt; i += T) s += val[p0 + i] * x[col[p0 + i]];
    const double a = block4(s, wsum);
    if (threadIdx.x == 0) {
        y[r0] = a * scale;
        const double v = f[r0] * scale;
        vcol[r0] = v;
        apart[blockIdx.x] = v * (a * scale);
    }
}

// ---- A: the shipped layout (strided product loop)
template <int BN>
__global__ __launch_bounds__(T) void kA(const int4* __restrict__ desc, const int* __restrict__ rowptr,
                                        const int* __restrict__ col, const double* __restrict__ val,
                                        const double* __restrict__ x, double* __restrict__ y,
                                        const double* __restrict__ fn2, const double* __restrict__ f,
                                        double* __restrict__ vcol, double* __restrict__ apart) {
    __shared__ double prod[BN];
    __shared__ int rbeg[T + 1];
    __shared__ double yrow[T];
    __shared__ double wsum[T / 64];
    const int t = threadIdx.x;
    const int4 d = desc[blockIdx.x];
    const int r0 = d.x, nr = d.y, p0 = d.z, cnt = d.w;
    const double scale = *fn2 > 0.0 ? 1.0 / sqrt(*fn2) : 0.0;
    if (cnt > BN) {
        long_row(r0, p0, cnt, col, val, x, y, scale, f, vcol, apart, wsum);
        return;
    }
    for (int i = t; i <= nr; i += T) rbeg[i] = rowptr[r0 + i] - p0;
    const double fr = t < nr ? f[r0 + t] : 0.0;
    for (int i = t; i < cnt; i += T) prod[i] = val[p0 + i] * x[col[p0 + i]];
    __syncthreads();
    int L = T / (nr > 0 ? nr : 1);
    L = L >= 64 ? 64 : L >= 32 ? 32 : L >= 16 ? 16 : L >= 8 ? 8 : L >= 4 ? 4 : L >= 2 ? 2 : 1;
    const int g = t / L, lane = t % L;
    double s = 0.0;
    if (g < nr)
        for (int i = rbeg[g] + lane; i < rbeg[g + 1]; i += L) s += prod[i];
    for (int o = L >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, L);
    if (g < nr && lane == 0) {
        const double yr = s * scale;
        y[r0 + g] = yr;
        yrow[g] = yr;
    }
    __syncthreads();
    double av = 0.0;
    if (t < nr) {
        const double v = fr * scale;
        vcol[r0 + t] = v;
        av = v * yrow[t];
    }
    av = block4(av, wsum);
    if (t == 0) apart[blockIdx.x] = av;
}

// ---- B: every global load of the block issued before any use (fixed trip count)
template <int BN>
__device__ __forceinline__ void blockB(int b, const int4* __restrict__ desc, const int* __restrict__ rowptr,
                                       const int* __restrict__ col, const double* __restrict__ val,
                                       const double* __restrict__ x, double* __restrict__ y,
                                       const double* __restrict__ fn2, const double* __restrict__ f,
                                       double* __restrict__ vcol, double* __restrict__ apart, double* prod, int* rbeg,
                                       double* yrow, double* wsum) {
    constexpr int PER = BN / T;
    const int t = threadIdx.x;
    const int4 d = desc[b];
    const int r0 = d.x, nr = d.y, p0 = d.z, cnt = d.w;
    if (cnt > BN) {
        const double scale = *fn2 > 0.0 ? 1.0 / sqrt(*fn2) : 0.0;
        double s = 0.0;
        for (int i = t; i < cnt; i += T) s += val[p0 + i] * x[col[p0 + i]];
        const double a = block4(s, wsum);
        if (t == 0) {
            y[r0] = a * scale;
            const double v = f[r0] * scale;
            vcol[r0] = v;
            apart[b] = v * (a * scale);
        }
        return;
    }
    int ci[PER];
    double vv[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int i = t + u * T;
        ci[u] = i < cnt ? col[p0 + i] : -1;
        vv[u] = i < cnt ? val[p0 + i] : 0.0;
    }
    const int rb0 = t <= nr ? rowptr[r0 + t] - p0 : 0;
    const int rb1 = (t == 0 && nr == T) ? rowptr[r0 + T] - p0 : 0;
    const double fr = t < nr ? f[r0 + t] : 0.0;
    const double n2 = *fn2;
    double xv[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) xv[u] = ci[u] >= 0 ? x[ci[u]] : 0.0;
    if (t <= nr) rbeg[t] = rb0;
    if (t == 0 && nr == T) rbeg[T] = rb1;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int i = t + u * T;
        if (i < cnt) prod[i] = vv[u] * xv[u];
    }
    const double scale = n2 > 0.0 ? 1.0 / sqrt(n2) : 0.0;
    __syncthreads();
    int L = T / (nr > 0 ? nr : 1);
    L = L >= 64 ? 64 : L >= 32 ? 32 : L >= 16 ? 16 : L >= 8 ? 8 : L >= 4 ? 4 : L >= 2 ? 2 : 1;
    const int g = t / L, lane = t % L;
    double s = 0.0;
    if (g < nr)
        for (int i = rbeg[g] + lane; i < rbeg[g + 1]; i += L) s += prod[i];
    for (int o = L >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, L);
    if (g < nr && lane == 0) {
        const double yr = s * scale;
        y[r0 + g] = yr;
        yrow[g] = yr;
    }
    __syncthreads();
    double av = 0.0;
    if (t < nr) {
        const double v = fr * scale;
        vcol[r0 + t] = v;
        av = v * yrow[t];
    }
    av = block4(av, wsum);
    if (t == 0) apart[b] = av;
}

template <int BN>
__global__ __launch_bounds__(T) void kB(const int4* __restrict__ desc, const int* __restrict__ rowptr,
                                        const int* __restrict__ col, const double* __restrict__ val,
                                        const double* __restrict__ x, double* __restrict__ y,
                                        const double* __restrict__ fn2, const double* __restrict__ f,
                                        double* __restrict__ vcol, double* __restrict__ apart) {
    __shared__ double prod[BN];
    __shared__ int rbeg[T + 1];
    __shared__ double yrow[T];
    __shared__ double wsum[T / 64];
    blockB<BN>(blockIdx.x, desc, rowptr, col, val, x, y, fn2, f, vcol, apart, prod, rbeg, yrow, wsum);
}

// ---- P: persistent grid, each workgroup walks row blocks b, b + grid, ...
template <int BN>
__global__ __launch_bounds__(T) void kP(int nb, const int4* __restrict__ desc, const int* __restrict__ rowptr,
                                        const int* __restrict__ col, const double* __restrict__ val,
                                        const double* __restrict__ x, double* __restrict__ y,
                                        const double* __restrict__ fn2, const double* __restrict__ f,
                                        double* __restrict__ vcol, double* __restrict__ apart) {
    __shared__ double prod[BN];
    __shared__ int rbeg[T + 1];
    __shared__ double yrow[T];
    __shared__ double wsum[T / 64];
    for (int b = blockIdx.x; b < nb; b += gridDim.x) {
        blockB<BN>(b, desc, rowptr, col, val, x, y, fn2, f, vcol, apart, prod, rbeg, yrow, wsum);
        __syncthreads();
    }
}

// ---- C: vector CSR, G lanes per row, no LDS staging; one partial per block of T/G rows
template <int G>
__global__ __launch_bounds__(T) void kC(int nrows, const int* __restrict__ rowptr, const int* __restrict__ col,
                                        const double* __restrict__ val, const double* __restrict__ x,
                                        double* __restrict__ y, const double* __restrict__ fn2,
                                        const double* __restrict__ f, double* __restrict__ vcol,
                                        double* __restrict__ apart) {
    __shared__ double wsum[T / 64];
    const int t = threadIdx.x;
    const int r = blockIdx.x * (T / G) + t / G, lane = t % G;
    double s = 0.0, v = 0.0;
    const double n2 = *fn2;
    if (r < nrows) {
        const int b = rowptr[r], e = rowptr[r + 1];
        if (lane == 0) v = f[r];
        for (int i = b + lane; i < e; i += G) s += val[i] * x[col[i]];
    }
    for (int o = G >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, G);
    const double scale = n2 > 0.0 ? 1.0 / sqrt(n2) : 0.0;
    double av = 0.0;
    if (r < nrows && lane == 0) {
        const double yr = s * scale;
        y[r] = yr;
        v *= scale;
        vcol[r] = v;
        av = v * yr;
    }
    av = block4(av, wsum);
    if (t == 0) apart[blockIdx.x] = av;
}

static std::vector<int> row_blocks(const std::vector<int>& rp, int64_t n, int bn) {
    std::vector<int> starts{0};
    int64_t rin = 0, nin = 0;
    for (int64_t r = 0; r < n; ++r) {
        const int64_t len = rp[r + 1] - rp[r];
        if (rin > 0 && (nin + len > bn || rin == T)) {
            starts.push_back(int(r));
            rin = nin = 0;
        }
        ++rin;
        nin += len;
        if (len > bn) {
            starts.push_back(int(r + 1));
            rin = nin = 0;
        }
    }
    if (starts.back() != int(n)) starts.push_back(int(n));
    std::vector<int> d;
    for (size_t b = 0; b + 1 < starts.size(); ++b) {
        const int a = starts[b], e = starts[b + 1];
        d.insert(d.end(), {a, e - a, rp[a], rp[e] - rp[a]});
    }
    return d;
}

int main(int argc, char** argv) {
    const double mult = argc > 1 ? std::atof(argv[1]) : 1.0;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 200;
    ek_hgr* h = nullptr;
    ek_csr* L = nullptr;
    if (ek_hgr_generate(mult, 1, &h) || ek_laplacian_build(h, &L)) {
        std::fprintf(stderr, "%s\n", ek_last_error());
        return 1;
    }
    int64_t n = 0, nnz = 0;
    int32_t vb = 0;
    ek_csr_dims(L, &n, &nnz, &vb);
    std::vector<int> rp(size_t(n) + 1), cl(static_cast<size_t>(nnz));
    std::vector<double> vl(static_cast<size_t>(nnz));
    ek_csr_copy(L, rp.data(), cl.data(), vl.data(), nullptr);
    std::vector<double> fh(static_cast<size_t>(n));
    uint64_t st = 7;
    for (auto& v : fh) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        v = double(st >> 11) / 9007199254740992.0 - 0.5;
    }
    double f2 = 0.0;
    for (double v : fh) f2 += v * v;
    const double sc = 1.0 / std::sqrt(f2);
    std::vector<double> yref(static_cast<size_t>(n));
    for (int64_t r = 0; r < n; ++r) {
        double s = 0.0;
        for (int p = rp[r]; p < rp[r + 1]; ++p) s += vl[p] * fh[cl[p]];
        yref[r] = s * sc;
    }
    int *d_rp, *d_cl;
    double *d_vl, *d_f, *d_y, *d_vc, *d_ap, *d_fn2;
    CK(hipMalloc(&d_rp, rp.size() * 4));
    CK(hipMalloc(&d_cl, cl.size() * 4));
    CK(hipMalloc(&d_vl, vl.size() * 8));
    CK(hipMalloc(&d_f, fh.size() * 8));
    CK(hipMalloc(&d_y, fh.size() * 8));
    CK(hipMalloc(&d_vc, fh.size() * 8));
    CK(hipMalloc(&d_ap, (size_t(n) + 1024) * 8));
    CK(hipMalloc(&d_fn2, 8));
    CK(hipMemcpy(d_rp, rp.data(), rp.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_cl, cl.data(), cl.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_vl, vl.data(), vl.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_f, fh.data(), fh.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_fn2, &f2, 8, hipMemcpyHostToDevice));
    const int bns[3] = {512, 1024, 2048};
    int* d_desc[3];
    int nb[3];
    for (int k = 0; k < 3; ++k) {
        const auto d = row_blocks(rp, n, bns[k]);
        nb[k] = int(d.size() / 4);
        CK(hipMalloc(&d_desc[k], d.size() * 4));
        CK(hipMemcpy(d_desc[k], d.data(), d.size() * 4, hipMemcpyHostToDevice));
    }
    const double bytes = 12.0 * double(nnz) + 4.0 * double(n + 1) + 16.0 * double(n);
    const double fused = bytes + 16.0 * double(n);
    std::printf("n=%lld nnz=%lld blocks(512/1024/2048)=%d/%d/%d bytes=%.0f fused=%.0f\n", (long long)n,
                (long long)nnz, nb[0], nb[1], nb[2], bytes, fused);

    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        CK(hipMemsetAsync(d_y, 0, size_t(n) * 8, s));
        for (int i = 0; i < 20; ++i) launch();
        CK(hipStreamSynchronize(s));
        std::vector<double> yh(static_cast<size_t>(n));
        CK(hipMemcpy(yh.data(), d_y, size_t(n) * 8, hipMemcpyDeviceToHost));
        double err = 0.0, ymax = 0.0;
        for (int64_t r = 0; r < n; ++r) {
            err = std::fmax(err, std::fabs(yh[r] - yref[r]));
            ymax = std::fmax(ymax, std::fabs(yref[r]));
        }
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < iters; ++i) launch();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us_batch = 1e3 * ms / iters;
        double us_pair = 0.0;
        for (int i = 0; i < 50; ++i) {
            CK(hipEventRecord(e0, s));
            launch();
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            us_pair += 1e3 * ms / 50;
        }
        std::printf("%-10s batch %7.2f us (%6.0f GB/s fused)  pair %7.2f us  maxerr %.2e rel\n", name, us_batch,
                    fused / us_batch * 1e-3, us_pair, err / ymax);
        std::fflush(stdout);
    };
#define LAUNCH_DESC(K, BN, k)                                                                                    \
    [&] {                                                                                                      \
        hipLaunchKernelGGL(K<BN>, dim3(nb[k]), dim3(T), 0, s, (const int4*)d_desc[k], d_rp, d_cl, d_vl, d_f, d_y, \
                           d_fn2, d_f, d_vc, d_ap);                                                            \
    }
#define LAUNCH_VEC(G)                                                                                          \
    [&] {                                                                                                      \
        hipLaunchKernelGGL(kC<G>, dim3((n + T / G - 1) / (T / G)), dim3(T), 0, s, int(n), d_rp, d_cl, d_vl, d_f, \
                           d_y, d_fn2, d_f, d_vc, d_ap);                                                       \
    }
    run("A1024", LAUNCH_DESC(kA, 1024, 1));
    run("A2048", LAUNCH_DESC(kA, 2048, 2));
    run("B512", LAUNCH_DESC(kB, 512, 0));
    run("B1024", LAUNCH_DESC(kB, 1024, 1));
    run("B2048", LAUNCH_DESC(kB, 2048, 2));
    for (int g : {256, 512, 1024}) {
        char nm[16];
        std::snprintf(nm, sizeof nm, "P512x%d", g);
        run(nm, [&] {
            hipLaunchKernelGGL(kP<512>, dim3(g), dim3(T), 0, s, nb[0], (const int4*)d_desc[0], d_rp, d_cl, d_vl, d_f,
                               d_y, d_fn2, d_f, d_vc, d_ap);
        });
        std::snprintf(nm, sizeof nm, "P1024x%d", g);
        run(nm, [&] {
            hipLaunchKernelGGL(kP<1024>, dim3(g), dim3(T), 0, s, nb[1], (const int4*)d_desc[1], d_rp, d_cl, d_vl, d_f,
                               d_y, d_fn2, d_f, d_vc, d_ap);
        });
    }
    run("C4", LAUNCH_VEC(4));
    run("C8", LAUNCH_VEC(8));
    run("C16", LAUNCH_VEC(16));
    // launch floor: grids doing no row work
    for (int g : {256, 1286, 2583}) {
        char nm[16];
        std::snprintf(nm, sizeof nm, "floor%d", g);
        run(nm, [&] {
            hipLaunchKernelGGL(kC<8>, dim3(g), dim3(T), 0, s, 0, d_rp, d_cl, d_vl, d_f, d_y, d_fn2, d_f, d_vc, d_ap);
        });
    }
    ek_csr_free(L);
    ek_hgr_free(h);
    return 0;
}
