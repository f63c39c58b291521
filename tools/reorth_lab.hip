// Reorthogonalisation design lab (not part of the product): kernel durations
// of the Lanczos projection (gemv-T) and update passes over the basis V at
// the ibm18 shape (n = 201,920, ldv = 202,752) for several basis widths J,
// against plain streaming reads of the same bytes, and update variants
// (block size, pre-reduced coefficients).  V stays resident in the MALL
// between launches, as inside the solve.  Timing: kernel start/end
// timestamps of hipExtLaunchKernelGGL (what rocprofv3 reports).
// Build: make -C tools; run: tools/build/reorth_lab
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../eig-kl-algorithm_amd/csrc/kernels_lanczos.hip"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

using namespace ek::dev;

// update with T threads per block, one double2 per thread, coefficients h
// given (zero-padded in LDS), two batches of UB columns in flight
template <int T, int UB>
__global__ __launch_bounds__(T) void upd_var(int ldv, const double* __restrict__ V, int ncols,
                                             const double* __restrict__ h, const double* __restrict__ src,
                                             double* __restrict__ dst) {
    __shared__ double hc[MAX_NCV + 2 * UB];
    const int jmax = ncols - 1;
    const size_t r = (size_t(blockIdx.x) * T + threadIdx.x) * 2;
    for (int j = threadIdx.x; j < ncols + 2 * UB; j += T) hc[j] = j < ncols ? h[j] : 0.0;
    auto load_batch = [&](double2* vb, int j0) {
#pragma unroll
        for (int u = 0; u < UB; ++u) vb[u] = *reinterpret_cast<const double2*>(V + size_t(min(j0 + u, jmax)) * ldv + r);
    };
    double2 ba[UB], bb[UB];
    double2 x = *reinterpret_cast<const double2*>(src + r);
    load_batch(ba, 0);
    __syncthreads();
    auto consume = [&](const double2* vb, int j0) {
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            const double hj = hc[j0 + u];
            x.x -= vb[u].x * hj;
            x.y -= vb[u].y * hj;
        }
    };
    for (int j0 = 0; j0 < ncols; j0 += 2 * UB) {
        load_batch(bb, j0 + UB);
        __builtin_amdgcn_sched_barrier(0);
        consume(ba, j0);
        __builtin_amdgcn_sched_barrier(0);
        load_batch(ba, j0 + 2 * UB);
        __builtin_amdgcn_sched_barrier(0);
        consume(bb, j0 + UB);
        __builtin_amdgcn_sched_barrier(0);
    }
    *reinterpret_cast<double2*>(dst + r) = x;
}

// streaming read of V[:, :ncols] (+ src), T threads x one double2 per thread
// per block, all columns; one double per block out (keeps the loads live)
template <int T, int UB>
__global__ __launch_bounds__(T) void read_rows(int ldv, const double* __restrict__ V, int ncols,
                                               const double* __restrict__ src, double* __restrict__ out) {
    const int jmax = ncols - 1;
    const size_t r = (size_t(blockIdx.x) * T + threadIdx.x) * 2;
    double2 x = *reinterpret_cast<const double2*>(src + r);
    for (int j0 = 0; j0 < ncols; j0 += UB) {
        double2 vb[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) vb[u] = *reinterpret_cast<const double2*>(V + size_t(min(j0 + u, jmax)) * ldv + r);
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            x.x += vb[u].x;
            x.y += vb[u].y;
        }
    }
    if (x.x == 12345.0) out[blockIdx.x] = x.y;
}

// streaming read of the fp32 shadow V32[:, :ncols] (+ src), one float2 per thread per column
template <int T, int UB>
__global__ __launch_bounds__(T) void read_rows32(int ldv, const float* __restrict__ V, int ncols,
                                                 const double* __restrict__ src, double* __restrict__ out) {
    const int jmax = ncols - 1;
    const size_t r = (size_t(blockIdx.x) * T + threadIdx.x) * 2;
    double2 x = *reinterpret_cast<const double2*>(src + r);
    for (int j0 = 0; j0 < ncols; j0 += UB) {
        float2 vb[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) vb[u] = *reinterpret_cast<const float2*>(V + size_t(min(j0 + u, jmax)) * ldv + r);
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            x.x += vb[u].x;
            x.y += vb[u].y;
        }
    }
    if (x.x == 12345.0) out[blockIdx.x] = x.y;
}

// the same bytes as 2-D tiles (1024 rows x 8 columns per 256-thread block)
__global__ __launch_bounds__(256) void read_tiles(int ldv, int nrb, const double* __restrict__ V, int ncols,
                                                  double* __restrict__ out) {
    const int ncg = (ncols + 7) / 8, rbk = blockIdx.x / ncg, j0 = (blockIdx.x % ncg) * 8, jmax = ncols - 1;
    double2 acc = make_double2(0.0, 0.0);
    double2 vs[2][8];
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
            vs[k][jj] = *reinterpret_cast<const double2*>(V + size_t(min(j0 + jj, jmax)) * ldv + size_t(rbk) * 1024 +
                                                          k * 512 + 2 * threadIdx.x);
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            acc.x += vs[k][jj].x;
            acc.y += vs[k][jj].y;
        }
    if (acc.x == 12345.0) out[blockIdx.x] = acc.y;
}

int main(int argc, char** argv) {
    const int n = 201920, ldv = 202752, NC = 101, nrb = ldv / GT_ROWS;
    const int iters = argc > 1 ? std::atoi(argv[1]) : 40;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::vector<double> hV(size_t(ldv) * NC, 0.0), hw(ldv, 0.0);
    uint64_t st = 88172645463325252ull;
    auto rnd = [&] {
        st ^= st << 13;
        st ^= st >> 7;
        st ^= st << 17;
        return double(st >> 11) / double(1ull << 53) - 0.5;
    };
    for (int j = 0; j < NC; ++j)
        for (int i = 0; i < n; ++i) hV[size_t(j) * ldv + i] = rnd() * 0.01;
    for (int i = 0; i < n; ++i) hw[i] = rnd();
    double *V, *w, *f1, *f2, *part, *h, *npart, *out, *psm, *hsm;
    float* V32;
    unsigned* fb;
    CK(hipMalloc(&V, hV.size() * 8));
    CK(hipMalloc(&V32, hV.size() * 4));
    CK(hipMalloc(&fb, 64));
    unsigned* gctr;
    CK(hipMalloc(&gctr, size_t(GT_HANDOFF_UINTS) * 4));
    CK(hipMemset(gctr, 0, size_t(GT_HANDOFF_UINTS) * 4));
    CK(hipMalloc(&psm, size_t(NC + 3) * nrb * 8));
    CK(hipMalloc(&hsm, size_t(NC + 3) * 8));
    {
        std::vector<float> h32(hV.size());
        for (size_t i = 0; i < hV.size(); ++i) h32[i] = float(hV[i]);
        CK(hipMemcpy(V32, h32.data(), h32.size() * 4, hipMemcpyHostToDevice));
    }
    CK(hipMalloc(&w, size_t(ldv) * 8));
    CK(hipMalloc(&f1, size_t(ldv) * 8));
    CK(hipMalloc(&f2, size_t(ldv) * 8));
    CK(hipMalloc(&part, size_t(NC + 2) * nrb * 8));
    CK(hipMalloc(&h, size_t(NC + 2) * 8));
    CK(hipMalloc(&npart, size_t(ldv / UPD_ROWS) * 8));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemcpy(V, hV.data(), hV.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(w, hw.data(), size_t(ldv) * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        for (int i = 0; i < 3; ++i) launch(nullptr, nullptr);
        double tot = 0.0;
        for (int i = 0; i < iters; ++i) {
            launch(e0, e1);
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        return 1e3 * tot / iters;
    };
    const double u0val = 1.0 / std::sqrt(double(n));
    for (int J : {20, 55, 100}) {
        const double vbytes = double(J) * n * 8;
        auto rep = [&](const char* name, double us, double bytes) {
            std::printf("J=%3d %-34s %8.2f us  %7.1f GB/s\n", J, name, us, bytes / us / 1e3);
        };
        rep("gemvt (prod, 1024x8 tiles)", timeit([&](hipEvent_t a, hipEvent_t b) {
                hipExtLaunchKernelGGL((k_gemvt<false, false>), dim3(nrb * ((J + 1 + GT_COLS - 1) / GT_COLS)), dim3(256), 0, s, a,
                                      b, 0, ldv, nrb, V, J, 1, u0val, n, w, part, nullptr, nullptr, nullptr, nullptr,
                                      nullptr, nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr,
                                      ek::dev::ProLaunch{});
            }),
            vbytes + 8.0 * n);
        rep("gemvt + column-sum hand-off", timeit([&](hipEvent_t a, hipEvent_t b) {
                hipExtLaunchKernelGGL((k_gemvt<false, false>), dim3(nrb * ((J + 1 + GT_COLS - 1) / GT_COLS)), dim3(256), 0, s, a,
                                      b, 0, ldv, nrb, V, J, 1, u0val, n, w, part, nullptr, nullptr, nullptr, nullptr,
                                      nullptr, nullptr, 1, nullptr, nullptr, 0, nullptr, gctr, h, nullptr, nullptr,
                                      ek::dev::ProLaunch{});
            }),
            vbytes + 8.0 * n);
        rep("update<true> (prod, RED)", timeit([&](hipEvent_t a, hipEvent_t b) {
                hipExtLaunchKernelGGL((k_update<true, false, false>), dim3(ldv / UPD_ROWS), dim3(256), 0, s, a, b, 0, ldv, V, J,
                                      1, u0val, n, nullptr, w, f1, npart, part, nrb, h, nullptr, nullptr, nullptr, nullptr, nullptr);
            }),
            vbytes + 16.0 * n);
        rep("update<false> (prod, h given)", timeit([&](hipEvent_t a, hipEvent_t b) {
                hipExtLaunchKernelGGL((k_update<false, false, false>), dim3(ldv / UPD_ROWS), dim3(256), 0, s, a, b, 0, ldv, V,
                                      J, 1, u0val, n, h, w, f2, npart, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
            }),
            vbytes + 16.0 * n);
        {  // the fp32 shadow: tiny coefficients (the accuracy test passes), ||src||^2 = 1
            std::vector<double> ps(size_t(J + 2) * nrb, 1e-22), hs(J + 3, 1e-22 * nrb);
            for (int b = 0; b < nrb; ++b) ps[size_t(J + 1) * nrb + b] = 1.0 / nrb;
            hs[J + 1] = 1.0;
            CK(hipMemcpy(psm, ps.data(), ps.size() * 8, hipMemcpyHostToDevice));
            CK(hipMemcpy(hsm, hs.data(), hs.size() * 8, hipMemcpyHostToDevice));
            CK(hipMemset(fb, 0, 4));
        }
        rep("update<true,B32> (RED)", timeit([&](hipEvent_t a, hipEvent_t b) {
                hipExtLaunchKernelGGL((k_update<true, true, false>), dim3(ldv / UPD_ROWS), dim3(256), 0, s, a, b, 0, ldv, V, J,
                                      1, u0val, n, nullptr, w, f1, npart, psm, nrb, h, V32, fb, nullptr, nullptr, nullptr);
            }),
            vbytes / 2 + 16.0 * n);
        rep("update<false,B32> (h given)", timeit([&](hipEvent_t a, hipEvent_t b) {
                hipExtLaunchKernelGGL((k_update<false, true, false>), dim3(ldv / UPD_ROWS), dim3(256), 0, s, a, b, 0, ldv, V,
                                      J, 1, u0val, n, hsm, w, f2, npart, nullptr, 0, nullptr, V32, fb, nullptr, nullptr, nullptr);
            }),
            vbytes / 2 + 16.0 * n);
        {
            unsigned nf = 0;
            CK(hipMemcpy(&nf, fb, 4, hipMemcpyDeviceToHost));
            if (nf) std::printf("  B32 fell back %u times\n", nf);
        }
        rep("read_rows32<256,16>", timeit([&](hipEvent_t a, hipEvent_t b) {
                hipExtLaunchKernelGGL((read_rows32<256, 16>), dim3(ldv / 512), dim3(256), 0, s, a, b, 0, ldv, V32, J, w,
                                      out);
            }),
            vbytes / 2 + 8.0 * n);
        {
            std::vector<double> a(ldv), b(ldv);
            CK(hipMemcpy(a.data(), f1, size_t(ldv) * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), f2, size_t(ldv) * 8, hipMemcpyDeviceToHost));
            if (std::memcmp(a.data(), b.data(), size_t(ldv) * 8)) std::printf("  update<true> != update<false>\n");
        }
        rep("reduce_cols", timeit([&](hipEvent_t a, hipEvent_t b) {
                hipExtLaunchKernelGGL(k_reduce_cols, dim3((J + 1 + 127) / 128), dim3(256), 0, s, a, b, 0, part, nrb,
                                      J + 1, h);
            }),
            8.0 * (J + 1) * nrb);
#define UPDV(T, UB)                                                                                       \
    rep("upd_var<" #T "," #UB "> (no u0)", timeit([&](hipEvent_t a, hipEvent_t b) {                       \
            hipExtLaunchKernelGGL((upd_var<T, UB>), dim3(ldv / (2 * T)), dim3(T), 0, s, a, b, 0, ldv, V, J, h, w, \
                                  f2);                                                                    \
        }),                                                                                               \
        vbytes + 16.0 * n)
        UPDV(256, 8);
        UPDV(128, 8);
        UPDV(64, 8);
        UPDV(64, 4);
        UPDV(128, 4);
#define READV(T, UB)                                                                                          \
    rep("read_rows<" #T "," #UB ">", timeit([&](hipEvent_t a, hipEvent_t b) {                                 \
            hipExtLaunchKernelGGL((read_rows<T, UB>), dim3(ldv / (2 * T)), dim3(T), 0, s, a, b, 0, ldv, V, J, w, out); \
        }),                                                                                                   \
        vbytes + 8.0 * n)
        READV(256, 8);
        READV(128, 8);
        READV(64, 8);
        READV(64, 16);
        rep("read_tiles (1024x8)", timeit([&](hipEvent_t a, hipEvent_t b) {
                hipExtLaunchKernelGGL(read_tiles, dim3(nrb * ((J + 7) / 8)), dim3(256), 0, s, a, b, 0, ldv, nrb, V, J,
                                      out);
            }),
            vbytes);
    }
    return 0;
}
