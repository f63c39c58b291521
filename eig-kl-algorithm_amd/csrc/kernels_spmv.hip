// fp64 CSR SpMV y = L x for gfx950 (the Lanczos operator, replacing
// Spectra's SparseSymMatProd<double>::perform_op at cEIG.cpp:194 and the
// reference GPU sparseMVKernel at gKL2.cu:65-89, which was one fp32 lane per
// row on a non-symmetric operator).
//
// Design (HBM/MALL-bound, ~0.17 flop/B, no MFMA): CSR-adaptive row blocks
// precomputed on the host so every 256-thread workgroup owns a contiguous
// nnz range of at most BLOCK_NNZ entries:
//   stream mode : the workgroup streams its val/col range with fully
//                 coalesced loads (8 B + 4 B per lane), gathers x, stores the
//                 products in LDS, then reduces each row with a power-of-two
//                 group of lanes (1..64 lanes per row, chosen from the rows in
//                 the block) — short circuit rows (avg 6.5 nnz) never waste a
//                 wave on one row;
//   vector mode : a row longer than BLOCK_NNZ gets a workgroup to itself and
//                 a strided + wave64 shuffle + LDS tree reduction.
// Every reduction has a fixed shape, so results are bitwise reproducible.
// Fused Lanczos epilogue: y is scaled by 1/sqrt(*fn2) and, when vcol != null,
// the basis column vcol[r] = f[r]/sqrt(*fn2) is written for the same rows
// (the matvec runs on the unscaled residual f, so there is no separate
// normalise kernel as in gKL2.cu:177-188).
#include <hip/hip_runtime.h>

#include "ek_internal.hpp"

namespace ek {
namespace dev {

std::vector<int32_t> spmv_row_blocks(const int32_t* rowptr, int64_t nrows, int block_nnz) {
    std::vector<int32_t> rb{0};
    int64_t rows_in = 0, nnz_in = 0;
    for (int64_t r = 0; r < nrows; ++r) {
        const int64_t len = rowptr[r + 1] - rowptr[r];
        if (rows_in > 0 && (nnz_in + len > block_nnz || rows_in == SPMV_THREADS)) {
            rb.push_back(int32_t(r));
            rows_in = nnz_in = 0;
        }
        ++rows_in;
        nnz_in += len;
        if (len > block_nnz) {  // long row: a workgroup of its own (vector mode)
            rb.push_back(int32_t(r + 1));
            rows_in = nnz_in = 0;
        }
    }
    if (rb.back() != int32_t(nrows)) rb.push_back(int32_t(nrows));
    return rb;
}

template <int BLOCK_NNZ>
__global__ __launch_bounds__(SPMV_THREADS) void k_spmv_adaptive(const int32_t* __restrict__ rb,
                                                                const int32_t* __restrict__ rowptr,
                                                                const int32_t* __restrict__ col,
                                                                const double* __restrict__ val,
                                                                const double* __restrict__ x, double* __restrict__ y,
                                                                const double* __restrict__ fn2,
                                                                const double* __restrict__ f,
                                                                double* __restrict__ vcol) {
    __shared__ double prod[BLOCK_NNZ];
    __shared__ double wsum[SPMV_THREADS / 64];
    const int t = threadIdx.x;
    const int r0 = rb[blockIdx.x], r1 = rb[blockIdx.x + 1];
    const int nr = r1 - r0;
    const int p0 = rowptr[r0];
    const int cnt = rowptr[r1] - p0;
    const double scale = fn2 ? 1.0 / sqrt(*fn2) : 1.0;

    if (cnt > BLOCK_NNZ) {  // vector mode: single long row
        double s = 0.0;
        for (int i = t; i < cnt; i += SPMV_THREADS) s += val[p0 + i] * x[col[p0 + i]];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if ((t & 63) == 0) wsum[t >> 6] = s;
        __syncthreads();
        if (t == 0) {
            double a = 0.0;
#pragma unroll
            for (int w = 0; w < SPMV_THREADS / 64; ++w) a += wsum[w];
            y[r0] = a * scale;
            if (vcol) vcol[r0] = f[r0] * scale;
        }
        return;
    }
    // stream mode: coalesced products into LDS
    for (int i = t; i < cnt; i += SPMV_THREADS) prod[i] = val[p0 + i] * x[col[p0 + i]];
    __syncthreads();
    // lanes per row: largest power of two with nr * L <= 256, capped at one wave
    int L = SPMV_THREADS / (nr > 0 ? nr : 1);
    L = L >= 64 ? 64 : L >= 32 ? 32 : L >= 16 ? 16 : L >= 8 ? 8 : L >= 4 ? 4 : L >= 2 ? 2 : 1;
    const int g = t / L, lane = t % L;
    double s = 0.0;
    int row = r0 + g;
    if (g < nr) {
        const int b = rowptr[row] - p0, e = rowptr[row + 1] - p0;
        for (int i = b + lane; i < e; i += L) s += prod[i];
    }
    for (int o = L >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, L);
    if (g < nr && lane == 0) {
        y[row] = s * scale;
        if (vcol) vcol[row] = f[row] * scale;
    }
}

void spmv(hipStream_t s, int nblocks, const int32_t* rb, const int32_t* rowptr, const int32_t* col,
          const double* val, const double* x, double* y, const double* fn2, const double* f, double* vcol,
          int block_nnz) {
    if (nblocks <= 0) return;
    switch (block_nnz) {
        case 512:
            hipLaunchKernelGGL(k_spmv_adaptive<512>, dim3(nblocks), dim3(SPMV_THREADS), 0, s, rb, rowptr, col, val,
                               x, y, fn2, f, vcol);
            break;
        case 2048:
            hipLaunchKernelGGL(k_spmv_adaptive<2048>, dim3(nblocks), dim3(SPMV_THREADS), 0, s, rb, rowptr, col, val,
                               x, y, fn2, f, vcol);
            break;
        default:
            hipLaunchKernelGGL(k_spmv_adaptive<1024>, dim3(nblocks), dim3(SPMV_THREADS), 0, s, rb, rowptr, col, val,
                               x, y, fn2, f, vcol);
            break;
    }
}

}  // namespace dev
}  // namespace ek
