// fp64 CSR SpMV y = L x for gfx950 (the Lanczos operator, replacing
// Spectra's SparseSymMatProd<double>::perform_op at cEIG.cpp:194 and the
// reference GPU sparseMVKernel at gKL2.cu:65-89, which was one fp32 lane per
// row on a non-symmetric operator).
//
// Design (HBM/MALL-bound, ~0.17 flop/B, no MFMA): CSR-adaptive row blocks
// precomputed on the host so every 256-thread workgroup owns a contiguous
// nnz range of at most BLOCK_NNZ entries, described by ONE 16-byte record
// {row0, nrows, nnz0, cnt} (a single load starts the dependency chain):
//   stream mode : the workgroup streams its val/col range with fully
//                 coalesced loads (8 B + 4 B per lane) while it stages its rows'
//                 boundaries in LDS, gathers x, stores the products in LDS,
//                 then reduces each row with a power-of-two group of lanes
//                 (1..64 lanes per row, chosen from the rows in the block) —
//                 short circuit rows (avg 6.5 nnz) never waste a wave;
//   vector mode : a row longer than BLOCK_NNZ gets a workgroup to itself and
//                 a strided + wave64 shuffle + LDS tree reduction.
// Every reduction has a fixed shape, so results are bitwise reproducible.
// Fused Lanczos epilogue: y is scaled by 1/sqrt(*fn2); when vcol != null the
// basis column vcol[r] = f[r]/sqrt(*fn2) is written for the same rows (the
// matvec runs on the unscaled residual f, so there is no separate normalise
// kernel as in gKL2.cu:177-188), and when apart != null the block's partial of
// alpha = vcol . y is written (fixed tree) for the three-term recurrence.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "ek_device.hpp"
#include "ek_internal.hpp"

namespace ek {
namespace dev {

// Host preparation of the row blocks and the coded segments: spmv_host.cpp.

__device__ __forceinline__ void finalize_publish(const StepFin& f, double n2) {
    f.fn2_out[0] = n2;
    if (f.step >= 0) {
        f.alpha[f.step] = *f.a3 + f.h2[f.step];
        if (f.step > 0) f.offd[f.step] = (isnan(f.bov_i[0]) ? sqrt(f.fn2_i[0]) : f.bov_i[0]) + f.h2[f.step - 1];
    }
}

// thread-strided partial of sum(x[0:n)): x[t] + x[t+256] + ... in order (the
// order of k_finalize_step), loads batched so they are in flight together
__device__ __forceinline__ double strided_sum(const double* __restrict__ x, int n, int stride,
                                              const int* __restrict__ idx = nullptr) {
    double s = 0.0;
    for (int i0 = threadIdx.x; i0 < n; i0 += 4 * SPMV_THREADS) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            v[u] = i0 + u * SPMV_THREADS < n
                       ? x[idx ? size_t(idx[i0 + u * SPMV_THREADS]) : size_t(i0 + u * SPMV_THREADS) * size_t(stride)]
                       : 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i0 + u * SPMV_THREADS < n) s += v[u];
    }
    return s;
}

// the fixed tree over the workgroup of the thread partials; every thread gets it.
// (A barrier-free form where every wave reduces all 1024 partials itself, same
// bits, measured slower inside the solve: 15.3 vs 12.7 us per SpMV.)
__device__ __forceinline__ double block_sum_all(double s, double* wsum) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
    __syncthreads();
    const double r = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
    __syncthreads();
    return r;
}

// The three-term recurrence's alpha = sum of every block's partial, reduced by
// the LAST block to finish (no separate launch; k_three_term's order: each
// thread sums the partials t, t + 256, ... in turn, then the fixed tree, so
// alpha has the bits k_three_term computes).  Hand-off (MI355X_MICROARCH.md,
// inter-workgroup visibility, the sc1 row): each block's partial is stored
// sc1 by thread 0, which waits for it (vmcnt 0) before its agent-scope add to
// the counter; the block whose add returns gridDim - 1 reads every partial
// with sc1 loads after a barrier, publishes alpha and re-arms the counter
// (visible to the next launch at the kernel boundary).
__device__ __forceinline__ void store_sc1(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), static_cast<unsigned long long>(__double_as_longlong(v)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_sc1(const double* p) {
    return __longlong_as_double(static_cast<long long>(__hip_atomic_load(
        reinterpret_cast<unsigned long long*>(const_cast<double*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}
// Which block is last: a two-level counter (one add per block on one of
// ALPHA_SUB counters, each on a 256-B line of its own, and one add on the top
// counter by the block completing each group).  Adds to ONE address from
// every block serialise at the memory side: ~8 ns each, +26 us per launch of
// 2,583 blocks when every block added to a single counter.
__device__ __forceinline__ bool alpha_last_block(unsigned* ctr) {
    const unsigned nb = gridDim.x, g = blockIdx.x % ALPHA_SUB;
    const unsigned gsize = (nb - g + ALPHA_SUB - 1) / ALPHA_SUB, ngroups = nb < ALPHA_SUB ? nb : ALPHA_SUB;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (__hip_atomic_fetch_add(ctr + g * 64, 1u, EK_HANDOFF_ORDER, __HIP_MEMORY_SCOPE_AGENT) != gsize - 1u) return false;
    return __hip_atomic_fetch_add(ctr + ALPHA_SUB * 64, 1u, EK_HANDOFF_ORDER, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1u;
}
__device__ __forceinline__ void alpha_handoff(const double* apart, double* alpha_out, unsigned* ctr, double* wsum,
                                              int* s_last) {
    if (threadIdx.x == 0) *s_last = alpha_last_block(ctr) ? 1 : 0;
    __syncthreads();
    if (!*s_last) return;
    // every partial's load in flight at once (16 per thread per trip, clamped
    // index, 0.0 added past the end: s + 0.0 == s as s never becomes -0): one
    // memory round trip instead of one per partial the thread sums
    constexpr int AB = 16;
    const int nb = int(gridDim.x);
    double s = 0.0;
    for (int i0 = int(threadIdx.x); i0 < nb; i0 += AB * SPMV_THREADS) {
        double v[AB];
#pragma unroll
        for (int u = 0; u < AB; ++u) v[u] = load_sc1(apart + min(i0 + u * SPMV_THREADS, nb - 1));
#pragma unroll
        for (int u = 0; u < AB; ++u) s += i0 + u * SPMV_THREADS < nb ? v[u] : 0.0;
    }
    s = block_sum_all(s, wsum);
    if (threadIdx.x < ALPHA_SUB + 1) ctr[threadIdx.x * 64] = 0u;  // re-armed for the next launch
    if (threadIdx.x == 0) *alpha_out = s;
}

// PK: entries are dictionary-coded 32-bit words in per-block segments
// (SpmvMat::seg, spmv_segment); `col` then holds the segments, `val` the
// dictionary and `rel` the row starts inside each segment.  Block b's entries
// and row starts sit at addresses given by b alone, so their loads go out
// together with the descriptor's instead of after it: the x gathers are two
// dependent memory round trips from the kernel start, not three.
#ifndef EK_SPMV_WAVES
#define EK_SPMV_WAVES 1  // minimum waves per SIMD asked of the compiler (its register budget; 1: unconstrained)
#endif
// LONG: some block is a single row longer than BLOCK_NNZ (vector mode);
// ALAST: the last block reduces alpha (alpha_out).  Without them the kernel
// carries neither path: fewer registers, more resident workgroups.
template <int BLOCK_NNZ, bool PK, bool LONG = true, bool ALAST = true>
__global__ __launch_bounds__(SPMV_THREADS, EK_SPMV_WAVES) void k_spmv_adaptive(const int4* __restrict__ desc,
                                                                const int32_t* __restrict__ rowptr,
                                                                const int32_t* __restrict__ col,
                                                                const double* __restrict__ val, int colbits,
                                                                const uint16_t* __restrict__ rel,
                                                                const double* __restrict__ x, double* __restrict__ y,
                                                                const double* __restrict__ fn2,
                                                                const double* __restrict__ f,
                                                                double* __restrict__ vcol, double* __restrict__ apart,
                                                                StepFin fin, double* __restrict__ alpha_out,
                                                                unsigned* __restrict__ actr) {
    constexpr int PER = BLOCK_NNZ / SPMV_THREADS;
    __shared__ double prod[BLOCK_NNZ];
    __shared__ int rbeg[SPMV_THREADS + 1];
    __shared__ double wsum[SPMV_THREADS / 64];
    __shared__ double wsum2[SPMV_THREADS / 64];
    __shared__ int s_last;
    const int t = threadIdx.x;
    if (fin.pub_rearm && blockIdx.x == 0 && t < PRO_PUB_WORDS) fin.pub_rearm[PRO_PUB_STRIDE * t] = 0u;
    uint32_t wd[PER];
    int rb0 = 0, rb1 = 0;
    if constexpr (PK) {  // speculative: a long-row block's segment is padding
#pragma unroll
        for (int u = 0; u < PER; ++u) wd[u] = uint32_t(col[size_t(blockIdx.x) * BLOCK_NNZ + t + u * SPMV_THREADS]);
        rb0 = rel[size_t(blockIdx.x) * SPMV_REL_STRIDE + t];
        if (t == 0) rb1 = rel[size_t(blockIdx.x) * SPMV_REL_STRIDE + SPMV_THREADS];
    }
    const int4 dsc = desc[blockIdx.x];
    const int r0 = dsc.x, nr = dsc.y, p0 = dsc.z, cnt = dsc.w;
    // ||f||^2: folded finalize of the previous Lanczos step (every block sums
    // the same partials in the same order; block 0 publishes) or read.  The
    // partials do not depend on the block descriptor, so their loads go out
    // early; the tree (with its barriers) runs after the block's gathers are
    // issued, and the scale is only needed by the epilogue.  (Measured inside
    // the solve: loading them in the segment's round trip, 13.1 us, or every
    // wave reducing all of them without barriers, 15.3 us, were both slower
    // than this form, 12.7 us.)
    // (fin.fast: the update's ||f'||^2 - ||h||^2, one value; the partials
    // only when it is NaN, a breakdown)
    const double fastv = fin.fast ? *fin.fast : __builtin_nan("");
    const bool sum_parts = fin.npart && isnan(fastv);  // (uniform over the workgroup)
    const double npart_t = sum_parts ? strided_sum(fin.npart, fin.nb, fin.nstride, fin.nidx) : 0.0;
    auto norm2 = [&]() -> double {
        if (fin.npart) {
            const double n2 = sum_parts ? block_sum_all(npart_t, wsum) : fastv;
            if (blockIdx.x == 0 && t == 0) finalize_publish(fin, n2);
            return n2;
        }
        return fn2 ? *fn2 : 1.0;
    };
    // an exact breakdown (f = 0) yields a zero column instead of NaN; the host
    // driver detects it and injects a fresh vector (Lanczos::inject)
    auto scale_of = [&](double n2) { return (fn2 || fin.npart) ? (n2 > 0.0 ? 1.0 / sqrt(n2) : 0.0) : 1.0; };

    if (LONG && cnt > BLOCK_NNZ) {  // vector mode: single long row
        const double scale = scale_of(norm2());
        if (fin.chk_dst && blockIdx.x == 0) chk_mirror(fin, t, SPMV_THREADS);
        double s = 0.0;
        const uint32_t cmask = (1u << colbits) - 1u;
        const int olo = fin.own_lo, ohi = fin.own_hi;  // (the halo SpMV: the own slot's entries are 0)
        for (int i = t; i < cnt; i += SPMV_THREADS) {
            if constexpr (PK) {
                const uint32_t wd = uint32_t(col[p0 + i]);
                const int c = int(wd & cmask);
                s += c >= olo && c < ohi ? 0.0 : val[wd >> colbits] * x[c];
            } else {
                const int c = col[p0 + i];
                s += c >= olo && c < ohi ? 0.0 : val[p0 + i] * x[c];
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if ((t & 63) == 0) wsum[t >> 6] = s;
        __syncthreads();
        if (t == 0) {
            const double a0 = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
            const double a = fin.ybase ? fin.ybase[r0] + a0 : a0;
            out_store(y + r0, a * scale);
            if (vcol) {
                const double v = f[r0] * scale;
                out_store(vcol + r0, v);
                if (fin.v32col) out_store(fin.v32col + r0, float(v));
                if (apart) store_sc1(apart + blockIdx.x, v * (a * scale));
                if (fin.wpart) fin.wpart[blockIdx.x] = (a * scale) * (a * scale);
            }
        }
        if (ALAST && alpha_out) alpha_handoff(apart, alpha_out, actr, wsum, &s_last);
        return;
    }
    // stream mode: every global load of the block is issued before the first
    // use (fixed trip count), products to LDS, row boundaries to LDS
    int ci[PER];
    double vv[PER];
    if constexpr (PK) {  // padding entries are (col 0, code 0): valid loads, never summed
        const uint32_t cmask = (1u << colbits) - 1u;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            ci[u] = int(wd[u] & cmask);
            vv[u] = val[wd[u] >> colbits];
        }
    } else {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = t + u * SPMV_THREADS;
            ci[u] = i < cnt ? col[p0 + i] : -1;
            vv[u] = i < cnt ? val[p0 + i] : 0.0;
        }
    }
    if constexpr (!PK) {
        rb0 = t <= nr ? rowptr[r0 + t] - p0 : 0;
        rb1 = (t == 0 && nr == SPMV_THREADS) ? rowptr[r0 + SPMV_THREADS] - p0 : 0;
    }
    // lanes per row: largest power of two with nr * L <= 256, capped at one wave
    int L = SPMV_THREADS / (nr > 0 ? nr : 1);
    L = L >= 64 ? 64 : L >= 32 ? 32 : L >= 16 ? 16 : L >= 8 ? 8 : L >= 4 ? 4 : L >= 2 ? 2 : 1;
    const int g = t / L, lane = t % L;
    // the epilogue runs in each row's first lane (it holds the row's sum): its
    // f is prefetched now (no LDS hand-off of y and no barrier before it)
    const double fr = (vcol && g < nr && lane == 0) ? f[r0 + g] : 0.0;
    double xv[PER];
    if (fin.own_hi > fin.own_lo) {  // the halo SpMV: the own slot's entries are summed by the owned-slot SpMV
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const bool own = ci[u] >= fin.own_lo && ci[u] < fin.own_hi;
            xv[u] = ci[u] >= 0 && !own ? x[ci[u]] : 0.0;
            vv[u] = own ? 0.0 : vv[u];
        }
    } else {
#pragma unroll
        for (int u = 0; u < PER; ++u) xv[u] = ci[u] >= 0 ? x[ci[u]] : 0.0;
    }
    const double scale = scale_of(norm2());  // overlaps the gathers in flight
    if (fin.chk_dst && blockIdx.x == 0) chk_mirror(fin, t, SPMV_THREADS);  // (the check's copy: block 0 only)
    if (t <= nr) rbeg[t] = rb0;
    if (t == 0 && nr == SPMV_THREADS) rbeg[SPMV_THREADS] = rb1;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int i = t + u * SPMV_THREADS;
        if (i < cnt) prod[i] = vv[u] * xv[u];
    }
    __syncthreads();
    double s = 0.0;
    if (g < nr)
        for (int i = rbeg[g] + lane; i < rbeg[g + 1]; i += L) s += prod[i];
    for (int o = L >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, L);
    // y, and the basis column + alpha / ||w||^2 terms of row g, in its first lane
    double av = 0.0, wv = 0.0;
    if (g < nr && lane == 0) {
        const double yr = (fin.ybase ? fin.ybase[r0 + g] + s : s) * scale;
        out_store(y + r0 + g, yr);
        if (vcol) {
            const double v = fr * scale;
            out_store(vcol + r0 + g, v);
            if (fin.v32col) out_store(fin.v32col + r0 + g, float(v));
            av = v * yr;
            wv = yr * yr;
        }
    }
    if (vcol) {
        if (apart) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) av += __shfl_xor(av, o, 64);
            if ((t & 63) == 0) wsum[t >> 6] = av;
            if (fin.wpart) {  // ||w||^2 partial (partial reorthogonalisation's beta estimate)
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) wv += __shfl_xor(wv, o, 64);
                if ((t & 63) == 0) wsum2[t >> 6] = wv;
            }
            __syncthreads();
            if (t == 0) store_sc1(apart + blockIdx.x, (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]));
            if (t == 0 && fin.wpart) fin.wpart[blockIdx.x] = (wsum2[0] + wsum2[1]) + (wsum2[2] + wsum2[3]);
        }
    }
    if (ALAST && alpha_out) alpha_handoff(apart, alpha_out, actr, wsum, &s_last);
}

void spmv(hipStream_t s, const SpmvMat& m, const double* x, double* y, const double* fn2, const double* f,
          double* vcol, double* apart, const StepFin* fin, hipEvent_t ev_start, hipEvent_t ev_stop, double* alpha_out,
          unsigned* actr) {
    if (m.panel.G > 0) {
        spmv_panel(s, m.panel, m.dict, x, y, fn2, f, vcol, apart, fin, ev_start, ev_stop, alpha_out, actr);
        return;
    }
    if (m.nblocks <= 0) return;
    const int4* d = reinterpret_cast<const int4*>(m.desc);
    const StepFin fv = fin ? *fin : StepFin{};
    const int32_t* c = m.pk ? reinterpret_cast<const int32_t*>(m.pk) : m.col;
    const double* v = m.pk ? m.dict : m.val;
    // with events: HIP records the kernel's own start/end timestamps (what
    // rocprofv3 reports), not event packets around it
    // (without events a plain launch: the one a captured HIP graph records)
#define EK_SPMV_LAUNCH_K(KERNEL_)                                                                                  \
    do {                                                                                                           \
        if (ev_start || ev_stop)                                                                                   \
            hipExtLaunchKernelGGL(KERNEL_, dim3(m.nblocks), dim3(SPMV_THREADS), 0, s, ev_start, ev_stop, 0, d,       \
                                  m.rowptr, c, v, m.colbits, m.rel, x, y, fn2, f, vcol, apart, fv, alpha_out, actr);  \
        else                                                                                                       \
            hipLaunchKernelGGL(KERNEL_, dim3(m.nblocks), dim3(SPMV_THREADS), 0, s, d, m.rowptr, c, v, m.colbits,      \
                               m.rel, x, y, fn2, f, vcol, apart, fv, alpha_out, actr);                              \
    } while (0)
#define EK_SPMV_LAUNCH(BN, PK) EK_SPMV_LAUNCH_K((k_spmv_adaptive<BN, PK>))
    if (m.pk) {
        if (m.has_long || alpha_out) EK_SPMV_LAUNCH(SPMV_SEG_NNZ, true);
        else EK_SPMV_LAUNCH_K((k_spmv_adaptive<SPMV_SEG_NNZ, true, false, false>));
    } else {
        if (m.block_nnz == SPMV_SEG_NNZ) {
            // the <.., false, false> variant compiles out the ALAST hand-off,
            // so a caller asking for alpha_out needs the full one
            if (m.has_long || alpha_out) EK_SPMV_LAUNCH(SPMV_SEG_NNZ, false);
            else EK_SPMV_LAUNCH_K((k_spmv_adaptive<SPMV_SEG_NNZ, false, false, false>));
        } else {
            switch (m.block_nnz) {
                case 512: EK_SPMV_LAUNCH(512, false); break;
                case 2048: EK_SPMV_LAUNCH(2048, false); break;
                default: EK_SPMV_LAUNCH(1024, false); break;
            }
        }
    }
#undef EK_SPMV_LAUNCH
#undef EK_SPMV_LAUNCH_K
}

// The gather-only ceiling of the CSR-segment form (ek_spmv_gather_bench;
// VERDICT r5 next-4): k_spmv_adaptive's grid and block descriptors, the same
// segment words (or plain col / val) and row starts streamed, and the same x
// and value-table gathers, with the products summed in registers — no LDS
// staging, no row reduction, no epilogue, no y.
template <int BLOCK_NNZ, bool PK>
__global__ __launch_bounds__(SPMV_THREADS) void k_spmv_gather_only(const int4* __restrict__ desc,
                                                                   const int32_t* __restrict__ col,
                                                                   const double* __restrict__ val, int colbits,
                                                                   const uint16_t* __restrict__ rel,
                                                                   const double* __restrict__ x,
                                                                   double* __restrict__ sink) {
    constexpr int PER = BLOCK_NNZ / SPMV_THREADS;
    const int t = threadIdx.x;
    const uint32_t cmask = (1u << colbits) - 1u;
    uint32_t wd[PER];
    int rb = 0;
    if constexpr (PK) {
#pragma unroll
        for (int u = 0; u < PER; ++u) wd[u] = uint32_t(col[size_t(blockIdx.x) * BLOCK_NNZ + t + u * SPMV_THREADS]);
        rb = rel[size_t(blockIdx.x) * SPMV_REL_STRIDE + t];
    }
    const int4 dsc = desc[blockIdx.x];
    const int p0 = dsc.z, cnt = dsc.w;
    double acc = 0.0;
    if (cnt > BLOCK_NNZ) {  // a long row (vector mode)
        for (int i = t; i < cnt; i += SPMV_THREADS) {
            if constexpr (PK) {
                const uint32_t w = uint32_t(col[p0 + i]);
                acc += val[w >> colbits] * x[w & cmask];
            } else {
                acc += val[p0 + i] * x[col[p0 + i]];
            }
        }
    } else {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = t + u * SPMV_THREADS;
            if constexpr (PK) {
                acc += val[wd[u] >> colbits] * x[wd[u] & cmask];
            } else if (i < cnt) {
                acc += val[p0 + i] * x[col[p0 + i]];
            }
        }
    }
    if (acc == -1.2345e300 && rb == 7) sink[blockIdx.x] = acc;  // (keeps every load; never true in practice)
}

// (lab: VERDICT r5 next-4's single-grid question, ek_spmv_gather_bench with
// EK_GATHER_MODE 1-3) A skipped Lanczos step is the SpMV, then a launch that
// reduces the SpMV's per-block partials (alpha) and updates every row
// elementwise (f = w - alpha v - beta u, with ||f||^2 partials).  Fusing the two
// into one grid replaces that kernel boundary by an in-launch grid-wide wait:
// every block's partial must be in before any block may update.  These lab
// kernels price the two forms on the product's grid and access pattern:
// k_lab_gather_step<false> + k_lab_step (mode 1: the boundary) against
// k_lab_gather_step<true> (mode 2: the wait; all blocks resident, counted by
// the host), and k_lab_step alone (mode 3: the update's own time).  The
// partials travel as agent-scope stores and loads and the arrival count is a
// relaxed add after vmcnt(0), the product's hand-off idiom (EK_HANDOFF_ORDER).
__device__ __forceinline__ double lab_block_sum(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int t = threadIdx.x;
    if ((t & 63) == 0) red[t >> 6] = v;
    __syncthreads();
    double r = 0.0;
    for (int i = 0; i < SPMV_THREADS / 64; ++i) r += red[i];
    __syncthreads();
    return r;
}
__device__ __forceinline__ void lab_step_body(const double* part, int G, int n, const double* w, const double* v,
                                              const double* u, double* f, double* fpart, double beta, double* red) {
    const int t = threadIdx.x;
    double a = 0.0;
    for (int i = t; i < G; i += SPMV_THREADS)
        a += __hip_atomic_load(part + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const double alpha = lab_block_sum(a, red);
    const int per = (n + int(gridDim.x) - 1) / int(gridDim.x);
    const int r0 = int(blockIdx.x) * per, r1 = min(n, r0 + per);
    double q = 0.0;
    for (int i = r0 + t; i < r1; i += SPMV_THREADS) {
        const double fi = w[i] - alpha * v[i] - beta * u[i];
        f[i] = fi;
        q += fi * fi;
    }
    q = lab_block_sum(q, red);
    if (t == 0) fpart[blockIdx.x] = q;
}
template <bool WAIT>
__global__ __launch_bounds__(SPMV_THREADS) void k_lab_gather_step(const int4* __restrict__ desc,
                                                                  const int32_t* __restrict__ col,
                                                                  const double* __restrict__ val, int colbits,
                                                                  const uint16_t* __restrict__ rel,
                                                                  const double* __restrict__ x, double* part,
                                                                  unsigned* ctr, unsigned target, int n,
                                                                  const double* w, const double* v, const double* u,
                                                                  double* f, double* fpart) {
    __shared__ double red[SPMV_THREADS / 64];
    constexpr int PER = SPMV_SEG_NNZ / SPMV_THREADS;
    const int t = threadIdx.x;
    const uint32_t cmask = (1u << colbits) - 1u;
    uint32_t wd[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) wd[k] = uint32_t(col[size_t(blockIdx.x) * SPMV_SEG_NNZ + t + k * SPMV_THREADS]);
    const int rb = rel[size_t(blockIdx.x) * SPMV_REL_STRIDE + t];
    const int4 dsc = desc[blockIdx.x];
    double acc = 0.0;
    if (dsc.w > SPMV_SEG_NNZ) {
        for (int i = t; i < dsc.w; i += SPMV_THREADS) {
            const uint32_t wv = uint32_t(col[dsc.z + i]);
            acc += val[wv >> colbits] * x[wv & cmask];
        }
    } else {
#pragma unroll
        for (int k = 0; k < PER; ++k) acc += val[wd[k] >> colbits] * x[wd[k] & cmask];
    }
    acc += double(rb) * 0.0;
    const double bs = lab_block_sum(acc, red);
    if (t == 0) __hip_atomic_store(part + blockIdx.x, bs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (WAIT) {
        // two-level arrival (one counter for every block serialises ~2k adds
        // on one line): block b adds to sub-counter b % 32 (64 uints apart);
        // the last of a sub adds to the top counter; the last of those stores
        // the generation into 32 flag lines, each polled by its sub's blocks
        if (t == 0) {
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the partial is stored before the arrival
            const unsigned G = gridDim.x, sub = blockIdx.x & 31u, nsub = G < 32u ? G : 32u;
            const unsigned per = (G - sub + 31u) / 32u;  // blocks of this sub
            const unsigned old = __hip_atomic_fetch_add(ctr + 64 * (1 + sub), 1u, EK_HANDOFF_ORDER, __HIP_MEMORY_SCOPE_AGENT);
            if (old + 1u == target * per) {
                const unsigned top = __hip_atomic_fetch_add(ctr, 1u, EK_HANDOFF_ORDER, __HIP_MEMORY_SCOPE_AGENT);
                if (top + 1u == target * nsub)
                    for (unsigned q = 0; q < nsub; ++q)
                        __hip_atomic_store(ctr + 64 * (33 + q), target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            while (__hip_atomic_load(ctr + 64 * (33 + sub), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target)
                __builtin_amdgcn_s_sleep(2);
        }
        __syncthreads();
        lab_step_body(part, int(gridDim.x), n, w, v, u, f, fpart, 0.5, red);
    }
}
__global__ __launch_bounds__(SPMV_THREADS) void k_lab_step(const double* part, int G, int n, const double* w,
                                                           const double* v, const double* u, double* f,
                                                           double* fpart) {
    __shared__ double red[SPMV_THREADS / 64];
    lab_step_body(part, G, n, w, v, u, f, fpart, 0.5, red);
}

int lab_step_capacity() {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&k_lab_gather_step<true>),
                                                     SPMV_THREADS, 0) != hipSuccess)
        return 0;
    return per * cus;
}

void lab_gather_step(hipStream_t s, const SpmvMat& m, int mode, const double* x, double* part, unsigned* ctr,
                     unsigned target, int n, const double* w, const double* v, const double* u, double* f,
                     double* fpart) {
    const int4* d = reinterpret_cast<const int4*>(m.desc);
    const int32_t* pk = reinterpret_cast<const int32_t*>(m.pk);
    if (mode == 1 || mode == 2) {
        if (mode == 2)
            hipLaunchKernelGGL((k_lab_gather_step<true>), dim3(m.nblocks), dim3(SPMV_THREADS), 0, s, d, pk, m.dict,
                               m.colbits, m.rel, x, part, ctr, target, n, w, v, u, f, fpart);
        else
            hipLaunchKernelGGL((k_lab_gather_step<false>), dim3(m.nblocks), dim3(SPMV_THREADS), 0, s, d, pk, m.dict,
                               m.colbits, m.rel, x, part, ctr, target, n, w, v, u, f, fpart);
    }
    if (mode == 1 || mode == 3)
        hipLaunchKernelGGL(k_lab_step, dim3(m.nblocks), dim3(SPMV_THREADS), 0, s, part, m.nblocks, n, w, v, u, f, fpart);
}

void spmv_gather_only(hipStream_t s, const SpmvMat& m, const double* x, double* sink) {
    if (m.panel.G > 0) {
        panel_gather_only(s, m.panel, m.dict, x, sink);
        return;
    }
    if (m.nblocks <= 0) return;
    const int4* d = reinterpret_cast<const int4*>(m.desc);
    if (m.pk)
        hipLaunchKernelGGL((k_spmv_gather_only<SPMV_SEG_NNZ, true>), dim3(m.nblocks), dim3(SPMV_THREADS), 0, s, d,
                           reinterpret_cast<const int32_t*>(m.pk), m.dict, m.colbits, m.rel, x, sink);
    else
        switch (m.block_nnz) {
            case SPMV_SEG_NNZ:
                hipLaunchKernelGGL((k_spmv_gather_only<SPMV_SEG_NNZ, false>), dim3(m.nblocks), dim3(SPMV_THREADS), 0, s,
                                   d, m.col, m.val, 0, m.rel, x, sink);
                break;
            case 512:
                hipLaunchKernelGGL((k_spmv_gather_only<512, false>), dim3(m.nblocks), dim3(SPMV_THREADS), 0, s, d, m.col,
                                   m.val, 0, m.rel, x, sink);
                break;
            case 2048:
                hipLaunchKernelGGL((k_spmv_gather_only<2048, false>), dim3(m.nblocks), dim3(SPMV_THREADS), 0, s, d,
                                   m.col, m.val, 0, m.rel, x, sink);
                break;
            default:
                hipLaunchKernelGGL((k_spmv_gather_only<1024, false>), dim3(m.nblocks), dim3(SPMV_THREADS), 0, s, d,
                                   m.col, m.val, 0, m.rel, x, sink);
                break;
        }
}

}  // namespace dev
}  // namespace ek
