// Dense fp64 kernels of the Lanczos iteration on gfx950: classical
// Gram-Schmidt (twice) against the basis V (column-major, ld multiple of
// GT_ROWS, padded rows are zero), norms, and the restart GEMM V*Q.
// All HBM-bound (the basis is read 4x per step); every reduction is a fixed
// tree (wave64 xor-butterfly + LDS across waves + fixed-order combine), so
// the solver is bitwise reproducible run to run.
//
// Reference counterparts: Spectra's Lanczos factorization + DGKS
// re-orthogonalisation inside SymEigsSolver (cEIG.cpp:195-198), and the
// reference GPU computeNormKernel / normalizeVectorKernel (gKL2.cu:143-188),
// whose float atomicAdd norm is replaced by deterministic fp64 trees.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "ek_device.hpp"
#include "ek_internal.hpp"

#ifndef EK_UPD_UB
#define EK_UPD_UB 8  // basis columns per load batch of the update (two batches in flight)
#endif

namespace ek {
namespace dev {

// Lab only (EXTRA_DEFS=-DEK_PRO_STAMPS, tools/pro_stamps.py): per workgroup of
// the projection launch with the in-launch decision, its role and wall-clock
// stamps (s_memrealtime, 100 MHz) at entry, at its phase marks and at exit,
// for steps [PRO_STAMP_LO, PRO_STAMP_LO + PRO_STAMP_NS) of the last cycle to
// reach them; read by ek_lab_pro_stamps.  Compiled out otherwise.
#ifdef EK_PRO_STAMPS
constexpr int PRO_STAMP_LO = 20, PRO_STAMP_NS = 80, PRO_STAMP_WG = 2048, PRO_STAMP_W = 6;
__device__ unsigned long long g_pro_stamps[size_t(PRO_STAMP_NS) * PRO_STAMP_WG * PRO_STAMP_W];
__device__ __forceinline__ void pro_stamp(int step, int slot, unsigned long long val) {
    const int k = step - PRO_STAMP_LO;
    if (threadIdx.x == 0 && k >= 0 && k < PRO_STAMP_NS && int(blockIdx.x) < PRO_STAMP_WG)
        g_pro_stamps[(size_t(k) * PRO_STAMP_WG + blockIdx.x) * PRO_STAMP_W + slot] = val;
}
#define PRO_STAMP(slot) pro_stamp(ncols - 1, (slot), __builtin_amdgcn_s_memrealtime())
#define PRO_ROLE(r) pro_stamp(ncols - 1, 0, (r))
#define PRO_DECISION(v) pro_stamp(ncols - 1, 5, (v))
#else
#define PRO_STAMP(slot) ((void)0)
#define PRO_ROLE(r) ((void)0)
#define PRO_DECISION(v) ((void)0)
#endif

// projection slots of one column-group phase of the in-launch-decision
// launch: nrb rounded up to the 8 XCDs (gemvt_body's column-group-0-first map)
#ifndef EK_PRO_CG0_FIRST
#define EK_PRO_CG0_FIRST 1
#endif
#ifndef EK_PRO_NORM_DIRECT  // the merged fp32-shadow form: the norm hand-off writes ||f||^2 for a skipped step
#define EK_PRO_NORM_DIRECT 1
#endif
__host__ __device__ constexpr int pro_slots(int nrb) { return EK_PRO_CG0_FIRST ? (nrb + 7) / 8 * 8 : nrb; }

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// thread-strided partial of sum(x[0:n)): x[t] + x[t+256] + ... in this order,
// with the loads batched so they are in flight together (a plain strided loop
// waits for each load before the next add)
// (16 per batch, unconditional clamped loads and adds of 0.0 past the end: a
// load behind a branch waits for the loads before it; s + 0.0 == s because s
// starts at +0 and these sums never become -0.0)
__device__ __forceinline__ double strided_sum256(const double* __restrict__ x, int n) {
    constexpr int SB = 16;
    double s = 0.0;
    if (n <= 0) return s;
    for (int i0 = threadIdx.x; i0 < n; i0 += SB * 256) {
        double v[SB];
#pragma unroll
        for (int u = 0; u < SB; ++u) v[u] = x[min(i0 + u * 256, n - 1)];
#pragma unroll
        for (int u = 0; u < SB; ++u) s += i0 + u * 256 < n ? v[u] : 0.0;
    }
    return s;
}

// strided_sum256 of two arrays at once: both arrays' loads in flight together
// (one round trip instead of two); each sum in strided_sum256's order
__device__ __forceinline__ void strided_sum256x2(const double* __restrict__ x, const double* __restrict__ y, int n,
                                                 double& sx, double& sy) {
    constexpr int SB = 16;
    sx = 0.0;
    sy = 0.0;
    if (n <= 0) return;
    for (int i0 = threadIdx.x; i0 < n; i0 += SB * 256) {
        double vx[SB], vy[SB];
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            vx[u] = x[min(i0 + u * 256, n - 1)];
            vy[u] = y[min(i0 + u * 256, n - 1)];
        }
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            sx += i0 + u * 256 < n ? vx[u] : 0.0;
            sy += i0 + u * 256 < n ? vy[u] : 0.0;
        }
    }
}

#ifndef EK_TT_ROWS
#define EK_TT_ROWS 1024
#endif
constexpr int TT_ROWS = EK_TT_ROWS;  // rows per three-term block (ldv is a multiple of GT_ROWS = 1024)
static_assert(GT_ROWS % TT_ROWS == 0, "ldv must be a multiple of TT_ROWS");

// block of 256: returns the block sum in thread 0
__device__ __forceinline__ double block_sum256(double v, double* lds4) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) lds4[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) r = (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
    __syncthreads();
    return r;
}

// Agent-scope (sc1) stores / loads: the hand-off of partials between
// workgroups of one launch (MI355X_MICROARCH.md, inter-workgroup visibility).
// The counter adds that pick the last workgroup: EK_HANDOFF_ORDER
// (ek_internal.hpp; relaxed after an explicit vmcnt(0) wait, the partials
// themselves agent-scope atomics).
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), static_cast<unsigned long long>(__double_as_longlong(v)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __longlong_as_double(static_cast<long long>(__hip_atomic_load(
        reinterpret_cast<unsigned long long*>(const_cast<double*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}
constexpr int GT_SUB = 8;  // first-level counters per column group of the projection's hand-off

// Basis loads.  NT: non-temporal (no Infinity-Cache allocation), for a basis
// larger than the MALL, which it would otherwise sweep clean every pass,
// evicting the matrix and x the next SpMV reads
typedef double v2d_t __attribute__((ext_vector_type(2)));
typedef float v2f_t __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ double2 ld_basis(const double* p) {
    if constexpr (NT) {
        const v2d_t v = __builtin_nontemporal_load(reinterpret_cast<const v2d_t*>(p));
        return make_double2(v.x, v.y);
    } else {
        return *reinterpret_cast<const double2*>(p);
    }
}
template <bool NT>
__device__ __forceinline__ float2 ld_basis32(const float* p) {
    if constexpr (NT) {
        const v2f_t v = __builtin_nontemporal_load(reinterpret_cast<const v2f_t*>(p));
        return make_float2(v.x, v.y);
    } else {
        return *reinterpret_cast<const float2*>(p);
    }
}
constexpr int CS_LANES = 8;  // lanes per column of the canonical column sum (col_sum2)

// partial dot products of w with GT_COLS basis columns over GT_ROWS rows.
// 1-D grid of nrb * ncg blocks (ncg = ceil((ncols + has_u0) / GT_COLS));
// 256 threads, each GT_ROWS/512 double2 rows; column ncols is the deflation
// vector u0.  The blocks are dealt round-robin over the 8 XCDs; the
// (row block, column group) map gives each XCD a contiguous run of row
// blocks with all their column groups (the guide's bijective XCD remap), so
// a row block's slice of w is fetched into one XCD's L2 and re-read from
// there by its other column groups.  Same partials, same bits.
// TT: the right-hand side is the three-term residual f' = w - alpha v_i -
// beta_i v_{i-1}, formed per row with k_three_term's operations (alpha from
// the SpMV's last block, beta_i from ||f_i||^2 or the injected override),
// and the column-group-0 block of each row block stores it to fp for the
// update: the three-term launch and its per-block re-reduction of the alpha
// partials are gone, the bits are the same.
// h_out != null (nrb <= 8 * 32): the column sums are reduced in this launch.
// The partials are stored sc1; each workgroup's first wave waits for its
// stores and adds to its column group's counter (GT_SUB first-level counters
// on 256-B lines of their own, then a top counter); the workgroup completing
// a column group sums that group's partials (sc1 loads) in col_sum2's order —
// the bits k_reduce_cols and the update's in-kernel sums give — and writes
// h_out, so the update needs no reduction of its own (its prologue was a
// serial ~4 us of every update workgroup).  The counters are re-armed by
// that workgroup for the next launch.
// B32 (the fp32 basis shadow, k_update<_, true>): the column-group-0 block of
// each row block also writes ||rhs||^2 over its rows to part column
// ncols + has_u0 (the update's accuracy test reads the sum), and with TT
// the fp32 copy of v_i to v32col (vi rows are loaded here anyway).
// Partial reorthogonalisation: the decision for step i (ek_internal.hpp
// pro_step).  Simon's omega recurrence (Simon 1984; PROPACK's update_mu) for
// omega_{i+1,j} ~ v_{i+1}^T v_j:
//   beta_{i+1} omega_{i+1,j} = beta_{j+1} omega_{i,j+1} + (alpha_j - alpha_i) omega_{i,j}
//                              + beta_j omega_{i,j-1} - beta_i omega_{i-1,j}  (+- eps1 ||L||)
// with omega_{k,k} = 1; against u0 (L u0 = 0) the same with alpha_j = 0 and no
// neighbours.  beta_{i+1} is not known before the projection kernel forms f',
// so it is estimated from ||w||^2 - alpha^2 - beta_i^2 (w = L v_i, v_i and
// v_{i-1} orthonormal to far better than the threshold); a step whose
// estimate cancels below 2^-20 ||w||^2 projects.  One workgroup; thread j < i
// owns omega_{i+1,j}, thread 255 the u0 entry.
// (the body of k_pro and of the projection's decider workgroup, PROI; 256
// threads; returns the decision to every thread)
__device__ __forceinline__ bool pro_decide(const double* __restrict__ apart, const double* __restrict__ wpart,
                                           int nparts, double* __restrict__ a3, const double* __restrict__ fn2_i,
                                           const double* __restrict__ bov_i, const double* __restrict__ alpha,
                                           const double* __restrict__ offd, double* __restrict__ omega,
                                           ProState* __restrict__ st, int* __restrict__ flags, int i, int seg0, int m,
                                           double thresh, double eps1) {
    // no contraction into FMAs: the decision must come out the same in every
    // kernel this is inlined into (k_pro, the projection's decider) — with
    // contraction on, the two copies fused different products, so omega and
    // a decision near the threshold differed
#pragma clang fp contract(off)
    __shared__ double lds4[4];
    __shared__ double sh[4];
    __shared__ double mx4[4];
    __shared__ int s_pair, s_forced;
    const int t = int(threadIdx.x);
    constexpr int U = MAX_NCV;  // the u0 entry of a ring row
    double* onew = omega + size_t((i + 1) % 3) * OMEGA_LD;       // omega_{i+1}
    double* ocur = omega + size_t(i % 3) * OMEGA_LD;             // omega_i
    const double* oprev = omega + size_t((i + 2) % 3) * OMEGA_LD;  // omega_{i-1}
    // the recurrence's operands do not depend on the sums: their loads go out
    // first, so they return while the partials are reduced
    double r_al = 0.0, r_o0 = 0.0, r_o1 = 0.0, c_m1 = 0.0, c_0 = 0.0, c_p1 = 0.0, p_0 = 0.0;
    if (t < i) {
        r_al = alpha[t];
        r_o1 = t + 1 < i ? offd[t + 1] : 0.0;
        r_o0 = t > 0 ? offd[t] : 0.0;
        c_m1 = t > 0 ? ocur[t - 1] : 0.0;
        c_0 = ocur[t];
        c_p1 = t + 1 < i ? ocur[t + 1] : 1.0;  // (omega_{i,i} = 1)
        p_0 = t < i - 1 ? oprev[t] : 1.0;      // (omega_{i-1,i-1} = 1)
    } else if (t == 255) {
        c_0 = ocur[MAX_NCV];
        p_0 = oprev[MAX_NCV];
    }
    double s_an = 0.0, s_f2 = 0.0, s_bo = 0.0;
    int s_fo = 0;
    if (t == 0) {
        s_an = st->anorm;
        s_fo = st->force;
        s_f2 = *fn2_i;
        s_bo = *bov_i;
    }
    // alpha in k_three_term's order (the bits of every other alpha path), ||w||^2 alike
    // (both trees in one pass: wave sums, then one barrier for the cross-wave adds)
    double sa, sw;
    strided_sum256x2(apart, wpart, nparts, sa, sw);
    sa = wave_sum(sa);
    sw = wave_sum(sw);
    if ((t & 63) == 0) {
        lds4[t >> 6] = sa;
        mx4[t >> 6] = sw;
    }
    __syncthreads();
    if (t == 0) {
        sa = (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
        sw = (mx4[0] + mx4[1]) + (mx4[2] + mx4[3]);
        const double a = sa;
        *a3 = a;
        const double b = i > 0 ? (isnan(s_bo) ? sqrt(s_f2) : s_bo) : 0.0;
        const double b2 = sw - a * a - b * b;
        const bool valid = b2 > 0x1p-20 * sw;  // false for NaN
        const double bn = valid ? sqrt(b2) : 0.0;
        const double an = fmax(s_an, fabs(a) + b + bn);
        st->anorm = an;
        const int pair = s_fo || i == seg0;  // the first step of a run starts a pair like a triggered one
        sh[0] = a;
        sh[1] = b;
        sh[2] = bn;
        sh[3] = an;
        s_pair = pair;
        s_forced = pair || i == m - 1 || !valid;  // (the cycle's last step: f_m orthogonal for the restart)
    }
    __syncthreads();
    const double a = sh[0], b = sh[1], bn = sh[2], an = sh[3];
    const bool forced = s_forced != 0;
    double nv = 0.0;
    if (!forced) {
        if (t < i) {
            const int j = t;
            double x = j + 1 < i ? r_o1 * c_p1 : b;  // (omega_{i,i} = 1)
            x += (r_al - a) * c_0;
            if (j > 0) x += r_o0 * c_m1;
            x -= b * p_0;
            nv = (x + copysign(eps1 * an, x)) / bn;
        } else if (t == 255) {
            const double x = -a * c_0 - b * p_0;
            nv = (x + copysign(eps1 * an, x)) / bn;
        }
    }
    __syncthreads();  // (mx4 held ||w||^2's wave sums)
    double mx = fabs(nv);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if ((t & 63) == 0) mx4[t >> 6] = mx;
    __syncthreads();
    const double mxa = fmax(fmax(mx4[0], mx4[1]), fmax(mx4[2], mx4[3]));
    const bool d = forced || !(mxa <= thresh);  // (NaN: project)
    // after a projection the next vector is orthogonal to rounding: omega = eps1
    if (t < i) onew[t] = d ? eps1 : nv;
    if (t == i) onew[i] = eps1;
    if (t == 255) onew[U] = d ? eps1 : nv;
    if (i == seg0) {  // omega_i of a run's first vector (a restart's kept basis, an injected vector)
        if (t < i) ocur[t] = eps1;
        if (t == 255) ocur[U] = eps1;
    }
    if (t == 0) {
        flags[i] = d ? 1 : 0;
        st->force = (d && !s_pair) ? 1 : 0;
        if (d) st->projected += 1;
    }
    return d;
}

// The end of a projection launch for a step that does not project (k_pro):
// column group 0 only.  The block's ||f'||^2 partial goes to column tot (the
// update's accuracy test and the next SpMV's ||f||^2 read its sum); the
// column sums h are zero (no correction of H: the finalize adds h[i], h[i-1]).
// With the hand-off the workgroup completing column group 0 writes them; else
// (k_reduce_cols sums the partials) this block's partials of columns i and
// i-1, the two the finalize reads, are zeroed.
// zero_h false (PROI: the norm's own hand-off, run before the decision by
// every column-group-0 workgroup, on counters of its own): h is left alone
// (a projecting step's column groups write it; a skipped step's update
// zeroes the two entries the finalize reads)
__device__ __forceinline__ void gemvt_skip_tail(int ncols, int has_u0, int nrb, int rbk, int t,
                                                double* __restrict__ part, const double* nred,
                                                unsigned* __restrict__ gctr, double* __restrict__ h_out,
                                                double* __restrict__ fn2_fast, bool zero_h = true,
                                                unsigned* __restrict__ done = nullptr) {
    const int tot = ncols + has_u0, i = ncols - 1;
    __syncthreads();  // nred complete
    const double nb = (nred[0] + nred[1]) + (nred[2] + nred[3]);
    if (!h_out) {
        if (t == 0) part[size_t(tot) * nrb + rbk] = nb;
        if (t == 1) part[size_t(i) * nrb + rbk] = 0.0;
        if (t == 2 && i > 0) part[size_t(i - 1) * nrb + rbk] = 0.0;
        return;
    }
    __shared__ int s_last;
    if (t == 0) {
        st_sc1(part + size_t(tot) * nrb + rbk, nb);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int g = rbk % GT_SUB;
        const unsigned gsize = unsigned((nrb - g + GT_SUB - 1) / GT_SUB), ngroups = unsigned(nrb < GT_SUB ? nrb : GT_SUB);
        int last = 0;
        if (__hip_atomic_fetch_add(gctr + g * 64, 1u, EK_HANDOFF_ORDER, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1u)
            last = __hip_atomic_fetch_add(gctr + GT_SUB * 64, 1u, EK_HANDOFF_ORDER, __HIP_MEMORY_SCOPE_AGENT) ==
                   ngroups - 1u;
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    if (zero_h)
        for (int j = t; j < tot; j += 256) h_out[j] = 0.0;
    // the norm column in col_sum2's order (8 lanes, every 8th block, xor tree)
    if (t < CS_LANES) {
        const double* pc = part + size_t(tot) * nrb;
        constexpr int CB = 32;
        double a = 0.0;
        for (int b0 = t; b0 < nrb; b0 += CS_LANES * CB) {
            double va[CB];
#pragma unroll
            for (int u = 0; u < CB; ++u) va[u] = ld_sc1(pc + min(b0 + CS_LANES * u, nrb - 1));
#pragma unroll
            for (int u = 0; u < CB; ++u) a += b0 + CS_LANES * u < nrb ? va[u] : 0.0;
        }
#pragma unroll
        for (int o = 1; o < CS_LANES; o <<= 1) a += __shfl_xor(a, o, 64);
        if (t == 0) {
            if (done) {  // (merged: the update in this launch reads it; write-through, then the signal)
                st_sc1(h_out + tot, a);
                // (fn2_fast here: ||f||^2 = ||f'||^2 for the next SpMV if the
                // step skips; a projecting step's update overwrites it after
                // this signal)
                if (fn2_fast) st_sc1(fn2_fast, a);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                h_out[tot] = a;
                if (fn2_fast) *fn2_fast = a;  // ||f||^2 = ||f'||^2 for the next SpMV (the update has nothing to do)
            }
        }
    }
    if (t < GT_SUB + 1) gctr[t * 64] = 0u;  // re-armed (column group 0's counters)
}

// PROI: the step's decision is taken in this launch (ek_internal.hpp
// ProLaunch); a poller's word, 1 + decision (thread 0)
// Dispatch order: every wait here is on a job with a LOWER logical index than
// the waiter (the decider is job 0; the update's jobs follow the whole
// projection).  With tickets (ProLaunch::tix, the default) a logical index is
// handed out only after every lower one of its class, so no wait depends on
// the order the hardware dispatches workgroups in; without them (EK_PRO_TICKETS
// =0) the logical index is blockIdx and the waits rely on index-order
// dispatch whenever the grid outgrows what is resident at once.  Either way
// the waits are bounded, and *err (the
// launch's ProState::timeouts, zero at the start of every solve) doubles as
// an abort word: the first waiter that gives up counts itself there, and
// every other waiter of the launch sees it within 256 polls and gives up too,
// so a broken hand-off costs one bound, not one per workgroup; the host then
// fails the solve with EK_EHIP (ctx.cpp).
__device__ __forceinline__ bool pro_aborted(int* err) {
    return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
__device__ __forceinline__ int pro_poll(const unsigned* pub, int* err) {
    unsigned v = 0u;
    // (bounded: the decider waits on nothing, so this ends in a few us; the
    // bound only keeps a broken hand-off from hanging the GPU)
    for (int it = 0; it < (1 << 22); ++it) {
        v = __hip_atomic_load(pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v != 0u) break;
        if ((it & 255) == 255 && pro_aborted(err)) break;
        __builtin_amdgcn_s_sleep(8);
    }
    if (v == 0u) atomicAdd(err, 1);  // (the host fails the solve)
    return v != 0u ? int(v) : 2;
}
// thread 0: wait until the counter reaches target (bounded like pro_poll);
// 1 when it did
__device__ __forceinline__ int pro_wait(const unsigned* ctr, unsigned target, int* err) {
    for (int it = 0; it < (1 << 22); ++it) {
        if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return 1;
        if ((it & 255) == 255 && pro_aborted(err)) break;
        __builtin_amdgcn_s_sleep(4);
    }
    atomicAdd(err, 1);  // (the host fails the solve)
    return 0;
}

// the merged update's own f' (the projection's formula and operands: it
// does not read the f' the projection stores in the same launch)
struct UpdTT {
    const double* w = nullptr;
    const double* vi = nullptr;
    const double* vim1 = nullptr;
    const double* fn2_i = nullptr;
    const double* bov_i = nullptr;
    const double* apart = nullptr;
    int nparts = 0;
    int* err = nullptr;  // ProState::timeouts
};
template <bool RED, bool B32, bool NT, bool MRG>
__device__ __forceinline__ void update_body(int blk, int ldv, const double* __restrict__ V, int ncols, int has_u0,
                                            double u0val, int nreal, const double* __restrict__ h,
                                            const double* __restrict__ src, double* __restrict__ dst,
                                            double* __restrict__ npart, const double* __restrict__ part, int nrb,
                                            double* __restrict__ h_out, const float* __restrict__ V32,
                                            unsigned* __restrict__ fb, double* __restrict__ fn2_fast,
                                            const unsigned* __restrict__ done, unsigned done_target, UpdTT tt);

template <bool TT, bool NT, int APE, bool PROI, bool MRG = false, bool B32U = false>
__device__ __forceinline__ void gemvt_body(int ldv, int nrb, const double* __restrict__ V, int ncols,
                                               int has_u0, double u0val, int nreal, const double* __restrict__ w,
                                               double* __restrict__ part, const double* __restrict__ alpha,
                                               const double* __restrict__ vi, const double* __restrict__ vim1,
                                               const double* __restrict__ fn2_i, const double* __restrict__ bov_i,
                                               double* __restrict__ fp, int nrm, float* __restrict__ v32col,
                                               const double* __restrict__ apart, int nparts,
                                               double* __restrict__ alpha_pub, unsigned* __restrict__ gctr,
                                               double* __restrict__ h_out, const int* __restrict__ flag,
                                               double* __restrict__ fn2_fast, ProLaunch pl) {
    // every product-sum below is written with explicit FMAs and nothing else
    // is contracted: with contraction left to the compiler, two
    // instantiations of this body (k_gemvt, k_gemvt_pro) fused different
    // products of the same expression, so the paths differed in the last bit
#pragma clang fp contract(off)
    __shared__ double red[4][GT_COLS];
    __shared__ double nred[4];
    __shared__ double lds4[4];
    __shared__ double s_alpha;
    const int t = threadIdx.x;
    const int ncg = (ncols + has_u0 + GT_COLS - 1) / GT_COLS;
    // PROI with pl.cgw: ncgl workgroups per row block walk the ncg groups
    const int ncgl = PROI && pl.cgw > 0 ? min(ncg, pl.cgw) : ncg;
    int nwg = int(gridDim.x), orig = int(blockIdx.x);
    if constexpr (PROI) {
        // The waits below are on jobs of LOWER logical index (the decider is
        // job 0; the update's jobs follow every projection job).  With tickets
        // (pl.tix) the logical index is the workgroup's place among the
        // arrivals of its residue class, so a job is only handed out once every
        // lower job of its class has been handed to a running workgroup: no
        // wait can be on a workgroup that is not yet resident, in any dispatch
        // order.  pl.rev (tests) reverses the physical index first.
        if (pl.rev) orig = nwg - 1 - orig;
        if (pl.tix) {
            __shared__ int s_orig;
            if (t == 0) {
                const unsigned x = unsigned(orig) & 7u, cnt = (unsigned(nwg) - x + 7u) >> 3;
                unsigned* q = pl.tix + PRO_PUB_STRIDE * x;
                const unsigned j = __hip_atomic_fetch_add(q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (j == cnt - 1u) __hip_atomic_store(q, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
                s_orig = int(x + 8u * j);
            }
            __syncthreads();
            orig = s_orig;
        }
    }
    if constexpr (PROI) PRO_STAMP(1);
    if constexpr (PROI) {
        // the decider: the first of 8 extra workgroups ahead of the map (the
        // other seven return; the offset keeps every workgroup's XCD) runs
        // k_pro's body and publishes at once to every XCD's word
        if (orig < 8) {
            PRO_ROLE(orig == 0 ? 1 : 2);
            if (orig == 0) {
                const bool d = pro_decide(apart, pl.wpart, nparts, pl.a3, fn2_i, bov_i, pl.alpha, pl.offd, pl.omega,
                                          pl.st, pl.flags, ncols - 1, pl.seg0, pl.m, pl.thresh, pl.eps1);
                if (t < PRO_PUB)
                    __hip_atomic_store(pl.pub + PRO_PUB_STRIDE * t, d ? 2u : 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                PRO_STAMP(2);
                PRO_DECISION(d ? 2 : 1);
            }
            PRO_STAMP(4);
            return;
        }
        orig -= 8;
        nwg -= 8;
        if constexpr (MRG) {
            // the update's workgroups, after every projection workgroup (so
            // they wait only on workgroups dispatched before them)
            const int nproj = pro_slots(nrb) * ncgl;
            if (orig >= nproj) {
                const int blk = orig - nproj, tot = ncols + has_u0;
                unsigned* done = pl.pub + PRO_PUB_STRIDE * PRO_PUB;
                __shared__ int s_ud;
                PRO_ROLE(5);
                if (t == 0) s_ud = pro_poll(pl.pub + PRO_PUB_STRIDE * (orig % 8), &pl.st->timeouts);
                PRO_STAMP(2);
                __syncthreads();
                if (s_ud == 1) {  // a skipped step: f = f'; ||f||^2 = ||f'||^2 once the norm is in
                    if (blk == 0) {
                        // (B32U: the norm's hand-off wrote ||f||^2 itself,
                        // one round trip sooner; the !B32U update writes NaN
                        // to it at its start, which would race with that)
                        if (t == 0 && !(B32U && EK_PRO_NORM_DIRECT)) {
                            (void)pro_wait(done, 1u, &pl.st->timeouts);
                            PRO_STAMP(3);
                            if (fn2_fast) *fn2_fast = ld_sc1(h_out + tot);
                        }
                        if (t < 2 && ncols - 1 - t >= 0) h_out[ncols - 1 - t] = 0.0;  // (the finalize's h[i], h[i-1])
                    }
                    PRO_STAMP(4);
                    return;
                }
                UpdTT tt;
                tt.w = w;
                tt.vi = vi;
                tt.vim1 = vim1;
                tt.fn2_i = fn2_i;
                tt.bov_i = bov_i;
                tt.apart = apart;
                tt.nparts = nparts;
                tt.err = &pl.st->timeouts;
                update_body<false, B32U, NT, true>(blk, ldv, V, ncols, has_u0, u0val, nreal, h_out, fp, fp, pl.npart,
                                                   nullptr, nrb, nullptr, pl.V32, pl.fb, fn2_fast, done,
                                                   unsigned(ncg + 1), tt);
                PRO_STAMP(4);
                return;
            }
            nwg = nproj;
        }
    }
    int xcd = orig % 8;
    const int q = nwg / 8, rr = nwg % 8;
    // partial reorthogonalisation (k_pro's decision for this step, uniform
    // over the launch): a step that does not project only forms f' and its
    // ||f'||^2 partials (column group 0); the other column groups have no
    // work.  Then the first nrb workgroups — the first dispatched — take the
    // row blocks in order, and the rest return at once
    // PROI: the decision comes from the decider workgroup, so the
    // projecting map is used either way; a column group > 0 waits for it
    // before anything (nothing to do unless the step projects), group 0 forms
    // f' first.  skip is uniform over the workgroup in every form
    bool skip = !PROI && flag && *flag == 0;
    if (skip && orig >= nrb) return;
    int rbk, j0;
    if (PROI && EK_PRO_CG0_FIRST) {
        // column group 0 first: its workgroups form f' and ||f'||^2, the
        // chain a skipped step waits on, so they are dispatched right after
        // the decider instead of spread over the whole projection (the last
        // of them entered ~3 us into the launch: tools/pro_stamps.py,
        // profiles/r05/pro_stamps_*.txt).  Phase p of ncgl holds column group
        // p of every row block; in each phase XCD x takes the same row blocks
        // (its contiguous share of nrb), so the tiles of a row block share an
        // L2 as before.  Slots past an XCD's share are empty.
        const int P1 = pro_slots(nrb), ph = orig / P1, o = orig % P1, idx = o / 8;
        xcd = o % 8;
        const int b8 = nrb / 8, e8 = nrb % 8;
        if (idx >= b8 + (xcd < e8 ? 1 : 0)) return;
        rbk = xcd * b8 + min(xcd, e8) + idx;
        j0 = ph * GT_COLS;
    } else {
        const int v = skip ? orig * ncgl : (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
        rbk = v / ncgl;
        j0 = (v % ncgl) * GT_COLS;
    }
    __shared__ int s_dec;
    if constexpr (PROI) {
        PRO_ROLE(j0 == 0 ? 3 : 4);
        if (j0 != 0) {
            if (t == 0) s_dec = pro_poll(pl.pub + PRO_PUB_STRIDE * xcd, &pl.st->timeouts);
            PRO_STAMP(2);
            __syncthreads();
            if (s_dec == 1) {
                PRO_STAMP(4);
                return;
            }
        }
    }
    // (PROI: the basis tile is loaded after f' is formed, at one place for
    // every column group: two load sites cost the kernel a spill)
    const bool v_first = !PROI && !skip;
    double acc[GT_COLS];
#pragma unroll
    for (int jj = 0; jj < GT_COLS; ++jj) acc[jj] = 0.0;
    const size_t nr = size_t(nreal);
    // every load of the block's tile is issued before the first use (column
    // index clamped to a valid column: no branch around a load, which would
    // make each load wait for the previous one); the arithmetic and its order
    // are unchanged
    constexpr int KR = GT_ROWS / 512;
    const int jmax = ncols > 0 ? ncols - 1 : 0;
    double2 xs[KR], vs[KR][GT_COLS], tv[KR], tu[KR];
    // up to AP_EARLY * 256 alpha partials: their loads go out FIRST (in-order
    // returns: alpha is then reduced while the tile is still in flight);
    // APE 12 up to 3,072 partials, 24 up to 6,144 (the 2x synthetics)
    constexpr int AP_EARLY = APE;
    const bool ap_early = TT && apart && nparts <= AP_EARLY * 256;
    double apv[AP_EARLY];
    if (ap_early) {
#pragma unroll
        for (int u = 0; u < AP_EARLY; ++u) apv[u] = apart[min(t + u * 256, nparts - 1)];
    }
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        const size_t r = size_t(rbk) * GT_ROWS + size_t(k) * 512 + 2 * size_t(t);
        xs[k] = *reinterpret_cast<const double2*>(w + r);
        if constexpr (TT) {
            tv[k] = *reinterpret_cast<const double2*>(vi + r);
            tu[k] = vim1 ? *reinterpret_cast<const double2*>(vim1 + r) : make_double2(0.0, 0.0);
        }
        if (v_first) {
#pragma unroll
            for (int jj = 0; jj < GT_COLS; ++jj)
                vs[k][jj] = ld_basis<NT>(V + size_t(min(j0 + jj, jmax)) * ldv + r);
        }
    }
    if constexpr (TT) {  // k_three_term's f' (same operations, same order)
        // apart != null: alpha = sum of the SpMV's per-block partials, reduced
        // by this workgroup in k_three_term's order (the same bits as the
        // SpMV's last-block reduction); the first workgroup publishes it for
        // the finalize.  Up to 3,072 partials their loads go out ahead of the
        // tile's (ap_early): the wave's loads return in order, so with them
        // behind the tile alpha waited for the whole tile and then for its
        // own round trip (projection 21.9 -> 20.5 us at the headline, rocprof)
        if (apart) {
            double sa = 0.0;  // strided_sum256's order: t, t + 256, ..., then + 0.0 past the end
            if (ap_early) {
#pragma unroll
                for (int u = 0; u < AP_EARLY; ++u) sa += t + u * 256 < nparts ? apv[u] : 0.0;
            } else {
                sa = strided_sum256(apart, nparts);
            }
            sa = block_sum256(sa, lds4);
            if (t == 0) {
                s_alpha = sa;
                if (orig == 0) *alpha_pub = sa;
            }
            __syncthreads();
        }
        const double a = apart ? s_alpha : *alpha;
        const double b = vim1 ? (isnan(*bov_i) ? sqrt(*fn2_i) : *bov_i) : 0.0;
#pragma unroll
        for (int k = 0; k < KR; ++k) {
            double2 y = xs[k];
            y.x = __builtin_fma(-a, tv[k].x, y.x);
            y.y = __builtin_fma(-a, tv[k].y, y.y);
            if (vim1) {
                y.x = __builtin_fma(-b, tu[k].x, y.x);
                y.y = __builtin_fma(-b, tu[k].y, y.y);
            }
            xs[k] = y;
            if (j0 == 0) {
                const size_t r = size_t(rbk) * GT_ROWS + size_t(k) * 512 + 2 * size_t(t);
                // (merged: stored only once the step is known to skip — a
                // projecting step's f is written by the update in this launch)
                if constexpr (!MRG) out_store2(fp + r, y);
                if (v32col) *reinterpret_cast<float2*>(v32col + r) = make_float2(float(tv[k].x), float(tv[k].y));
            }
        }
    }
    if (nrm && j0 == 0) {  // ||rhs||^2 over this row block: a fixed tree (the same in TT and plain forms)
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < KR; ++k) s += __builtin_fma(xs[k].x, xs[k].x, xs[k].y * xs[k].y);
        s = wave_sum(s);
        if ((t & 63) == 0) nred[t >> 6] = s;
    }
    if constexpr (PROI) {
        if (j0 == 0) {
            // ||f'||^2 (both outcomes need it): its hand-off before the decision
            PRO_STAMP(2);
            gemvt_skip_tail(ncols, has_u0, nrb, rbk, t, part, nred, gctr + GT_NORM_CTR, h_out,
                            MRG && !(B32U && EK_PRO_NORM_DIRECT) ? nullptr : fn2_fast, false,
                            MRG ? pl.pub + PRO_PUB_STRIDE * PRO_PUB : nullptr);
            PRO_STAMP(3);
            if (t == 0) s_dec = pro_poll(pl.pub + PRO_PUB_STRIDE * xcd, &pl.st->timeouts);
            __syncthreads();
            skip = s_dec == 1;
            if constexpr (MRG) {
                if (skip) {  // f = f'
#pragma unroll
                    for (int k = 0; k < KR; ++k)
                        out_store2(fp + size_t(rbk) * GT_ROWS + size_t(k) * 512 + 2 * size_t(t), xs[k]);
                }
            }
            if (skip) {
                PRO_STAMP(4);
                return;
            }
        }
    }
    if (skip) {
        gemvt_skip_tail(ncols, has_u0, nrb, rbk, t, part, nred, gctr, h_out, fn2_fast);
        return;
    }
    // the tiles: this workgroup's column groups (one unless PROI walks several)
    const int jstep = ncgl * GT_COLS, jend = PROI ? ncg * GT_COLS : j0 + 1;
    for (int jc = j0; jc < jend; jc += jstep) {
    if (PROI) {
        if (jc != j0) {
            __syncthreads();  // (red and s_last of the previous tile read)
#pragma unroll
            for (int jj = 0; jj < GT_COLS; ++jj) acc[jj] = 0.0;
        }
#pragma unroll
        for (int k = 0; k < KR; ++k) {
            const size_t r = size_t(rbk) * GT_ROWS + size_t(k) * 512 + 2 * size_t(t);
#pragma unroll
            for (int jj = 0; jj < GT_COLS; ++jj) vs[k][jj] = ld_basis<NT>(V + size_t(min(jc + jj, jmax)) * ldv + r);
        }
    }
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        const size_t r = size_t(rbk) * GT_ROWS + size_t(k) * 512 + 2 * size_t(t);
        const double2 x = xs[k];
#pragma unroll
        for (int jj = 0; jj < GT_COLS; ++jj) {
            const int j = jc + jj;
            if (j < ncols) {
                const double2 v = vs[k][jj];
                acc[jj] += __builtin_fma(v.x, x.x, v.y * x.y);
            } else if (has_u0 && j == ncols) {
                acc[jj] = __builtin_fma(u0val, (r < nr ? x.x : 0.0) + (r + 1 < nr ? x.y : 0.0), acc[jj]);
            }
        }
    }
    // wave reduction of the 8 column sums as a reduce-scatter: each xor step
    // halves the values a lane carries (10 shuffles instead of 8 x 6); lane L
    // ends with column 4*b5 + 2*b4 + b3 (bits of L) summed over the wave
    static_assert(GT_COLS == 8, "the reduce-scatter is written for 8 columns");
    const int lane = t & 63;
    double a4[4], a2[2];
    {
        const bool hi = lane & 32;
#pragma unroll
        for (int k = 0; k < 4; ++k) a4[k] = (hi ? acc[k + 4] : acc[k]) + __shfl_xor(hi ? acc[k] : acc[k + 4], 32, 64);
    }
    {
        const bool hi = lane & 16;
#pragma unroll
        for (int k = 0; k < 2; ++k) a2[k] = (hi ? a4[k + 2] : a4[k]) + __shfl_xor(hi ? a4[k] : a4[k + 2], 16, 64);
    }
    double a1;
    {
        const bool hi = lane & 8;
        a1 = (hi ? a2[1] : a2[0]) + __shfl_xor(hi ? a2[0] : a2[1], 8, 64);
    }
    a1 += __shfl_xor(a1, 4, 64);
    a1 += __shfl_xor(a1, 2, 64);
    a1 += __shfl_xor(a1, 1, 64);
    if ((lane & 7) == 0) red[t >> 6][((lane >> 5) & 1) * 4 + ((lane >> 4) & 1) * 2 + ((lane >> 3) & 1)] = a1;
    __syncthreads();
    const int tot = ncols + has_u0;
    if (!h_out) {
        if (t < GT_COLS && jc + t < tot) part[size_t(jc + t) * nrb + rbk] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
        if (nrm && jc == 0 && t == 0) part[size_t(tot) * nrb + rbk] = (nred[0] + nred[1]) + (nred[2] + nred[3]);
        continue;
    }
    // hand-off: every store below is made by wave 0
    __shared__ int s_last;
    if (t < GT_COLS && jc + t < tot) st_sc1(part + size_t(jc + t) * nrb + rbk, (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]));
    if (!PROI && nrm && jc == 0 && t == 0) st_sc1(part + size_t(tot) * nrb + rbk, (nred[0] + nred[1]) + (nred[2] + nred[3]));
    const int cg = jc / GT_COLS;
    unsigned* ctr = gctr + size_t(cg) * (GT_SUB + 1) * 64;
    if (t == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int g = rbk % GT_SUB;
        const unsigned gsize = unsigned((nrb - g + GT_SUB - 1) / GT_SUB), ngroups = unsigned(nrb < GT_SUB ? nrb : GT_SUB);
        int last = 0;
        if (__hip_atomic_fetch_add(ctr + g * 64, 1u, EK_HANDOFF_ORDER, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1u)
            last = __hip_atomic_fetch_add(ctr + GT_SUB * 64, 1u, EK_HANDOFF_ORDER, __HIP_MEMORY_SCOPE_AGENT) ==
                   ngroups - 1u;
        s_last = last;
    }
    __syncthreads();
    if (!s_last) continue;
    // this group's columns (+ ||rhs||^2 in group 0): 8 lanes per column, lane
    // l summing blocks l, l + 8, ... in order (col_sum2's loads and adds), then
    // the xor tree
    const int gq = t / CS_LANES, l = t % CS_LANES;
    const int ncol = min(GT_COLS, tot - jc) + ((nrm && jc == 0 && !PROI) ? 1 : 0);  // (PROI: the norm went before)
    if (gq < ncol) {
        const int j = gq < GT_COLS && jc + gq < tot ? jc + gq : tot;  // (the last group member: the norm column)
        const double* pc = part + size_t(j) * nrb;
        constexpr int CB = 32;
        double a = 0.0;
        for (int b0 = l; b0 < nrb; b0 += CS_LANES * CB) {
            double va[CB];
#pragma unroll
            for (int u = 0; u < CB; ++u) va[u] = ld_sc1(pc + min(b0 + CS_LANES * u, nrb - 1));
#pragma unroll
            for (int u = 0; u < CB; ++u) a += b0 + CS_LANES * u < nrb ? va[u] : 0.0;
        }
#pragma unroll
        for (int o = 1; o < CS_LANES; o <<= 1) a += __shfl_xor(a, o, 64);
        if (l == 0) {
            if constexpr (MRG) st_sc1(h_out + j, a);
            else h_out[j] = a;
        }
    }
    if constexpr (MRG) {  // this column group's h is in: signal the update (every storing wave drained)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0)
            __hip_atomic_fetch_add(pl.pub + PRO_PUB_STRIDE * PRO_PUB, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t < GT_SUB + 1) ctr[t * 64] = 0u;  // re-armed for the next launch (visible at the kernel boundary)
    }  // tiles
    if constexpr (PROI) PRO_STAMP(4);
}

#define EK_GEMVT_PARAMS                                                                                               \
    int ldv, int nrb, const double *__restrict__ V, int ncols, int has_u0, double u0val, int nreal,                  \
        const double *__restrict__ w, double *__restrict__ part, const double *__restrict__ alpha,                   \
        const double *__restrict__ vi, const double *__restrict__ vim1, const double *__restrict__ fn2_i,            \
        const double *__restrict__ bov_i, double *__restrict__ fp, int nrm, float *__restrict__ v32col,              \
        const double *__restrict__ apart, int nparts, double *__restrict__ alpha_pub, unsigned *__restrict__ gctr,   \
        double *__restrict__ h_out, const int *__restrict__ flag, double *__restrict__ fn2_fast, ProLaunch pl
#define EK_GEMVT_ARGS                                                                                                \
    ldv, nrb, V, ncols, has_u0, u0val, nreal, w, part, alpha, vi, vim1, fn2_i, bov_i, fp, nrm, v32col, apart, nparts,  \
        alpha_pub, gctr, h_out, flag, fn2_fast, pl
template <bool TT, bool NT, int APE = 12>
__global__ __launch_bounds__(256) void k_gemvt(EK_GEMVT_PARAMS) {
    gemvt_body<TT, NT, APE, false>(EK_GEMVT_ARGS);
}
// the projection with the in-launch decision (PROI); MRG: + the update's
// workgroups (B32U: its fp32-shadow form)
// (4 waves per SIMD: 128 VGPRs at most, four 256-thread workgroups per CU;
// the tickets took the compiler's own choice to 129)
template <bool NT, int APE, bool MRG, bool B32U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_gemvt_pro(EK_GEMVT_PARAMS) {
    gemvt_body<true, NT, APE, true, MRG, B32U>(EK_GEMVT_ARGS);
}
#undef EK_GEMVT_PARAMS
#undef EK_GEMVT_ARGS

// The sharded step's projection (ctx.cpp Lanczos::factorize_mr): the partial
// dot products of THREE vectors with the same basis columns in one sweep of
// V — w = L v_i, v_i and v_{i-1} — so the three-term coefficient alpha and the
// Gram-Schmidt coefficients of f' = w - alpha v_i - beta v_{i-1} come out of
// ONE all-reduce: V^T f' = V^T w - alpha V^T v_i - beta V^T v_{i-1}, with
// alpha = (V^T w)_i.  part[(k * tot + j) * nrb + b] for vector k (0: w, 1: v_i,
// 2: v_{i-1}), column j < tot = ncols + has_u0 (column ncols = u0), and
// part[3 tot * nrb + b] = ||w||^2 over row block b (k_update_mr's test for a
// cancelled f').  Same tiling, XCD remap and fixed-shape reductions as k_gemvt.
__global__ __launch_bounds__(256) void k_gemvt3(int ldv, int nrb, const double* __restrict__ V, int ncols,
                                                int has_u0, double u0val, int nreal, const double* __restrict__ w,
                                                const double* __restrict__ va, const double* __restrict__ vb,
                                                double* __restrict__ part) {
    __shared__ double red[3][4][GT_COLS];
    __shared__ double nred[4];
    const int t = threadIdx.x;
    const int tot = ncols + has_u0;
    const int ncg = (tot + GT_COLS - 1) / GT_COLS;
    const int nwg = int(gridDim.x), orig = int(blockIdx.x), xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
    const int v = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
    const int rbk = v / ncg, j0 = (v % ncg) * GT_COLS;
    const size_t nr = size_t(nreal);
    constexpr int KR = GT_ROWS / 512;
    const int jmax = ncols > 0 ? ncols - 1 : 0;
    double2 xs[3][KR], vs[KR][GT_COLS];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        const size_t r = size_t(rbk) * GT_ROWS + size_t(k) * 512 + 2 * size_t(t);
        xs[0][k] = *reinterpret_cast<const double2*>(w + r);
        xs[1][k] = *reinterpret_cast<const double2*>(va + r);
        xs[2][k] = *reinterpret_cast<const double2*>(vb + r);
#pragma unroll
        for (int jj = 0; jj < GT_COLS; ++jj)
            vs[k][jj] = *reinterpret_cast<const double2*>(V + size_t(min(j0 + jj, jmax)) * ldv + r);
    }
    double acc[3][GT_COLS];
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int jj = 0; jj < GT_COLS; ++jj) acc[m][jj] = 0.0;
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        const size_t r = size_t(rbk) * GT_ROWS + size_t(k) * 512 + 2 * size_t(t);
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            const double2 x = xs[m][k];
#pragma unroll
            for (int jj = 0; jj < GT_COLS; ++jj) {
                const int j = j0 + jj;
                if (j < ncols) {
                    const double2 vv = vs[k][jj];
                    acc[m][jj] += vv.x * x.x + vv.y * x.y;
                } else if (has_u0 && j == ncols) {
                    acc[m][jj] += u0val * ((r < nr ? x.x : 0.0) + (r + 1 < nr ? x.y : 0.0));
                }
            }
        }
    }
    if (j0 == 0) {  // ||w||^2 over this row block (the same tree as k_gemvt's nrm)
        double s2 = 0.0;
#pragma unroll
        for (int k = 0; k < KR; ++k) s2 += xs[0][k].x * xs[0][k].x + xs[0][k].y * xs[0][k].y;
        s2 = wave_sum(s2);
        if ((t & 63) == 0) nred[t >> 6] = s2;
    }
    // the reduce-scatter of k_gemvt, once per vector
    const int lane = t & 63;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
        double a4[4], a2[2];
        {
            const bool hi = lane & 32;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                a4[k] = (hi ? acc[m][k + 4] : acc[m][k]) + __shfl_xor(hi ? acc[m][k] : acc[m][k + 4], 32, 64);
        }
        {
            const bool hi = lane & 16;
#pragma unroll
            for (int k = 0; k < 2; ++k) a2[k] = (hi ? a4[k + 2] : a4[k]) + __shfl_xor(hi ? a4[k] : a4[k + 2], 16, 64);
        }
        double a1;
        {
            const bool hi = lane & 8;
            a1 = (hi ? a2[1] : a2[0]) + __shfl_xor(hi ? a2[0] : a2[1], 8, 64);
        }
        a1 += __shfl_xor(a1, 4, 64);
        a1 += __shfl_xor(a1, 2, 64);
        a1 += __shfl_xor(a1, 1, 64);
        if ((lane & 7) == 0) red[m][t >> 6][((lane >> 5) & 1) * 4 + ((lane >> 4) & 1) * 2 + ((lane >> 3) & 1)] = a1;
    }
    __syncthreads();
    if (t < 3 * GT_COLS) {
        const int m = t / GT_COLS, c = t % GT_COLS;
        if (j0 + c < tot)
            part[(size_t(m) * tot + size_t(j0 + c)) * nrb + rbk] =
                (red[m][0][c] + red[m][1][c]) + (red[m][2][c] + red[m][3][c]);
    }
    if (j0 == 0 && t == 3 * GT_COLS) part[size_t(3 * tot) * nrb + rbk] = (nred[0] + nred[1]) + (nred[2] + nred[3]);
}

// The canonical order of a column sum over the projection partials: 8 lanes
// per column, lane l summing blocks l, l+8, l+16, ... in order, then a fixed
// xor tree over the 8 lanes (every lane of the group gets the sum).  Used by
// k_reduce_cols and by the fused update alike, so both give the same bits.
// The loads are unconditional (clamped index) and so are the adds (0.0 past
// the end): a load behind a branch waits for the loads before it.  s + 0.0
// == s here because s starts at +0 and a sum of these partials never becomes
// -0.0.  Two columns at a time, all their loads in flight together: one
// round trip for up to 8 * CB row blocks (ibm18 shape: 198).  (Two lanes per
// column, as before, took four dependent round trips and every update
// workgroup ~7.5 us of its 20.)
__device__ __forceinline__ void col_sum2(const double* __restrict__ pa, const double* __restrict__ pb, int nrb, int l,
                                         double* sa, double* sb) {
    constexpr int CB = 32;
    double a = 0.0, b = 0.0;
    for (int b0 = l; b0 < nrb; b0 += CS_LANES * CB) {
        double va[CB], vb[CB];
#pragma unroll
        for (int u = 0; u < CB; ++u) {
            const int i = min(b0 + CS_LANES * u, nrb - 1);
            va[u] = pa[i];
            vb[u] = pb[i];
        }
#pragma unroll
        for (int u = 0; u < CB; ++u) {
            const bool live = b0 + CS_LANES * u < nrb;
            a += live ? va[u] : 0.0;
            b += live ? vb[u] : 0.0;
        }
    }
#pragma unroll
    for (int o = 1; o < CS_LANES; o <<= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
    }
    *sa = a;
    *sb = b;
}

// h[j] = sum_b part[j*nrb + b] for j < ncols, in col_sum2's order (lane l of
// 8 sums blocks l, l+8, ... in turn, then the xor tree: the same bits as the
// update's in-kernel sums).  The partials are staged in LDS by the whole
// workgroup first, every load in flight at once, and the 8-lane chains then
// run from LDS: with the chains reading memory themselves (8 lanes per column,
// 32 loads in flight each) a column of 1,972 row blocks (10x) took 8 dependent
// memory trips, 34.8 us per launch.  RC_COLS columns per workgroup; row-block
// chunks of RC_CHUNK (chunk starts are multiples of 8: the chains carry on).
constexpr int RC_COLS = 2, RC_CHUNK = 2048, RC_LD = RC_CHUNK + 8;  // +8: the two columns' chains on disjoint banks
__global__ __launch_bounds__(256) void k_reduce_cols(const double* __restrict__ part, int nrb, int ncols,
                                                     double* __restrict__ h) {
    __shared__ double st[RC_COLS * RC_LD];
    constexpr int PT = RC_CHUNK / 256;
    const int t = int(threadIdx.x), j0 = int(blockIdx.x) * RC_COLS;
    const int g = t / CS_LANES, l = t % CS_LANES;
    double a = 0.0;
    for (int c0 = 0; c0 < nrb; c0 += RC_CHUNK) {
        const int cn = min(RC_CHUNK, nrb - c0);
        double v[RC_COLS][PT];
#pragma unroll
        for (int q = 0; q < RC_COLS; ++q) {
            const double* src = part + size_t(min(j0 + q, ncols - 1)) * nrb + c0;
#pragma unroll
            for (int u = 0; u < PT; ++u) v[q][u] = src[min(t + 256 * u, cn - 1)];
        }
#pragma unroll
        for (int q = 0; q < RC_COLS; ++q)
#pragma unroll
            for (int u = 0; u < PT; ++u)
                if (t + 256 * u < cn) st[q * RC_LD + t + 256 * u] = v[q][u];
        __syncthreads();
        if (g < RC_COLS) {
            const double* col = st + g * RC_LD;
            int i = l;
            for (; i + 3 * CS_LANES < cn; i += 4 * CS_LANES) {  // four reads in flight, adds in order
                const double x0 = col[i], x1 = col[i + CS_LANES], x2 = col[i + 2 * CS_LANES], x3 = col[i + 3 * CS_LANES];
                a += x0;
                a += x1;
                a += x2;
                a += x3;
            }
            for (; i < cn; i += CS_LANES) a += col[i];
        }
        __syncthreads();
    }
#pragma unroll
    for (int o = 1; o < CS_LANES; o <<= 1) a += __shfl_xor(a, o, 64);
    if (g < RC_COLS && l == 0 && j0 + g < ncols) h[j0 + g] = a;
}

// dst = src - V[:, :ncols] h - u0 h[ncols]; 256 threads x 2 rows (double2).
// RED: h is first reduced from the projection partials (column j: two lanes
// each summing every other block in order, then one add — the same in every
// workgroup; workgroup 0 publishes h_out).
//
// B32: the basis is read from its fp32 shadow V32 (half the bytes) when the
// correction is small enough for that to be exact to fp64 rounding.  With
// unit columns, |V - fl32(V)| <= 2^-24 |V| elementwise, so the shadow changes
// V h by at most 2^-24 sum_j |h_j| in norm; the test sum_j |h_j| <= 2^-29
// ||src|| bounds that by 2^-53 ||src||, below the rounding of the fp64
// update itself.  In a reorthogonalised Lanczos step h is the loss of
// orthogonality, O(eps ||w||), so the test holds by many orders of magnitude;
// when it does not (an injected vector, a residual that cancelled to near
// zero) every workgroup takes the same decision (the same h and norm, the
// same sums) and runs the fp64 loop (*fb counts those launches).
// ||src||^2 comes as one more column of the partials (k_gemvt's nrm) or h.
// MRG: the update inside the projection launch (k_gemvt_pro's last ldv/512
// workgroups, blk = this one's index among them): h and f' come from the
// same launch, so the first basis batches go out, then thread 0 waits for
// *done to reach done_target (every h entry stored write-through), and f'
// and h are read with agent-scope (sc1) loads
template <bool RED, bool B32, bool NT, bool MRG>
__device__ __forceinline__ void update_body(int blk, int ldv, const double* __restrict__ V, int ncols, int has_u0,
                                            double u0val, int nreal, const double* __restrict__ h,
                                            const double* __restrict__ src, double* __restrict__ dst,
                                            double* __restrict__ npart, const double* __restrict__ part, int nrb,
                                            double* __restrict__ h_out, const float* __restrict__ V32,
                                            unsigned* __restrict__ fb, double* __restrict__ fn2_fast,
                                            const unsigned* __restrict__ done, unsigned done_target, UpdTT tt) {
    // explicit FMAs, no contraction: the same bits in every instantiation
    // (the k_update launch and the update inside the projection launch)
#pragma clang fp contract(off)
    if constexpr (!B32) {  // the next SpMV sums this launch's ||f||^2 partials
        if (fn2_fast && blk == 0 && threadIdx.x == 0) *fn2_fast = __builtin_nan("");
    }
    constexpr int UB = EK_UPD_UB;
    constexpr int UB32 = 2 * EK_UPD_UB;  // fp32 columns per batch: the same bytes in flight
    constexpr int UBX = B32 ? UB32 : UB;
    // hc: the basis coefficients, zero past ncols (whole batches read it
    // unconditionally); hu0: the deflation vector's; snrm: ||src||^2 (B32)
    __shared__ double hc[MAX_NCV + 2 * UBX];
    __shared__ double hu0, snrm;
    __shared__ double lds4[4];
    const int tot = ncols + has_u0;
    const int totr = tot + (B32 ? 1 : 0);  // values reduced / read: + ||src||^2
    // Basis columns in batches of UB, two batches in flight: batch b+1's
    // loads are issued before batch b is used, and batch 0's (with src)
    // before h is reduced, so the projection reduce and every batch overlap a
    // round trip.  Clamped column index and unconditional subtractions (a
    // column past ncols is subtracted with coefficient 0): a load or a use
    // behind a branch makes the load wait for the ones before it, and a
    // branch splits the loop into blocks the scheduler hoists the next
    // batch's loads across.  The subtractions keep their sequential order;
    // x - v*0 == x for every x but -0.0, which these sums do not produce (a
    // difference of equal values rounds to +0).
    // The two buffers swap roles in a loop unrolled by two: with a register
    // copy `cur = nxt` (which needs nxt's data) the compiler waited for the
    // next batch at every trip (vmcnt(0) at the back edge), so only one batch
    // was ever in flight: 20.3 us per step at ibm18 shape.
    // (One row per thread with 8-B loads in 512-thread blocks, twice the
    // waves: 28 vs 20 us per step.)
    const int jmax = ncols > 0 ? ncols - 1 : 0;
    const size_t r = (size_t(blk) * 256 + threadIdx.x) * 2;
    auto load_batch = [&](double2* vb, int j0) {
#pragma unroll
        for (int u = 0; u < UB; ++u) vb[u] = ld_basis<NT>(V + size_t(min(j0 + u, jmax)) * ldv + r);
    };
    double2 x = make_double2(0.0, 0.0);
    if constexpr (!MRG) {
        x = *reinterpret_cast<const double2*>(src + r);
    } else {
        // f' = w - alpha v_i - beta v_{i-1} from operands of earlier launches,
        // alpha in the projection's order (strided partials, block tree): the
        // projection's bits.  Before the basis batches go out (registers)
        const double2 ttw = *reinterpret_cast<const double2*>(tt.w + r);
        const double2 ttv = *reinterpret_cast<const double2*>(tt.vi + r);
        const double2 ttu = tt.vim1 ? *reinterpret_cast<const double2*>(tt.vim1 + r) : make_double2(0.0, 0.0);
        __shared__ double s_al;
        const double sa = block_sum256(strided_sum256(tt.apart, tt.nparts), lds4);
        if (threadIdx.x == 0) s_al = sa;
        __syncthreads();
        const double a = s_al;
        const double b = tt.vim1 ? (isnan(*tt.bov_i) ? sqrt(*tt.fn2_i) : *tt.bov_i) : 0.0;
        x = ttw;
        x.x = __builtin_fma(-a, ttv.x, x.x);
        x.y = __builtin_fma(-a, ttv.y, x.y);
        if (tt.vim1) {
            x.x = __builtin_fma(-b, ttu.x, x.x);
            x.y = __builtin_fma(-b, ttu.y, x.y);
        }
    }
    auto consume = [&](const double2* vb, int j0) {
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            const double hj = hc[j0 + u];
            x.x = __builtin_fma(-vb[u].x, hj, x.x);
            x.y = __builtin_fma(-vb[u].y, hj, x.y);
        }
    };
    // past the end: clamped re-reads of column jmax (cache hits), coefficient 0
    // (scheduling barriers keep each batch's loads ahead of the other's use:
    // left alone the scheduler sank them below it)
    auto run64 = [&](double2* ba, double2* bb) {
        for (int j0 = 0; j0 < ncols; j0 += 2 * UB) {
            consume(ba, j0);
            __builtin_amdgcn_sched_barrier(0);
            load_batch(ba, j0 + 2 * UB);
            __builtin_amdgcn_sched_barrier(0);
            consume(bb, j0 + UB);
            __builtin_amdgcn_sched_barrier(0);
            load_batch(bb, j0 + 3 * UB);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // the first two batches are issued before the coefficients are reduced
    // (B32: the shadow's; the fp64 fallback issues its own afterwards)
    double2 ba[UB], bb[UB];
    float2 fa[UB32], fbb[UB32];
    // MRG: the shadow's column i is being written in this launch (the
    // projection's column-group-0 workgroups): the shadow loop stops before
    // it (clamped to column i-1, its coefficient taken as 0 there) and column
    // i is subtracted last as fl32 of the fp64 column — the same value and
    // the same order of operations as the shadow loop over all columns
    constexpr bool COLI = MRG && B32;
    const int jmax32 = COLI ? (ncols > 1 ? ncols - 2 : 0) : jmax;
    auto load32 = [&](float2* vb, int j0) {
#pragma unroll
        for (int u = 0; u < UB32; ++u)
            vb[u] = ld_basis32<NT>(V32 + size_t(min(j0 + u, jmax32)) * ldv + r);
    };
    double2 vi64 = make_double2(0.0, 0.0);
    if constexpr (COLI) vi64 = ld_basis<NT>(V + size_t(jmax) * ldv + r);
    if constexpr (B32) {
        load32(fa, 0);
        load32(fbb, UB32);
    } else {
        load_batch(ba, 0);
        load_batch(bb, UB);
    }
    if constexpr (MRG) {
        if (threadIdx.x == 0) (void)pro_wait(done, done_target, tt.err);
        __syncthreads();
    }
    auto put = [&](int j, double v) {
        if (j < ncols) hc[j] = v;
        else if (j < tot) hu0 = v;
        else snrm = v;
    };
    if constexpr (RED) {
        const int g = int(threadIdx.x) / CS_LANES, l = int(threadIdx.x) % CS_LANES;
        for (int ja = g; ja < totr; ja += 64) {  // lane groups: uniform trip counts
            const int jb = ja + 32;
            double sa, sb;
            col_sum2(part + size_t(ja) * nrb, part + size_t(min(jb, totr - 1)) * nrb, nrb, l, &sa, &sb);
            if (l == 0) {
                put(ja, sa);
                if (blk == 0) h_out[ja] = sa;
                if (jb < totr) {
                    put(jb, sb);
                    if (blk == 0) h_out[jb] = sb;
                }
            }
        }
    } else if constexpr (MRG) {
        for (int j = threadIdx.x; j < totr; j += 256) put(j, ld_sc1(h + j));
    } else {
        for (int j = threadIdx.x; j < totr; j += 256) put(j, h[j]);
    }
    for (int j = ncols + int(threadIdx.x); j < ncols + 2 * UBX; j += 256) hc[j] = 0.0;
    __syncthreads();
    if constexpr (B32) {
        // sum |h_j| per wave, the same order in every wave and workgroup
        // (MAX_NCV <= 128: two values a lane)
        static_assert(MAX_NCV <= 128, "two coefficients per lane");
        const int lane = int(threadIdx.x) & 63;
        double a = (lane < ncols ? fabs(hc[lane]) : 0.0) + (lane + 64 < ncols ? fabs(hc[lane + 64]) : 0.0);
        a = wave_sum(a);
        const bool ok = a <= 0x1p-29 * sqrt(snrm);  // false for NaN
        // ||f||^2 = ||f'||^2 - ||h||^2 - h_u0^2 (f = f' - V h - u0 h_u0 with
        // the columns and u0 orthonormal): the next SpMV reads this one value
        // instead of summing the ||f||^2 partials in every workgroup.  Exact
        // to O(eps ||f'||^2) like the direct sum while ||h||^2 <= 2^-20
        // ||f'||^2 (no cancellation); otherwise (a breakdown) NaN: the SpMV
        // sums the partials
        if (fn2_fast && blk == 0 && threadIdx.x == 0) {
            double q = 0.0;
            for (int j = 0; j < ncols; ++j) q = __builtin_fma(hc[j], hc[j], q);
            if (has_u0) q = __builtin_fma(hu0, hu0, q);
            *fn2_fast = q <= 0x1p-20 * snrm ? snrm - q : __builtin_nan("");
        }
        if (ok) {
            auto consume32 = [&](const float2* vb, int j0) {
#pragma unroll
                for (int u = 0; u < UB32; ++u) {
                    const double hj = hc[j0 + u];
                    x.x = __builtin_fma(-double(vb[u].x), hj, x.x);
                    x.y = __builtin_fma(-double(vb[u].y), hj, x.y);
                }
            };
            double hi = 0.0;
            if constexpr (COLI) {  // (column i's coefficient: 0 inside the loop)
                hi = hc[jmax];
                __syncthreads();
                if (threadIdx.x == 0) hc[jmax] = 0.0;
                __syncthreads();
            }
            const int nloop = COLI ? ncols - 1 : ncols;
            for (int j0 = 0; j0 < nloop; j0 += 2 * UB32) {
                consume32(fa, j0);
                __builtin_amdgcn_sched_barrier(0);
                load32(fa, j0 + 2 * UB32);
                __builtin_amdgcn_sched_barrier(0);
                consume32(fbb, j0 + UB32);
                __builtin_amdgcn_sched_barrier(0);
                load32(fbb, j0 + 3 * UB32);
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (COLI) {
                if (ncols > 0) {
                    x.x = __builtin_fma(-double(float(vi64.x)), hi, x.x);
                    x.y = __builtin_fma(-double(float(vi64.y)), hi, x.y);
                }
            }
        } else {
            if (fb && blk == 0 && threadIdx.x == 0) atomicAdd(fb, 1u);
            load_batch(ba, 0);
            load_batch(bb, UB);
            run64(ba, bb);
        }
    } else {
        run64(ba, bb);
    }
    if (has_u0) {
        const double c = u0val * hu0;
        if (r < size_t(nreal)) x.x -= c;
        if (r + 1 < size_t(nreal)) x.y -= c;
    }
    *reinterpret_cast<double2*>(dst + r) = x;
    if (npart) {
        const double s = block_sum256(__builtin_fma(x.x, x.x, x.y * x.y), lds4);
        if (threadIdx.x == 0) npart[blk] = s;
    }
}

template <bool RED, bool B32, bool NT>
__global__ __launch_bounds__(256) void k_update(int ldv, const double* __restrict__ V, int ncols, int has_u0,
                                                double u0val, int nreal, const double* __restrict__ h,
                                                const double* __restrict__ src, double* __restrict__ dst,
                                                double* __restrict__ npart, const double* __restrict__ part, int nrb,
                                                double* __restrict__ h_out, const float* __restrict__ V32,
                                                unsigned* __restrict__ fb, double* __restrict__ fn2_fast,
                                                const int* __restrict__ flag, unsigned* __restrict__ pub_rearm) {
    // PROI: the projection's decision words, zero again for the next launch
    // (every reader of them has finished: the previous launch)
    if (pub_rearm && blockIdx.x == 0 && threadIdx.x < PRO_PUB) pub_rearm[PRO_PUB_STRIDE * threadIdx.x] = 0u;
    // partial reorthogonalisation: a step k_pro left unprojected keeps f = f'
    // (the projection kernel stored it); ||f||^2 = ||f'||^2 (h[tot]) for the
    // next SpMV
    if (flag && *flag == 0) {  // (the projection's hand-off already wrote it; with k_reduce_cols, here)
        if (fn2_fast && blockIdx.x == 0 && threadIdx.x == 0) *fn2_fast = h[ncols + has_u0];
        // PROI: the projection left h alone; the finalize reads h[i], h[i-1]
        if (pub_rearm && blockIdx.x == 0 && threadIdx.x < 2 && ncols - 1 - int(threadIdx.x) >= 0)
            const_cast<double*>(h)[ncols - 1 - int(threadIdx.x)] = 0.0;
        return;
    }
    update_body<RED, B32, NT, false>(int(blockIdx.x), ldv, V, ncols, has_u0, u0val, nreal, h, src, dst, npart, part,
                                     nrb, h_out, V32, fb, fn2_fast, nullptr, 0u, UpdTT{});
}

// The sharded step's update (after the one all-reduce of k_gemvt3's column
// sums, hall = [V^T w | V^T v_i | V^T v_{i-1}], tot values each):
//   alpha = (V^T w)_i, beta = ||f_{i-1}|| (or the injected override, 0 at i = 0),
//   h = V^T w - alpha V^T v_i - beta V^T v_{i-1}   (the projection of f'),
//   dst = f' - V h - u0 h_u0,  f' = w - alpha v_i - beta v_{i-1},
// with ||dst||^2 partials -> npart, and block 0 publishes the projected
// matrix entries alpha[i] = alpha + h[i], offd[i] = beta + h[i-1] (Spectra's
// H += V^T f correction, as k_finalize_step's three-term form).  f' is formed
// with k_three_term's operation order; the subtractions of V h keep
// k_update's order.
__global__ __launch_bounds__(256) void k_update_mr(int ldv, const double* __restrict__ V, int ncols, int has_u0,
                                                   double u0val, int nreal, const double* __restrict__ hall,
                                                   const double* __restrict__ w, const double* __restrict__ vi,
                                                   const double* __restrict__ vim1, const double* __restrict__ fn2_i,
                                                   const double* __restrict__ bov_i, double* __restrict__ dst,
                                                   double* __restrict__ npart, double* __restrict__ alpha,
                                                   double* __restrict__ offd, double* __restrict__ cflag,
                                                   double cancel) {
    constexpr int UB = EK_UPD_UB;
    __shared__ double hc[MAX_NCV + 2 * UB];
    __shared__ double hu0;
    __shared__ double lds4[4];
    const int tot = ncols + has_u0, i = ncols - 1;
    const int jmax = ncols > 0 ? ncols - 1 : 0;
    const size_t r = (size_t(blockIdx.x) * 256 + threadIdx.x) * 2;
    auto load_batch = [&](double2* vb, int j0) {
#pragma unroll
        for (int u = 0; u < UB; ++u) vb[u] = *reinterpret_cast<const double2*>(V + size_t(min(j0 + u, jmax)) * ldv + r);
    };
    double2 ba[UB], bb[UB];
    const double2 xw = *reinterpret_cast<const double2*>(w + r);
    const double2 xv = *reinterpret_cast<const double2*>(vi + r);
    const double2 xu = vim1 ? *reinterpret_cast<const double2*>(vim1 + r) : make_double2(0.0, 0.0);
    load_batch(ba, 0);
    load_batch(bb, UB);
    const double a = hall[i];
    const double braw = i > 0 ? (isnan(*bov_i) ? sqrt(*fn2_i) : *bov_i) : 0.0;
    const double b = vim1 ? braw : 0.0;
    for (int j = threadIdx.x; j < tot; j += 256) {
        const double hj = (hall[j] - a * hall[tot + j]) - b * hall[2 * tot + j];
        if (j < ncols) hc[j] = hj;
        else hu0 = hj;
    }
    for (int j = ncols + int(threadIdx.x); j < ncols + 2 * UB; j += 256) hc[j] = 0.0;
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        alpha[i] = a + hc[i];
        if (i > 0) offd[i] = braw + hc[i - 1];
        // ||f'||^2 from the same sums (v_i, v_{i-1} unit and orthogonal to
        // rounding): a cancelled f' (||f'||^2 < cancel ||w||^2) leaves the
        // projection of f' by linearity with an error eps ||w|| instead of
        // eps ||f'||, so the host re-projects the next vector (Lanczos::repair)
        const double w2 = hall[3 * tot];
        const double vw = i > 0 ? hall[i - 1] : 0.0, vv = i > 0 ? hall[tot + i - 1] : 0.0;
        const double vn = i > 0 ? hall[2 * tot + i - 1] : 0.0;
        const double f2 = w2 - 2.0 * a * a - 2.0 * b * vw + a * a * hall[tot + i] + b * b * vn + 2.0 * a * b * vv;
        cflag[i] = f2 < cancel * w2 ? 1.0 : 0.0;  // (NaN: 0 — a breakdown is the host's own test)
    }
    double2 x = xw;
    x.x -= a * xv.x;
    x.y -= a * xv.y;
    if (vim1) {
        x.x -= b * xu.x;
        x.y -= b * xu.y;
    }
    auto consume = [&](const double2* vb, int j0) {
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            const double hj = hc[j0 + u];
            x.x -= vb[u].x * hj;
            x.y -= vb[u].y * hj;
        }
    };
    for (int j0 = 0; j0 < ncols; j0 += 2 * UB) {
        consume(ba, j0);
        __builtin_amdgcn_sched_barrier(0);
        load_batch(ba, j0 + 2 * UB);
        __builtin_amdgcn_sched_barrier(0);
        consume(bb, j0 + UB);
        __builtin_amdgcn_sched_barrier(0);
        load_batch(bb, j0 + 3 * UB);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (has_u0) {
        const double c = u0val * hu0;
        if (r < size_t(nreal)) x.x -= c;
        if (r + 1 < size_t(nreal)) x.y -= c;
    }
    *reinterpret_cast<double2*>(dst + r) = x;
    const double s = block_sum256(x.x * x.x + x.y * x.y, lds4);
    if (threadIdx.x == 0) npart[blockIdx.x] = s;
}

// fn2_out = sum(npart); H(step,step) / H(step-1,step) from the projections:
// CGS2 (a3 == null): h1 + h2 of both passes; three-term (a3 != null):
// alpha + h2[step] and beta_step + h2[step-1] (Spectra's H += Vf correction).
__global__ __launch_bounds__(256) void k_finalize_step(const double* __restrict__ npart, int nb,
                                                       double* __restrict__ fn2_out, const double* __restrict__ h1,
                                                       const double* __restrict__ h2, int step,
                                                       double* __restrict__ alpha, double* __restrict__ offd,
                                                       const double* __restrict__ a3, const double* __restrict__ beff_i,
                                                       const double* __restrict__ bov_i) {
    __shared__ double lds4[4];
    double s = strided_sum256(npart, nb);
    s = block_sum256(s, lds4);
    if (threadIdx.x == 0) {
        fn2_out[0] = s;
        if (step >= 0 && a3) {
            alpha[step] = *a3 + h2[step];
            if (step > 0) offd[step] = (isnan(bov_i[0]) ? sqrt(beff_i[0]) : bov_i[0]) + h2[step - 1];
        } else if (step >= 0) {
            alpha[step] = h1[step] + h2[step];
            if (step > 0) offd[step] = h1[step - 1] + h2[step - 1];
        }
    }
}

// out[0] = sum(a[0:n)), out[1] = sum(b[0:n)) in pro_decide's order (the
// sharded partially reorthogonalised step: this rank's alpha and ||w||^2
// from its SpMV partials, all-reduced before k_pro reads them as one partial)
__global__ __launch_bounds__(256) void k_sum_pair(const double* __restrict__ a, const double* __restrict__ b, int n,
                                                  double* __restrict__ out) {
    __shared__ double la[4], lb[4];
    double sa, sb;
    strided_sum256x2(a, b, n, sa, sb);
    sa = wave_sum(sa);
    sb = wave_sum(sb);
    if ((threadIdx.x & 63) == 0) {
        la[threadIdx.x >> 6] = sa;
        lb[threadIdx.x >> 6] = sb;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        out[0] = (la[0] + la[1]) + (la[2] + la[3]);
        out[1] = (lb[0] + lb[1]) + (lb[2] + lb[3]);
    }
}

__global__ __launch_bounds__(256) void k_pro(const double* __restrict__ apart, const double* __restrict__ wpart,
                                             int nparts, double* __restrict__ a3, const double* __restrict__ fn2_i,
                                             const double* __restrict__ bov_i, const double* __restrict__ alpha,
                                             const double* __restrict__ offd, double* __restrict__ omega,
                                             ProState* __restrict__ st, int* __restrict__ flags, int i, int seg0, int m,
                                             double thresh, double eps1) {
    (void)pro_decide(apart, wpart, nparts, a3, fn2_i, bov_i, alpha, offd, omega, st, flags, i, seg0, m, thresh, eps1);
}

// Three-term recurrence f' = w - alpha v_i - beta_i v_{i-1}, alpha = sum of the
// SpMV's per-block partials (nparts > 0: every block reduces them itself, in
// the same fixed order, so no extra launch; nparts == 0: alpha precomputed,
// e.g. all-reduced across ranks).  Block 0 publishes alpha for the finalize.
__global__ __launch_bounds__(256) void k_three_term(const double* __restrict__ apart, int nparts,
                                                    double* __restrict__ alpha_io, const double* __restrict__ w,
                                                    const double* __restrict__ vi, const double* __restrict__ vim1,
                                                    const double* __restrict__ fn2_i, const double* __restrict__ bov_i,
                                                    double* __restrict__ fp, float* __restrict__ v32col) {
#pragma clang fp contract(off)  // (gemvt_body's f', the same FMAs)
    __shared__ double lds4[4];
    __shared__ double s_alpha;
    // TT_ROWS rows per block (2 double2 per thread): fewer blocks re-reduce the
    // alpha partials.  The row loads go out first: they do not depend on
    // alpha and overlap the reduction of its partials.
    constexpr int KR = TT_ROWS / 512;
    double2 x[KR], v[KR], u[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        const size_t r = size_t(blockIdx.x) * TT_ROWS + size_t(k) * 512 + 2 * size_t(threadIdx.x);
        x[k] = *reinterpret_cast<const double2*>(w + r);
        v[k] = *reinterpret_cast<const double2*>(vi + r);
        u[k] = vim1 ? *reinterpret_cast<const double2*>(vim1 + r) : make_double2(0.0, 0.0);
    }
    // beta_i = ||f_i||, or 0 after an injected restart vector (override not NaN)
    const double b = vim1 ? (isnan(*bov_i) ? sqrt(*fn2_i) : *bov_i) : 0.0;
    if (nparts > 0) {
        double s = strided_sum256(apart, nparts);
        s = block_sum256(s, lds4);
        if (threadIdx.x == 0) {
            s_alpha = s;
            if (blockIdx.x == 0) *alpha_io = s;
        }
    } else if (threadIdx.x == 0) {
        s_alpha = *alpha_io;
    }
    __syncthreads();
    const double a = s_alpha;
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        const size_t r = size_t(blockIdx.x) * TT_ROWS + size_t(k) * 512 + 2 * size_t(threadIdx.x);
        double2 y = x[k];
        y.x = __builtin_fma(-a, v[k].x, y.x);
        y.y = __builtin_fma(-a, v[k].y, y.y);
        if (vim1) {
            y.x = __builtin_fma(-b, u[k].x, y.x);
            y.y = __builtin_fma(-b, u[k].y, y.y);
        }
        *reinterpret_cast<double2*>(fp + r) = y;
        if (v32col) *reinterpret_cast<float2*>(v32col + r) = make_float2(float(v[k].x), float(v[k].y));
    }
}

// out[:, j] = sum_{i<m} V[:, i] Q[i, j], j < kk; 1-D grid of (ldv/512) row
// blocks x ceil(kk/8) column groups.  Every column group of a row block reads
// the same m x 512 tile of V: with the blocks dealt round-robin over the 8
// XCDs, the (row block, column group) map gives each XCD a contiguous run of
// row blocks with all their column groups (k_gemvt's remap), so the tile is
// fetched from memory once and re-read from that XCD's L2.  (A 2-D grid ran
// every row block of column group 0 first: at 10x, V = 1.6 GB, the tile came
// from HBM once per column group, 1.34 ms per restart.)
template <int IB>
__global__ __launch_bounds__(256) void k_gemm_vq(int ldv, const double* __restrict__ V, int m,
                                                 const double* __restrict__ Q, int kk, double* __restrict__ out,
                                                 float* __restrict__ out32) {
    constexpr int TJ = 8;
    // coefficient rows past m are zero (the last trip's clamped basis rows
    // are multiplied by 0.0, as before: the same products and sums)
    __shared__ __attribute__((aligned(16))) double qs[MAX_NCV + IB][TJ];
    const int ncg = (kk + TJ - 1) / TJ;
    const int nwg = int(gridDim.x), orig = int(blockIdx.x), xcd = orig % 8, q8 = nwg / 8, rr = nwg % 8;
    const int vb = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + orig / 8;
    const int rbk = vb / ncg, j0 = (vb % ncg) * TJ;
    const int mp = (m + IB - 1) / IB * IB;
    for (int i = threadIdx.x; i < mp * TJ; i += 256) {
        const int row = i / TJ, jj = i % TJ;
        qs[row][jj] = (row < m && j0 + jj < kk) ? Q[size_t(j0 + jj) * m + row] : 0.0;
    }
    __syncthreads();
    const size_t r = (size_t(rbk) * 256 + threadIdx.x) * 2;
    double2 acc[TJ];
#pragma unroll
    for (int jj = 0; jj < TJ; ++jj) acc[jj] = make_double2(0.0, 0.0);
    // IB basis rows' loads in flight per trip (clamped index; the sums keep
    // their order, so IB does not change a bit)
    for (int i0 = 0; i0 < m; i0 += IB) {
        double2 v[IB];
#pragma unroll
        for (int u = 0; u < IB; ++u) v[u] = *reinterpret_cast<const double2*>(V + size_t(min(i0 + u, m - 1)) * ldv + r);
        // (every load of the trip issued before the first product: left
        // alone the scheduler interleaved them, two loads in flight)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < IB; ++u) {
            const double2* qr = reinterpret_cast<const double2*>(&qs[i0 + u][0]);
            double q[TJ];
#pragma unroll
            for (int h = 0; h < TJ / 2; ++h) {
                const double2 qq = qr[h];
                q[2 * h] = qq.x;
                q[2 * h + 1] = qq.y;
            }
#pragma unroll
            for (int jj = 0; jj < TJ; ++jj) {
                acc[jj].x += v[u].x * q[jj];
                acc[jj].y += v[u].y * q[jj];
            }
        }
    }
#pragma unroll
    for (int jj = 0; jj < TJ; ++jj)
        if (j0 + jj < kk) {
            *reinterpret_cast<double2*>(out + size_t(j0 + jj) * ldv + r) = acc[jj];
            if (out32)
                *reinterpret_cast<float2*>(out32 + size_t(j0 + jj) * ldv + r) =
                    make_float2(float(acc[jj].x), float(acc[jj].y));
        }
}

// f = f*sigma + x*hk, per-block sum of f^2
__global__ __launch_bounds__(256) void k_axpby_norm(double* __restrict__ f, double sigma,
                                                    const double* __restrict__ x, double hk,
                                                    double* __restrict__ npart) {
    __shared__ double lds4[4];
    const size_t r = (size_t(blockIdx.x) * 256 + threadIdx.x) * 2;
    double2 a = *reinterpret_cast<const double2*>(f + r);
    const double2 b = *reinterpret_cast<const double2*>(x + r);
    a.x = a.x * sigma + b.x * hk;
    a.y = a.y * sigma + b.y * hk;
    *reinterpret_cast<double2*>(f + r) = a;
    const double s = block_sum256(a.x * a.x + a.y * a.y, lds4);
    if (threadIdx.x == 0) npart[blockIdx.x] = s;
}

// per-block sum (or sum of squares) of x over real rows
__global__ __launch_bounds__(256) void k_sum_partial(const double* __restrict__ x, int nreal,
                                                     double* __restrict__ npart, int squares) {
    __shared__ double lds4[4];
    const size_t r = (size_t(blockIdx.x) * 256 + threadIdx.x) * 2;
    const double2 a = *reinterpret_cast<const double2*>(x + r);
    const double ax = r < size_t(nreal) ? a.x : 0.0, ay = r + 1 < size_t(nreal) ? a.y : 0.0;
    const double s = block_sum256(squares ? ax * ax + ay * ay : ax + ay, lds4);
    if (threadIdx.x == 0) npart[blockIdx.x] = s;
}

// per 512-row block: sum over the real rows of (w[r] - lambda x[r])^2 (the
// final residual, a diagnostic: a fixed tree per block, the blocks summed on
// the host in order)
__global__ __launch_bounds__(256) void k_resid_partial(const double* __restrict__ w, const double* __restrict__ x,
                                                       double lambda, int nreal, double* __restrict__ part) {
    __shared__ double lds4[4];
    const size_t r = (size_t(blockIdx.x) * 256 + threadIdx.x) * 2;
    const double2 a = *reinterpret_cast<const double2*>(w + r);
    const double2 b = *reinterpret_cast<const double2*>(x + r);
    const double tx = r < size_t(nreal) ? a.x - lambda * b.x : 0.0, ty = r + 1 < size_t(nreal) ? a.y - lambda * b.y : 0.0;
    const double s = block_sum256(tx * tx + ty * ty, lds4);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// x[r] -= (*mean_sum) * inv_n on real rows (projection off the constant vector)
__global__ __launch_bounds__(256) void k_sub_mean(double* __restrict__ x, int nreal, const double* __restrict__ sum,
                                                  double inv_n) {
    const size_t r = size_t(blockIdx.x) * 256 + threadIdx.x;
    if (r < size_t(nreal)) x[r] -= (*sum) * inv_n;
}

void gemvt(hipStream_t s, int ldv, int nrb, const double* V, int ncols, int has_u0, double u0val, int nreal,
           const double* w, double* part, int nrm, unsigned* gctr, double* h_out, bool nt) {
    const int cols = ncols + has_u0;
    if (cols <= 0) return;
    const dim3 g(nrb * ((cols + GT_COLS - 1) / GT_COLS));
    if (nt)
        hipLaunchKernelGGL((k_gemvt<false, true>), g, dim3(256), 0, s, ldv, nrb, V, ncols, has_u0, u0val, nreal, w, part,
                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nrm, nullptr, nullptr, 0, nullptr, gctr,
                           h_out, nullptr, nullptr, ProLaunch{});
    else
        hipLaunchKernelGGL((k_gemvt<false, false>), g, dim3(256), 0, s, ldv, nrb, V, ncols, has_u0, u0val, nreal, w, part,
                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nrm, nullptr, nullptr, 0, nullptr, gctr,
                           h_out, nullptr, nullptr, ProLaunch{});
}

int gemvt_pro_grid(int nrb, int ncgl, int ldv, bool merged) {
    return (EK_PRO_CG0_FIRST ? pro_slots(nrb) : nrb) * ncgl + 8 + (merged ? ldv / UPD_ROWS : 0);
}

int gemvt_pro_capacity(bool nt, bool wide, bool merged, bool b32u, int num_cu) {
    int per = 0;
#define EK_PRO_OCC(NT_, APE_, M_, B_)                                                                         \
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&k_gemvt_pro<NT_, APE_, M_, B_>), \
                                                       256, 0)
#define EK_PRO_OCC_NT(APE_)                                     \
    do {                                                        \
        if (nt) {                                               \
            if (!merged) EK_PRO_OCC(true, APE_, false, false);  \
            else if (b32u) EK_PRO_OCC(true, APE_, true, true);  \
            else EK_PRO_OCC(true, APE_, true, false);           \
        } else {                                                \
            if (!merged) EK_PRO_OCC(false, APE_, false, false); \
            else if (b32u) EK_PRO_OCC(false, APE_, true, true); \
            else EK_PRO_OCC(false, APE_, true, false);          \
        }                                                       \
    } while (0)
    if (wide) EK_PRO_OCC_NT(24);
    else EK_PRO_OCC_NT(12);
#undef EK_PRO_OCC_NT
#undef EK_PRO_OCC
    return per * num_cu;
}

void gemvt_tt(hipStream_t s, int ldv, int nrb, const double* V, int ncols, int has_u0, double u0val, int nreal,
              const double* w, const double* alpha, const double* vi, const double* vim1, const double* fn2_i,
              const double* bov_i, double* fp, double* part, float* v32col, const double* apart, int nparts,
              unsigned* gctr, double* h_out, bool nt, const int* flag, double* fn2_fast, const ProLaunch* pl) {
    const int cols = ncols + has_u0;
    const bool mrg = pl && pl->merged;
    const int ncg = (cols + GT_COLS - 1) / GT_COLS, ncgl = pl && pl->cgw > 0 ? std::min(ncg, pl->cgw) : ncg;
    const dim3 g((pl && EK_PRO_CG0_FIRST ? pro_slots(nrb) : nrb) * ncgl + (pl ? 8 : 0) + (mrg ? ldv / UPD_ROWS : 0));
    // pl (PROI): the decision in this launch (8 more workgroups); alpha reduced by every
    // workgroup from apart (required) and published to pl->a3
    ProLaunch pv = pl ? *pl : ProLaunch{};
    if (pv.tix && pv.cap > 0 && int(g.x) <= pv.cap) pv.tix = nullptr;  // the whole grid is resident: order-free
#define EK_GEMVT_TT(KERNEL_)                                                                                           \
    hipLaunchKernelGGL(KERNEL_, g, dim3(256), 0, s, ldv, nrb, V, ncols, has_u0, u0val, nreal,                         \
                       w, part, apart ? nullptr : alpha, vi, vim1, fn2_i, bov_i, fp, (v32col || flag || pl) ? 1 : 0,   \
                       v32col, apart, nparts, apart ? const_cast<double*>(alpha) : nullptr, gctr, h_out, flag,       \
                       fn2_fast, pv)
    const bool wide = apart && nparts > 12 * 256;  // 24 partials a thread (up to 6,144; beyond: strided_sum256)
    if (pl) {
        if (!apart || !pl->pub || !gctr || !h_out) {
            std::fprintf(stderr, "gemvt_tt: the in-launch decision needs the alpha partials and the hand-off\n");
            std::abort();
        }
#define EK_GEMVT_PRO(NT_, APE_)                                                      \
    do {                                                                            \
        if (!mrg) EK_GEMVT_TT((k_gemvt_pro<NT_, APE_, false, false>));              \
        else if (pl->V32) EK_GEMVT_TT((k_gemvt_pro<NT_, APE_, true, true>));        \
        else EK_GEMVT_TT((k_gemvt_pro<NT_, APE_, true, false>));                    \
    } while (0)
        if (nt) {
            if (wide) EK_GEMVT_PRO(true, 24);
            else EK_GEMVT_PRO(true, 12);
        } else {
            if (wide) EK_GEMVT_PRO(false, 24);
            else EK_GEMVT_PRO(false, 12);
        }
#undef EK_GEMVT_PRO
    } else if (nt) {
        if (wide) EK_GEMVT_TT((k_gemvt<true, true, 24>));
        else EK_GEMVT_TT((k_gemvt<true, true, 12>));
    } else {
        if (wide) EK_GEMVT_TT((k_gemvt<true, false, 24>));
        else EK_GEMVT_TT((k_gemvt<true, false, 12>));
    }
#undef EK_GEMVT_TT
}


void gemvt3(hipStream_t s, int ldv, int nrb, const double* V, int ncols, int has_u0, double u0val, int nreal,
            const double* w, const double* va, const double* vb, double* part) {
    const int cols = ncols + has_u0;
    if (cols <= 0) return;
    hipLaunchKernelGGL(k_gemvt3, dim3(nrb * ((cols + GT_COLS - 1) / GT_COLS)), dim3(256), 0, s, ldv, nrb, V, ncols,
                       has_u0, u0val, nreal, w, va, vb, part);
}

void update_mr(hipStream_t s, int ldv, const double* V, int ncols, int has_u0, double u0val, int nreal,
               const double* hall, const double* w, const double* vi, const double* vim1, const double* fn2_i,
               const double* bov_i, double* dst, double* npart, double* alpha, double* offd, double* cflag,
               double cancel) {
    hipLaunchKernelGGL(k_update_mr, dim3(ldv / UPD_ROWS), dim3(256), 0, s, ldv, V, ncols, has_u0, u0val, nreal, hall,
                       w, vi, vim1, fn2_i, bov_i, dst, npart, alpha, offd, cflag, cancel);
}

void reduce_cols(hipStream_t s, const double* part, int nrb, int ncols_total, double* h) {
    if (ncols_total <= 0) return;
    hipLaunchKernelGGL(k_reduce_cols, dim3((ncols_total + RC_COLS - 1) / RC_COLS), dim3(256), 0, s, part, nrb,
                       ncols_total, h);
}

#define EK_UPDATE_LAUNCH(RED, B32, NT, ...) \
    hipLaunchKernelGGL((k_update<RED, B32, NT>), dim3(ldv / UPD_ROWS), dim3(256), 0, s, __VA_ARGS__)
void update(hipStream_t s, int ldv, const double* V, int ncols, int has_u0, double u0val, int nreal,
            const double* h, const double* src, double* dst, double* npart, const float* V32, unsigned* fb,
            double* fn2_fast, bool nt, const int* flag, unsigned* pub_rearm) {
    if (V32 && nt)
        EK_UPDATE_LAUNCH(false, true, true, ldv, V, ncols, has_u0, u0val, nreal, h, src, dst, npart, nullptr, 0, nullptr,
                         V32, fb, fn2_fast, flag, pub_rearm);
    else if (V32)
        EK_UPDATE_LAUNCH(false, true, false, ldv, V, ncols, has_u0, u0val, nreal, h, src, dst, npart, nullptr, 0,
                         nullptr, V32, fb, fn2_fast, flag, pub_rearm);
    else if (nt)
        EK_UPDATE_LAUNCH(false, false, true, ldv, V, ncols, has_u0, u0val, nreal, h, src, dst, npart, nullptr, 0,
                         nullptr, nullptr, nullptr, flag ? fn2_fast : nullptr, flag, pub_rearm);
    else
        EK_UPDATE_LAUNCH(false, false, false, ldv, V, ncols, has_u0, u0val, nreal, h, src, dst, npart, nullptr, 0,
                         nullptr, nullptr, nullptr, flag ? fn2_fast : nullptr, flag, pub_rearm);
}

void update_r(hipStream_t s, int ldv, const double* V, int ncols, int has_u0, double u0val, int nreal,
              const double* part, int nrb, double* h_out, const double* src, double* dst, double* npart,
              const float* V32, unsigned* fb, double* fn2_fast, bool nt) {
    if (V32 && nt)
        EK_UPDATE_LAUNCH(true, true, true, ldv, V, ncols, has_u0, u0val, nreal, nullptr, src, dst, npart, part, nrb,
                         h_out, V32, fb, fn2_fast, nullptr, nullptr);
    else if (V32)
        EK_UPDATE_LAUNCH(true, true, false, ldv, V, ncols, has_u0, u0val, nreal, nullptr, src, dst, npart, part, nrb,
                         h_out, V32, fb, fn2_fast, nullptr, nullptr);
    else if (nt)
        EK_UPDATE_LAUNCH(true, false, true, ldv, V, ncols, has_u0, u0val, nreal, nullptr, src, dst, npart, part, nrb,
                         h_out, nullptr, nullptr, nullptr, nullptr, nullptr);
    else
        EK_UPDATE_LAUNCH(true, false, false, ldv, V, ncols, has_u0, u0val, nreal, nullptr, src, dst, npart, part, nrb,
                         h_out, nullptr, nullptr, nullptr, nullptr, nullptr);
}
#undef EK_UPDATE_LAUNCH

void finalize_step(hipStream_t s, const double* npart, int nb, double* fn2_out, const double* h1, const double* h2,
                   int step, double* alpha, double* offd, const double* a3, const double* fn2_i, const double* bov_i) {
    hipLaunchKernelGGL(k_finalize_step, dim3(1), dim3(256), 0, s, npart, nb, fn2_out, h1, h2, step, alpha, offd, a3,
                       fn2_i, bov_i);
}

void pro_step(hipStream_t s, const double* apart, const double* wpart, int nparts, double* a3, const double* fn2_i,
              const double* bov_i, const double* alpha, const double* offd, double* omega, ProState* st, int* flags,
              int i, int seg0, int m, double thresh, double eps1) {
    hipLaunchKernelGGL(k_pro, dim3(1), dim3(256), 0, s, apart, wpart, nparts, a3, fn2_i, bov_i, alpha, offd, omega, st,
                       flags, i, seg0, m, thresh, eps1);
}

// The mid-cycle convergence check's operands in ONE launch straight into the
// host's pinned slot (device-accessible host memory): alpha[0:b), offd[0:b),
// fn2[0:b) (and the sharded step's cancellation flags) at the slot's m-based
// offsets — instead of one DMA blit per array
__global__ __launch_bounds__(256) void k_chk_gather(const double* __restrict__ alpha, const double* __restrict__ offd,
                                                    const double* __restrict__ fn2, const double* __restrict__ flags,
                                                    int b, int bf, int m, size_t flags_off,
                                                    double* __restrict__ dst, unsigned* __restrict__ done,
                                                    unsigned seq) {
    for (int i = int(threadIdx.x); i < bf; i += 256) {
        if (i < b) {
            dst[i] = alpha[i];
            dst[m + i] = offd[i];
            if (flags) dst[flags_off + size_t(i)] = flags[i];
        }
        dst[2 * m + i] = fn2[i];
    }
    if (done) {
        // the completion word the host polls instead of an event: every
        // thread's stores to the pinned slot complete and are released to
        // the system (vmcnt(0) + the system-scope fence) before the barrier,
        // then one system-scope store of the sequence number
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

void chk_gather(hipStream_t s, const double* alpha, const double* offd, const double* fn2, const double* flags, int b,
                int m, size_t flags_off, double* dst, int bf, unsigned* done, unsigned seq) {
    hipLaunchKernelGGL(k_chk_gather, dim3(1), dim3(256), 0, s, alpha, offd, fn2, flags, b, bf < 0 ? b : bf, m,
                       flags_off, dst, done, seq);
}

// The implicit restart's uploads in ONE launch straight from the host's
// pinned staging (device-accessible host memory, like k_chk_gather's slot):
// Q, the kept projected matrix for k_pro's omega recurrence (alpha[0:na) =
// kp[0:na), offd[1:na) = kp[na+1:2na)) and the next cycle's beta overrides
// reset (all-ones bits: the NaN hipMemsetAsync(0xFF) wrote) — instead of three
// DMA blits and a fill, ~4 us each at these sizes
__global__ __launch_bounds__(256) void k_restart_upload(const double* __restrict__ q_src, int nq, double* __restrict__ qd,
                                                        const double* __restrict__ kp, int na, double* __restrict__ alpha,
                                                        double* __restrict__ offd, double* __restrict__ bov, int nbov) {
    const int t = int(blockIdx.x * 256 + threadIdx.x), stride = int(gridDim.x * 256);
    for (int i = t; i < nq; i += stride) qd[i] = q_src[i];
    if (kp) {
        for (int i = t; i < na; i += stride) alpha[i] = kp[i];
        for (int i = t + 1; i < na; i += stride) offd[i] = kp[na + i];
    }
    for (int i = t; i < nbov; i += stride) bov[i] = __longlong_as_double(-1ll);
}

void restart_upload(hipStream_t s, const double* q_src, int nq, double* qd, const double* kp, int na, double* alpha,
                    double* offd, double* bov, int nbov) {
    const int nb = std::max(1, std::min(32, (std::max(nq, nbov) + 255) / 256));
    hipLaunchKernelGGL(k_restart_upload, dim3(nb), dim3(256), 0, s, q_src, nq, qd, kp, na, alpha, offd, bov, nbov);
}

void sum_pair(hipStream_t s, const double* a, const double* b, int n, double* out) {
    hipLaunchKernelGGL(k_sum_pair, dim3(1), dim3(256), 0, s, a, b, n, out);
}

void three_term(hipStream_t s, int ldv, const double* apart, int nparts, double* alpha_io, const double* w,
                const double* vi, const double* vim1, const double* fn2_i, const double* bov_i, double* fp,
                float* v32col) {
    hipLaunchKernelGGL(k_three_term, dim3(ldv / TT_ROWS), dim3(256), 0, s, apart, nparts, alpha_io, w, vi, vim1, fn2_i,
                       bov_i, fp, v32col);
}

// The breakdown restart vector (ctx.cpp inject): element g of the global
// sequence st_{g} = st0 * 48271^(g+1) mod (2^31 - 1), as double(st) / p - 0.5
// — the host loop's values, each lane jumping ahead by square-and-multiply
// (operands < 2^31, so every product fits 64 bits).  Padding rows get 0.
__global__ __launch_bounds__(256) void k_inject(double* __restrict__ f, int ldv, long long row0, long long nrows,
                                                unsigned long long st0) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= ldv) return;
    if (i >= nrows) {
        f[i] = 0.0;
        return;
    }
    constexpr unsigned long long P = 2147483647ull;
    unsigned long long e = (unsigned long long)(row0 + i) + 1ull, b = 48271ull, pw = 1ull;
    while (e) {
        if (e & 1ull) pw = pw * b % P;
        b = b * b % P;
        e >>= 1;
    }
    const unsigned long long st = st0 * pw % P;
    f[i] = double(st) / 2147483647.0 - 0.5;
}

// V[r, j] = 0 for the padded rows r in [nreal, ldv) of the first ncols columns:
// what the basis needs at a solve's start (no kernel writes a padded row
// with anything but 0 afterwards), instead of clearing the whole buffers
__global__ __launch_bounds__(256) void k_zero_pad(double* __restrict__ V, int ldv, int nreal, int ncols) {
    const int pad = ldv - nreal;
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long long)pad * ncols) return;
    const int j = int(i / pad), r = nreal + int(i % pad);
    V[size_t(j) * ldv + r] = 0.0;
}

void zero_pad_rows(hipStream_t s, double* V, int ldv, int nreal, int ncols) {
    const long long tot = (long long)(ldv - nreal) * ncols;
    if (tot > 0) hipLaunchKernelGGL(k_zero_pad, dim3(unsigned((tot + 255) / 256)), dim3(256), 0, s, V, ldv, nreal, ncols);
}

void inject_random(hipStream_t s, double* f, int ldv, long long row0, long long nrows, unsigned long long st0) {
    hipLaunchKernelGGL(k_inject, dim3((ldv + 255) / 256), dim3(256), 0, s, f, ldv, row0, nrows, st0);
}

void gemm_vq(hipStream_t s, int ldv, const double* V, int m, const double* Q, int kk, double* out, float* out32) {
    static const int ib = [] {
        const char* e = std::getenv("EK_VQ_IB");
        return e && e[0] ? std::atoi(e) : 16;
    }();
    const dim3 g((ldv / UPD_ROWS) * ((kk + 7) / 8));
    if (ib >= 32) hipLaunchKernelGGL(k_gemm_vq<32>, g, dim3(256), 0, s, ldv, V, m, Q, kk, out, out32);
    else if (ib >= 16) hipLaunchKernelGGL(k_gemm_vq<16>, g, dim3(256), 0, s, ldv, V, m, Q, kk, out, out32);
    else hipLaunchKernelGGL(k_gemm_vq<8>, g, dim3(256), 0, s, ldv, V, m, Q, kk, out, out32);
}

void axpby_norm(hipStream_t s, int ldv, double* f, double sigma, const double* x, double hk, double* npart) {
    hipLaunchKernelGGL(k_axpby_norm, dim3(ldv / UPD_ROWS), dim3(256), 0, s, f, sigma, x, hk, npart);
}

// Lanczos start vector: x[r] = st_{row0+r+1} / (2^31 - 1) - 0.5 for the
// Park-Miller sequence st_k = 16807^k mod (2^31 - 1) (Spectra SimpleRandom's
// range), 0 on padded rows.  Each element by square-and-multiply: exact
// integers, so the same doubles as the sequential host loop.
__global__ __launch_bounds__(256) void k_start_vector(double* __restrict__ x, int ldv, long long row0, int nreal) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= ldv) return;
    double v = 0.0;
    if (r < nreal) {
        constexpr unsigned long long P = 2147483647ull;
        unsigned long long e = (unsigned long long)(row0 + r + 1), b = 16807ull, st = 1ull;
        while (e) {
            if (e & 1ull) st = (st * b) % P;
            b = (b * b) % P;
            e >>= 1;
        }
        v = double(st) / 2147483647.0 - 0.5;
    }
    x[r] = v;
}

void start_vector(hipStream_t s, int ldv, long long row0, int nreal, double* x) {
    hipLaunchKernelGGL(k_start_vector, dim3((ldv + 255) / 256), dim3(256), 0, s, x, ldv, row0, nreal);
}

void resid_partial(hipStream_t s, int ldv, const double* w, const double* x, double lambda, int nreal, double* part) {
    hipLaunchKernelGGL(k_resid_partial, dim3(ldv / UPD_ROWS), dim3(256), 0, s, w, x, lambda, nreal, part);
}

void sum_partial(hipStream_t s, int ldv, const double* x, int nreal, double* npart, int squares) {
    hipLaunchKernelGGL(k_sum_partial, dim3(ldv / UPD_ROWS), dim3(256), 0, s, x, nreal, npart, squares);
}

void scale_sub_mean(hipStream_t s, int ldv, double* x, int nreal, const double* mean_sum, double inv_n) {
    hipLaunchKernelGGL(k_sub_mean, dim3(ldv / 256), dim3(256), 0, s, x, nreal, mean_sum, inv_n);
}

}  // namespace dev
}  // namespace ek

#ifdef EK_PRO_STAMPS
// lab (tools/pro_stamps.py): the stamp table, [step - 20][workgroup][6] u64
extern "C" int ek_lab_pro_stamps(unsigned long long* out, long long count) {
    const long long cap = (long long)(sizeof(ek::dev::g_pro_stamps) / sizeof(unsigned long long));
    if (count > cap) count = cap;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(ek::dev::g_pro_stamps), size_t(count) * 8, 0, hipMemcpyDeviceToHost) ==
                   hipSuccess
               ? int(count)
               : -1;
}
#endif
