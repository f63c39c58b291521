// Column-panel SpMV for Laplacians whose x does not fit an XCD's L2
// (SparseSymMatProd::perform_op, cEIG.cpp:194, at the 2x / 10x synthetic
// sizes of SURVEY §8d configs 4-5).
//
// Why: the CSR-adaptive kernel (kernels_spmv.hip) gathers x[col] for every
// entry.  With x = 16 MB (10x) each XCD's 4 MB L2 keeps a quarter of it, so
// most 8-byte gathers fetch a whole line from the MALL: rocprofv3 measured
// 1.20 GB of memory-side traffic per 197 MB (algorithmic) launch, 165 us.
//
// Layout: the columns are cut into P panels of 2^pb columns (1 MB of x); a
// persistent grid of G workgroups each owns a contiguous row range with an
// equal share of the entries (<= 8,192 rows), and its entries are stored
// bucketed by panel — bucket (w, p) holds workgroup w's entries whose column
// lies in panel p, in (row, column) order — as a 32-bit word
// (code << pb) | (column within the panel) plus a 16-bit row index relative
// to the workgroup's first row.  Every workgroup walks the panels in the same
// order, so at any moment the XCD's workgroups gather from one or two 1-MB
// panels that stay in its L2: each XCD fetches each line of x about once per
// launch instead of once per entry.
//
// Sums: each row's products are added strictly in ascending column order
// into a +0.0-initialised fp64 accumulator in LDS (the first lane of the
// row's run in a chunk adds the run sequentially; runs of one row in later
// chunks and panels follow after a barrier), so y[r] is the left-to-right
// sequential sum over the row — deterministic, independent of the grid, the
// panel width and the shard map (sharded columns are remapped monotonically).
// The fused Lanczos prologue/epilogue (||f||^2 from the previous step's
// partials, y scaled, the basis column and the alpha partials) is the
// adaptive kernel's.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "ek_internal.hpp"

namespace ek {
namespace dev {

namespace {

constexpr int PT = 256;       // threads per workgroup
constexpr int PCH = 4 * PT;   // entries per chunk (4 per thread)

// thread-strided partial of npart (the adaptive kernel's strided_sum order)
__device__ __forceinline__ double panel_strided_sum(const double* __restrict__ x, int n, int stride) {
    double s = 0.0;
    for (int i0 = threadIdx.x; i0 < n; i0 += 4 * PT) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = i0 + u * PT < n ? x[size_t(i0 + u * PT) * size_t(stride)] : 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i0 + u * PT < n) s += v[u];
    }
    return s;
}

__device__ __forceinline__ double panel_block_sum(double s, double* wsum) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
    __syncthreads();
    const double r = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
    __syncthreads();
    return r;
}

__device__ __forceinline__ void panel_store_sc1(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), static_cast<unsigned long long>(__double_as_longlong(v)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double panel_load_sc1(const double* p) {
    return __longlong_as_double(static_cast<long long>(__hip_atomic_load(
        reinterpret_cast<unsigned long long*>(const_cast<double*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}

// bucket sizes: cnt[w * P + p] = entries of workgroup w in panel p
__global__ __launch_bounds__(PT) void k_panel_count(const int32_t* __restrict__ rowptr,
                                                    const uint32_t* __restrict__ pk, int colbits,
                                                    const int32_t* __restrict__ wrow, int pb, int P,
                                                    int* __restrict__ cnt) {
    __shared__ int c[MAX_PANELS];
    const int w = blockIdx.x;
    for (int p = threadIdx.x; p < P; p += PT) c[p] = 0;
    __syncthreads();
    const uint32_t cmask = (1u << colbits) - 1u;
    const int e0 = rowptr[wrow[w]], e1 = rowptr[wrow[w + 1]];
    for (int e = e0 + int(threadIdx.x); e < e1; e += PT) atomicAdd(&c[int((pk[e] & cmask) >> pb)], 1);
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += PT) cnt[w * P + p] = c[p];
}

// the buckets, in (row, column) order within each: a stable multi-split of
// the workgroup's CSR entries by panel, chunk by chunk (per-wave ballots for
// the rank among the chunk's entries of the same panel)
__global__ __launch_bounds__(PT) void k_panel_fill(const int32_t* __restrict__ rowptr,
                                                   const uint32_t* __restrict__ pk, int colbits,
                                                   const int32_t* __restrict__ wrow, int pb, int P,
                                                   const long long* __restrict__ start, uint32_t* __restrict__ word,
                                                   uint16_t* __restrict__ rid) {
    __shared__ long long cur[MAX_PANELS];
    __shared__ int wtot[PT / 64][MAX_PANELS];
    const int w = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (int p = t; p < P; p += PT) cur[p] = start[w * P + p];
    const int r0 = wrow[w], r1 = wrow[w + 1];
    const int e0 = rowptr[r0], e1 = rowptr[r1];
    const uint32_t cmask = (1u << colbits) - 1u, pmask = (1u << pb) - 1u;
    const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
    __syncthreads();
    for (int base = e0; base < e1; base += PT) {
        const int e = base + t;
        const bool valid = e < e1;
        const uint32_t wd = valid ? pk[e] : 0u;
        const uint32_t col = wd & cmask;
        const int p = valid ? int(col >> pb) : -1;
        int row = 0;
        if (valid) {  // the entry's row: last r in [r0, r1) with rowptr[r] <= e
            int lo = r0, hi = r1 - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (rowptr[mid] <= e) lo = mid;
                else hi = mid - 1;
            }
            row = lo;
        }
        int rank = 0;
        for (int q = 0; q < P; ++q) {
            const unsigned long long m = __ballot(p == q);
            if (p == q) rank = __popcll(m & below);
            if (lane == 0) wtot[wv][q] = __popcll(m);
        }
        __syncthreads();
        if (valid) {
            for (int v = 0; v < wv; ++v) rank += wtot[v][p];
            const long long pos = cur[p] + rank;
            word[pos] = ((wd >> colbits) << pb) | (col & pmask);
            rid[pos] = uint16_t(row - r0);
        }
        __syncthreads();
        for (int q = t; q < P; q += PT) {
            int s = 0;
            for (int v = 0; v < PT / 64; ++v) s += wtot[v][q];
            cur[q] += s;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(PT) void k_spmv_panel(SpmvPanel m, const double* __restrict__ dict,
                                                   const double* __restrict__ x, double* __restrict__ y,
                                                   const double* __restrict__ fn2, const double* __restrict__ f,
                                                   double* __restrict__ vcol, double* __restrict__ apart, StepFin fin,
                                                   double* __restrict__ alpha_out, unsigned* __restrict__ actr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* prod = reinterpret_cast<double*>(smem);      // [PCH]
    double* acc = prod + PCH;                            // [max_rows]
    uint16_t* rl = reinterpret_cast<uint16_t*>(acc + m.max_rows);  // [PCH]
    __shared__ double wsum[PT / 64];
    __shared__ long long bst[MAX_PANELS + 1];
    __shared__ int s_last;
    const int w = blockIdx.x, t = threadIdx.x;
    const int r0 = m.wrow[w], nr = m.wrow[w + 1] - r0;
    const int P = m.P, pb = m.pb;
    const uint32_t pmask = (1u << pb) - 1u;
    for (int p = t; p <= P; p += PT) bst[p] = m.start[size_t(w) * P + p];
    for (int r = t; r < nr; r += PT) acc[r] = 0.0;
    // ||f||^2 of the previous step (its partials' loads go out first)
    const double npart_t = fin.npart ? panel_strided_sum(fin.npart, fin.nb, fin.nstride) : 0.0;
    __syncthreads();
    for (int p = 0; p < P; ++p) {
        const long long b1 = bst[p + 1];
        const double* xp = x + (size_t(p) << pb);
        for (long long c0 = bst[p]; c0 < b1; c0 += PCH) {
            const int cnt = int(min((long long)PCH, b1 - c0));
            uint32_t wd[4];
            uint16_t rr[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = t + u * PT;
                wd[u] = i < cnt ? m.word[c0 + i] : 0u;
                rr[u] = i < cnt ? m.rid[c0 + i] : uint16_t(0);
            }
            double xv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) xv[u] = xp[wd[u] & pmask];  // word 0 past cnt: a valid address
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = t + u * PT;
                if (i < cnt) {
                    prod[i] = dict[wd[u] >> pb] * xv[u];
                    rl[i] = rr[u];
                }
            }
            __syncthreads();
            // the first entry of each row's run adds the run in order
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = t + u * PT;
                if (i < cnt && (i == 0 || rl[i - 1] != rr[u])) {
                    const int r = rr[u];
                    double s = acc[r];
                    int j = i;
                    do {
                        s += prod[j];
                        ++j;
                    } while (j < cnt && rl[j] == rr[u]);
                    acc[r] = s;
                }
            }
            __syncthreads();
        }
    }
    double n2 = fn2 ? *fn2 : 1.0;
    if (fin.npart) {
        n2 = panel_block_sum(npart_t, wsum);
        if (w == 0 && t == 0) {
            fin.fn2_out[0] = n2;
            if (fin.step >= 0) {
                fin.alpha[fin.step] = *fin.a3 + fin.h2[fin.step];
                if (fin.step > 0)
                    fin.offd[fin.step] = (isnan(fin.bov_i[0]) ? sqrt(fin.fn2_i[0]) : fin.bov_i[0]) + fin.h2[fin.step - 1];
            }
        }
    }
    const double scale = (fn2 || fin.npart) ? (n2 > 0.0 ? 1.0 / sqrt(n2) : 0.0) : 1.0;
    double av = 0.0;
    for (int r = t; r < nr; r += PT) {
        const double yr = acc[r] * scale;
        y[r0 + r] = yr;
        if (vcol) {
            const double v = f[r0 + r] * scale;
            vcol[r0 + r] = v;
            av += v * yr;
        }
    }
    if (apart) {
        const double s = panel_block_sum(av, wsum);
        if (t == 0) panel_store_sc1(apart + w, s);
    }
    if (alpha_out) {  // kernels_spmv.hip alpha_handoff: the last workgroup reduces alpha
        if (t == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned old = __hip_atomic_fetch_add(actr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = old == gridDim.x - 1u ? 1 : 0;
        }
        __syncthreads();
        if (s_last) {
            double s = 0.0;
            for (int i = t; i < int(gridDim.x); i += PT) s += panel_load_sc1(apart + i);
            s = panel_block_sum(s, wsum);
            if (t == 0) {
                *alpha_out = s;
                *actr = 0u;
            }
        }
    }
}

}  // namespace

size_t panel_lds_bytes(int max_rows) { return size_t(PCH) * 8 + size_t(max_rows) * 8 + size_t(PCH) * 2; }

void panel_count(hipStream_t s, int G, const int32_t* rowptr, const uint32_t* pk, int colbits, const int32_t* wrow,
                 int pb, int P, int* cnt) {
    hipLaunchKernelGGL(k_panel_count, dim3(G), dim3(PT), 0, s, rowptr, pk, colbits, wrow, pb, P, cnt);
}

void panel_fill(hipStream_t s, int G, const int32_t* rowptr, const uint32_t* pk, int colbits, const int32_t* wrow,
                int pb, int P, const long long* start, uint32_t* word, uint16_t* rid) {
    hipLaunchKernelGGL(k_panel_fill, dim3(G), dim3(PT), 0, s, rowptr, pk, colbits, wrow, pb, P, start, word, rid);
}

void spmv_panel(hipStream_t s, const SpmvPanel& m, const double* dict, const double* x, double* y, const double* fn2,
                const double* f, double* vcol, double* apart, const StepFin* fin, hipEvent_t ev_start,
                hipEvent_t ev_stop, double* alpha_out, unsigned* actr) {
    const StepFin fv = fin ? *fin : StepFin{};
    hipExtLaunchKernelGGL(k_spmv_panel, dim3(m.G), dim3(PT), panel_lds_bytes(m.max_rows), s, ev_start, ev_stop, 0, m,
                          dict, x, y, fn2, f, vcol, apart, fv, alpha_out, actr);
}

}  // namespace dev
}  // namespace ek
