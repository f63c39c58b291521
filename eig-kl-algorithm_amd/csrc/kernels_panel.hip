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

#include "ek_device.hpp"
#include "ek_internal.hpp"

namespace ek {
namespace dev {

namespace {

constexpr int PT = 256;       // threads per workgroup
#ifndef EK_PANEL_DEPTH
#define EK_PANEL_DEPTH 2  // chunks in flight: 2 = chunk k+1's gathers issued before chunk k's LDS phase
#endif
#ifndef EK_PANEL_PER
#define EK_PANEL_PER 2
#endif
constexpr int PER = EK_PANEL_PER;  // entries per thread per chunk
constexpr int PCH = PER * PT;  // entries per chunk

// thread-strided partial of npart (the adaptive kernel's strided_sum order)
__device__ __forceinline__ double panel_strided_sum(const double* __restrict__ x, int n, int stride,
                                                    const int* __restrict__ idx = nullptr) {
    double s = 0.0;
    for (int i0 = threadIdx.x; i0 < n; i0 += 4 * PT) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            v[u] = i0 + u * PT < n ? x[idx ? size_t(idx[i0 + u * PT]) : size_t(i0 + u * PT) * size_t(stride)] : 0.0;
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

template <bool LDICT>
__global__ __launch_bounds__(PT) void k_spmv_panel(SpmvPanel m, const double* __restrict__ dict,
                                                   const double* __restrict__ x, double* __restrict__ y,
                                                   const double* __restrict__ fn2, const double* __restrict__ f,
                                                   double* __restrict__ vcol, double* __restrict__ apart, StepFin fin,
                                                   double* __restrict__ alpha_out, unsigned* __restrict__ actr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* prod = reinterpret_cast<double*>(smem);  // [2][PCH] (double-buffered chunks)
    double* acc = prod + 2 * PCH;                    // [max_rows]
    uint16_t* rl = reinterpret_cast<uint16_t*>(acc + m.max_rows);  // [2][PCH]
    __shared__ double wsum[PT / 64];
    __shared__ long long bst[MAX_PANELS + 1];
    __shared__ int s_last;
    const int w = blockIdx.x, t = threadIdx.x;
    if (fin.pub_rearm && w == 0 && t < PRO_PUB_WORDS) fin.pub_rearm[PRO_PUB_STRIDE * t] = 0u;
    const int r0 = m.wrow[w], nr = m.wrow[w + 1] - r0;
    // the value table in LDS when it fits (PANEL_LDS_DICT entries): the
    // per-entry lookup is then an LDS read instead of a second global gather
    double* sdict = reinterpret_cast<double*>(rl + 2 * PCH);
    if constexpr (LDICT)
        for (int i = t; i < m.ndict; i += PT) sdict[i] = dict[i];
    const int P = m.P, pb = m.pb;
    const uint32_t pmask = (1u << pb) - 1u;
    for (int p = t; p <= P; p += PT) bst[p] = m.start[size_t(w) * P + p];
    for (int r = t; r < nr; r += PT) acc[r] = 0.0;
    // ||f||^2 of the previous step: the update's ||f'||^2 - ||h||^2 (fin.fast)
    // or, when that is NaN (a breakdown), the partials, whose loads go out first
    const double fastv = fin.fast ? *fin.fast : __builtin_nan("");
    const bool sum_parts = fin.npart && isnan(fastv);  // (uniform over the workgroup)
    const double npart_t = sum_parts ? panel_strided_sum(fin.npart, fin.nb, fin.nstride, fin.nidx) : 0.0;
    __syncthreads();
    // The workgroup's chunks, panel by panel (every workgroup walks the panels
    // in the same order).  The next chunk's words and row indices are loaded
    // while this chunk's gathers are in flight; the LDS staging alternates
    // between two buffers, so one barrier per chunk orders both the staging
    // and the accumulators (a row's runs in consecutive chunks are added
    // after that barrier, in chunk order).
    // Software pipeline, two chunks deep: chunk k+1's gathers of x and of the
    // value table go out before chunk k's products are staged, and chunk
    // k+2's words and row indices before those, so a chunk's dependent
    // gathers overlap the previous chunk's LDS phase.
    auto advance = [&](int& pp, long long& cc) {  // to the next non-empty chunk (pp == P: done)
        while (pp < P && cc >= bst[pp + 1]) {
            ++pp;
            if (pp < P) cc = bst[pp];
        }
    };
    auto chunk_cnt = [&](int pp, long long cc) { return pp < P ? int(min((long long)PCH, bst[pp + 1] - cc)) : 0; };
    auto load_words = [&](int pp, long long cc, uint32_t* wd, uint16_t* rr) {
        const int cnt = chunk_cnt(pp, cc);
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = t + u * PT;
            wd[u] = i < cnt ? m.word[cc + i] : 0u;
            rr[u] = i < cnt ? m.rid[cc + i] : uint16_t(0xffff);  // 0xffff: no entry
        }
    };
    const int olo = fin.own_lo, ohi = fin.own_hi;  // (the halo SpMV: the own slot's entries are 0)
    auto gather = [&](int pp, const uint32_t* wd, double* xv, double* dv) {
        const double* xp = x + (size_t(pp < P ? pp : 0) << pb);
        const int cbase = (pp < P ? pp : 0) << pb;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int cg = cbase + int(wd[u] & pmask);
            const bool own = cg >= olo && cg < ohi;
            xv[u] = own ? 0.0 : xp[wd[u] & pmask];  // word 0 past cnt: a valid address
            dv[u] = own ? 0.0 : (LDICT ? sdict[wd[u] >> pb] : dict[wd[u] >> pb]);
        }
    };
    // chunk k (p, c0), k+1 (p1, c1), k+2 (p2, c2)
    int p = 0;
    long long c0 = bst[0];
    advance(p, c0);
    int p1 = p;
    long long c1 = c0 + PCH;
    advance(p1, c1);
    uint32_t wd0[PER], wd1[PER], wd2[PER];
    uint16_t rr0[PER], rr1[PER], rr2[PER];
    double xv0[PER], dv0[PER], xv1[PER], dv1[PER];
    load_words(p, c0, wd0, rr0);
    load_words(p1, c1, wd1, rr1);
    gather(p, wd0, xv0, dv0);
    int buf = 0;
    while (p < P) {
        const int cnt = chunk_cnt(p, c0);
        int p2 = p1;
        long long c2 = c1 + PCH;
        advance(p2, c2);
#if EK_PANEL_DEPTH == 2
        gather(p1, wd1, xv1, dv1);     // chunk k+1's gathers
#endif
        load_words(p2, c2, wd2, rr2);  // chunk k+2's words
        double* pr = prod + buf * PCH;
        uint16_t* rb = rl + buf * PCH;
        double my[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = t + u * PT;
            my[u] = dv0[u] * xv0[u];
            if (i < cnt) {
                pr[i] = my[u];
                rb[i] = rr0[u];
            }
        }
        __syncthreads();
        // The first entry of each row's run adds the run in order.  A thread's
        // entries are 256 apart, so its heads are distinct rows: every LDS read
        // they need (the previous and next entries' rows, the accumulators) is
        // issued at once, and a run of one entry (most of them: ~1.2 entries
        // per row and panel at 10x) needs no further read.
        int prv[PER], nxt[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = t + u * PT;
            prv[u] = rb[max(i - 1, 0)];
            nxt[u] = rb[min(i + 1, PCH - 1)];
        }
        bool hd[PER];
        double a0[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = t + u * PT;
            hd[u] = i < cnt && (i == 0 || prv[u] != int(rr0[u]));
            a0[u] = acc[hd[u] ? int(rr0[u]) : 0];
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            if (!hd[u]) continue;
            const int i = t + u * PT;
            double sum = a0[u] + my[u];
            if (i + 1 < cnt && nxt[u] == int(rr0[u])) {
                int j = i + 1;
                do {
                    sum += pr[j];
                    ++j;
                } while (j < cnt && rb[j] == rr0[u]);
            }
            acc[rr0[u]] = sum;
        }
#if EK_PANEL_DEPTH != 2
        gather(p1, wd1, xv1, dv1);  // chunk k+1's gathers, after this chunk's LDS phase
#endif
        // rotate
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            wd1[u] = wd2[u];
            rr0[u] = rr1[u];
            rr1[u] = rr2[u];
            xv0[u] = xv1[u];
            dv0[u] = dv1[u];
        }
        p = p1;
        c0 = c1;
        p1 = p2;
        c1 = c2;
        buf ^= 1;
    }
    __syncthreads();  // the last chunk's runs are in acc
    double n2 = fn2 ? *fn2 : 1.0;
    if (fin.npart) {
        n2 = sum_parts ? panel_block_sum(npart_t, wsum) : fastv;
        if (w == 0 && t == 0) {
            fin.fn2_out[0] = n2;
            if (fin.step >= 0) {
                fin.alpha[fin.step] = *fin.a3 + fin.h2[fin.step];
                if (fin.step > 0)
                    fin.offd[fin.step] = (isnan(fin.bov_i[0]) ? sqrt(fin.fn2_i[0]) : fin.bov_i[0]) + fin.h2[fin.step - 1];
            }
        }
    }
    if (fin.chk_dst && w == 0) chk_mirror(fin, t, PT);  // (the check's copy: workgroup 0 only)
    const double scale = (fn2 || fin.npart) ? (n2 > 0.0 ? 1.0 / sqrt(n2) : 0.0) : 1.0;
    double av = 0.0, wv = 0.0;
    for (int r = t; r < nr; r += PT) {
        const double yr = (fin.ybase ? fin.ybase[r0 + r] + acc[r] : acc[r]) * scale;
        y[r0 + r] = yr;
        if (vcol) {
            const double v = f[r0 + r] * scale;
            vcol[r0 + r] = v;
            if (fin.v32col) fin.v32col[r0 + r] = float(v);
            av += v * yr;
            wv += yr * yr;
        }
    }
    if (apart) {
        const double s = panel_block_sum(av, wsum);
        if (t == 0) panel_store_sc1(apart + w, s);
        if (fin.wpart) {  // ||w||^2 partial (partial reorthogonalisation's beta estimate)
            const double q = panel_block_sum(wv, wsum);
            if (t == 0) fin.wpart[w] = q;
        }
    }
    if (alpha_out) {  // kernels_spmv.hip alpha_handoff: the last workgroup reduces alpha
        if (t == 0) {
            const unsigned nb = gridDim.x, g = blockIdx.x % ALPHA_SUB;
            const unsigned gsize = (nb - g + ALPHA_SUB - 1) / ALPHA_SUB, ngroups = nb < ALPHA_SUB ? nb : ALPHA_SUB;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            s_last = __hip_atomic_fetch_add(actr + g * 64, 1u, EK_HANDOFF_ORDER, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1u &&
                             __hip_atomic_fetch_add(actr + ALPHA_SUB * 64, 1u, EK_HANDOFF_ORDER,
                                                    __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1u
                         ? 1
                         : 0;
        }
        __syncthreads();
        if (s_last) {
            double s = 0.0;
            for (int i = t; i < int(gridDim.x); i += PT) s += panel_load_sc1(apart + i);
            s = panel_block_sum(s, wsum);
            if (t < ALPHA_SUB + 1) actr[t * 64] = 0u;
            if (t == 0) *alpha_out = s;
        }
    }
}

}  // namespace

size_t panel_lds_bytes(int max_rows, int ndict) {
    return 2 * size_t(PCH) * 8 + size_t(max_rows) * 8 + 2 * size_t(PCH) * 2 +
           (ndict <= PANEL_LDS_DICT ? size_t(ndict) * 8 : 0);
}

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
    const size_t lds = panel_lds_bytes(m.max_rows, m.ndict);
    if (!ev_start && !ev_stop) {  // a plain launch: the one a captured HIP graph records
        if (m.ndict <= PANEL_LDS_DICT)
            hipLaunchKernelGGL((k_spmv_panel<true>), dim3(m.G), dim3(PT), lds, s, m, dict, x, y, fn2, f, vcol, apart, fv,
                               alpha_out, actr);
        else
            hipLaunchKernelGGL((k_spmv_panel<false>), dim3(m.G), dim3(PT), lds, s, m, dict, x, y, fn2, f, vcol, apart,
                               fv, alpha_out, actr);
        return;
    }
    if (m.ndict <= PANEL_LDS_DICT)
        hipExtLaunchKernelGGL(k_spmv_panel<true>, dim3(m.G), dim3(PT), lds, s, ev_start, ev_stop, 0, m, dict, x, y, fn2,
                              f, vcol, apart, fv, alpha_out, actr);
    else
        hipExtLaunchKernelGGL(k_spmv_panel<false>, dim3(m.G), dim3(PT), lds, s, ev_start, ev_stop, 0, m, dict, x, y,
                              fn2, f, vcol, apart, fv, alpha_out, actr);
}

// The gather-only ceiling of the panel form (ek_spmv_gather_bench; VERDICT
// r5 next-4): the same grid, the same chunks in the same panel order, the same
// word / row-index stream and the same x and value-table gathers, with the
// products summed in registers — no LDS staging, no row runs, no barrier, no
// y.  Its time is what the product kernel's access pattern costs by itself.
template <bool LDICT>
__global__ __launch_bounds__(PT) void k_panel_gather_only(SpmvPanel m, const double* __restrict__ dict,
                                                          const double* __restrict__ x, double* __restrict__ sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* sdict = reinterpret_cast<double*>(smem);
    const int w = blockIdx.x, t = threadIdx.x;
    if constexpr (LDICT) {
        for (int i = t; i < m.ndict; i += PT) sdict[i] = dict[i];
        __syncthreads();
    }
    const uint32_t pmask = (1u << m.pb) - 1u;
    double acc = 0.0;
    unsigned rsum = 0u;
    for (int p = 0; p < m.P; ++p) {
        const long long a = m.start[size_t(w) * m.P + p], b = m.start[size_t(w) * m.P + p + 1];
        const double* xp = x + (size_t(p) << m.pb);
        for (long long c = a; c < b; c += PCH) {
            uint32_t wd[PER];
            uint16_t rr[PER];
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const long long i = c + t + u * PT;
                wd[u] = i < b ? m.word[i] : 0u;
                rr[u] = i < b ? m.rid[i] : uint16_t(0);
            }
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const double dv = LDICT ? sdict[wd[u] >> m.pb] : dict[wd[u] >> m.pb];
                acc += dv * xp[wd[u] & pmask];
                rsum += rr[u];
            }
        }
    }
    if (acc == -1.2345e300 && rsum == 7u) sink[w] = acc;  // (keeps every load; never true in practice)
}

void panel_gather_only(hipStream_t s, const SpmvPanel& m, const double* dict, const double* x, double* sink) {
    if (m.ndict <= PANEL_LDS_DICT)
        hipLaunchKernelGGL((k_panel_gather_only<true>), dim3(m.G), dim3(PT), size_t(m.ndict) * 8 + 16, s, m, dict, x,
                           sink);
    else
        hipLaunchKernelGGL((k_panel_gather_only<false>), dim3(m.G), dim3(PT), 16, s, m, dict, x, sink);
}

}  // namespace dev
}  // namespace ek
