// Kernighan-Lin on gfx950: per-node gain compute + max-gain-pair selection,
// bit-exact with the reference cKL (cKL.cpp:225-390).
//
// Parity rules (SURVEY §8c checklist):
//   * gain(u) = E - I with I/E two SEQUENTIAL fp32 accumulators over the row
//     in cKL order (forward = libstdc++ map order, backward = ascending id),
//     I taking neighbours on side 0 (split[0]) — no in-row parallel reduction;
//   * node1 = first position in remain[0] with the maximum gain (strict '>'
//     scan from -FLT_MAX), node2 = first position in remain[1] with the
//     minimum gain (strict '<' from FLT_MAX); +0 and -0 tie;
//   * gain = (g1 - g2) - 2*w(node1,node2); cut -= gain; running minimum keeps
//     the first occurrence; stop after more than floor(log2 n)+5 consecutive
//     gains <= 0 or when a side runs out.
//
// Layout / MI355X mapping:
//   * k_gain_scan   : one lane per row (the sequential fp32 order forbids
//                     splitting a row), all n rows; also fp64 per-block
//                     partials of the initial cut.
//   * k_chunk_init  : one wave64 per 256-position chunk of each remain[]
//                     list; the chunk's best (gain, first position) packed in
//                     a 64-bit key whose unsigned max IS the cKL selection
//                     rule, so a wave64 shuffle max is an exact argmax.
//   * k_kl_loop     : the whole swap loop in ONE persistent 1024-thread
//                     workgroup (no grid-wide sync, no host round trip per
//                     iteration — the reference gKL paid 2 launches + PCIe
//                     copies of remain and membership per iteration,
//                     gKL.cu:188-227).  Per iteration: argmax over chunk keys,
//                     edge weight lookup, swap, recompute the gains of
//                     N(node1) u N(node2) (one lane per row), re-key only the
//                     chunks those nodes live in.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "ek_internal.hpp"

namespace ek {
namespace dev {

typedef unsigned long long u64;

__device__ __forceinline__ uint32_t ord_f32(float g) {
    if (g == 0.0f) g = 0.0f;  // -0 == +0 under cKL's comparisons
    const uint32_t u = __float_as_uint(g);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
// remain[0]: larger gain wins, then smaller position; invalid (NaN, <= -FLT_MAX) -> 0
__device__ __forceinline__ u64 key_max(float g, int pos) {
    if (!(g > -FLT_MAX)) return 0ull;
    return (u64(ord_f32(g)) << 32) | u64(~uint32_t(pos));
}
// remain[1]: smaller gain wins, then smaller position; invalid (NaN, >= FLT_MAX) -> 0
__device__ __forceinline__ u64 key_min(float g, int pos) {
    if (!(g < FLT_MAX)) return 0ull;
    return (u64(ord_f32(-g)) << 32) | u64(~uint32_t(pos));
}
__device__ __forceinline__ u64 wave_max_u64(u64 v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const u64 x = __shfl_xor(v, o, 64);
        v = x > v ? x : v;
    }
    return v;
}

// connections(node), cKL.cpp:225-251, over the cKL-ordered row.
__device__ __forceinline__ float row_gain(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                          const float* __restrict__ w, const uint8_t* __restrict__ side, int u,
                                          float* ext_out) {
    float internal = 0.0f, external = 0.0f;
    const int p1 = rowptr[u + 1];
    for (int p = rowptr[u]; p < p1; ++p) {
        const float wt = w[p];
        if (side[col[p]] == 0) internal += wt;
        else external += wt;
    }
    if (ext_out) *ext_out = external;
    return external - internal;
}

__device__ __forceinline__ u64 chunk_key(const KLDev& d, int s, int c, int lane) {
    const int32_t* order = s ? d.order1 : d.order0;
    const int ns = s ? d.n1 : d.n0;
    u64 k = 0ull;
#pragma unroll
    for (int q = 0; q < KL_CHUNK / 64; ++q) {
        const int p = c * KL_CHUNK + q * 64 + lane;
        if (p < ns) {
            const int u = order[p];
            if (!d.locked[u]) {
                const u64 kk = s ? key_min(d.gain[u], p) : key_max(d.gain[u], p);
                k = kk > k ? kk : k;
            }
        }
    }
    return wave_max_u64(k);
}

__global__ __launch_bounds__(256) void k_gain_scan(KLDev d) {
    __shared__ double lds4[4];
    const int u = blockIdx.x * 256 + threadIdx.x;
    double c = 0.0;
    if (u < d.n) {
        float ext = 0.0f;
        d.gain[u] = row_gain(d.rowptr, d.col, d.w, d.side, u, &ext);
        if (d.side[u] == 0) c = double(ext);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) lds4[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) d.cut_part[blockIdx.x] = (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
}

// initial cut (cKL.cpp:199-223): fp64 sum of the per-node fp32 externals of
// side-0 nodes, rounded once to fp32 (DESIGN.md "initial cut").
__global__ __launch_bounds__(256) void k_cut_final(KLDev d, int nb) {
    __shared__ double lds4[4];
    double s = 0.0;
    for (int i = threadIdx.x; i < nb; i += 256) s += d.cut_part[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) lds4[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) *d.cut0 = float((lds4[0] + lds4[1]) + (lds4[2] + lds4[3]));
}

__global__ __launch_bounds__(256) void k_chunk_init(KLDev d) {
    const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (wv < d.nck0) {
        const u64 k = chunk_key(d, 0, wv, lane);
        if (lane == 0) d.ckey0[wv] = k;
    } else if (wv < d.nck0 + d.nck1) {
        const u64 k = chunk_key(d, 1, wv - d.nck0, lane);
        if (lane == 0) d.ckey1[wv - d.nck0] = k;
    }
}

__global__ __launch_bounds__(KL_LOOP_THREADS) void k_kl_loop(KLDev d, int limit, ek_swap* __restrict__ log,
                                                             long long cap, KLOut* __restrict__ out) {
    constexpr int NW = KL_LOOP_THREADS / 64;
    __shared__ u64 red0[NW], red1[NW];
    __shared__ int s_a, s_b, s_stop, s_go;
    __shared__ float s_w;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // loop-carried scalars live in thread 0 only
    float cut = *d.cut0, best = cut;
    long long best_it = 0, it = 0;
    unsigned term = 0;
    for (;;) {
        // 1. selection: max over chunk keys of both lists (cKL.cpp:341-355)
        u64 k0 = 0ull, k1 = 0ull;
        for (int c = tid; c < d.nck0; c += KL_LOOP_THREADS) k0 = d.ckey0[c] > k0 ? d.ckey0[c] : k0;
        for (int c = tid; c < d.nck1; c += KL_LOOP_THREADS) k1 = d.ckey1[c] > k1 ? d.ckey1[c] : k1;
        k0 = wave_max_u64(k0);
        k1 = wave_max_u64(k1);
        if (lane == 0) {
            red0[wv] = k0;
            red1[wv] = k1;
        }
        __syncthreads();
        if (tid == 0) {
            u64 a = 0ull, b = 0ull;
            for (int i = 0; i < NW; ++i) {
                a = red0[i] > a ? red0[i] : a;
                b = red1[i] > b ? red1[i] : b;
            }
            s_go = (a != 0ull && b != 0ull);  // cKL.cpp:357,387-388
            if (s_go) {
                s_a = d.order0[~uint32_t(a & 0xffffffffull)];
                s_b = d.order1[~uint32_t(b & 0xffffffffull)];
            }
            s_w = 0.0f;
        }
        __syncthreads();
        if (!s_go) break;
        const int A = s_a, B = s_b;
        // 2. w(A,B) (getEdgeWeight, cKL.cpp:75-82): B occurs at most once in A's row
        {
            const int pa0 = d.rowptr[A], pa1 = d.rowptr[A + 1];
            for (int p = pa0 + tid; p < pa1; p += KL_LOOP_THREADS)
                if (d.col[p] == B) s_w = d.w[p];
        }
        __syncthreads();
        // 3. pair gain, running cut, log, swap (cKL.cpp:358-386, swip :274-286)
        if (tid == 0) {
            const float gA = d.gain[A], gB = d.gain[B];
            const float gain = gA - gB - 2.0f * s_w;
            cut -= gain;
            ++it;
            if (cut < best) {
                best = cut;
                best_it = it;
            }
            if (it <= cap) log[it - 1] = ek_swap{uint32_t(it), uint32_t(A), uint32_t(B), gA, gB, gain, cut, 0u};
            d.locked[A] = 1;
            d.locked[B] = 1;
            d.side[A] = 1;
            d.side[B] = 0;
            int stop = 0;
            if (gain <= 0.0f) {
                if (++term > unsigned(limit)) stop = 1;
            } else {
                term = 0;
            }
            if (it >= d.n0 || it >= d.n1) stop = 1;  // a remain[] list is exhausted
            s_stop = stop;
        }
        __syncthreads();
        // 4. gains of N(A) u N(B) (updateAffectedNodeGains, cKL.cpp:253-272)
        const int pa = d.rowptr[A], la = d.rowptr[A + 1] - pa;
        const int pb = d.rowptr[B], lb = d.rowptr[B + 1] - pb;
        for (int i = tid; i < la + lb; i += KL_LOOP_THREADS) {
            const int u = i < la ? d.col[pa + i] : d.col[pb + i - la];
            d.gain[u] = row_gain(d.rowptr, d.col, d.w, d.side, u, nullptr);
        }
        __syncthreads();
        // 5. re-key the chunks holding A, B and every affected node
        for (int i = wv; i < la + lb + 2; i += NW) {
            const int u = i < la ? d.col[pa + i] : i < la + lb ? d.col[pb + i - la] : (i == la + lb ? A : B);
            const int s = d.side_init[u];
            const int c = d.pos[u] / KL_CHUNK;
            const u64 k = chunk_key(d, s, c, lane);
            if (lane == 0) (s ? d.ckey1 : d.ckey0)[c] = k;
        }
        __syncthreads();
        if (s_stop) break;
    }
    if (tid == 0) {
        out->iterations = it;
        out->best_iter = best_it;
        out->initial_cut = *d.cut0;
        out->best_cut = best;
        out->final_cut = cut;
        out->status = 0u;
    }
}

// sides after the first *count swaps: copy (this launch), then apply the
// swaps (next launch; every node is swapped at most once, so they commute).
__global__ __launch_bounds__(256) void k_replay(int n, const uint8_t* __restrict__ side_init,
                                                uint8_t* __restrict__ out) {
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += 256ll * gridDim.x) out[i] = side_init[i];
}

__global__ __launch_bounds__(256) void k_replay_swaps(const ek_swap* __restrict__ log, const long long* __restrict__ count,
                                                      long long cap, uint8_t* __restrict__ out) {
    const long long cnt = *count < cap ? *count : cap;
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < cnt; i += 256ll * gridDim.x) {
        out[log[i].node_left] = 1;
        out[log[i].node_right] = 0;
    }
}

// integer hyperedge cut: nets whose pins are not all on one side
__global__ __launch_bounds__(256) void k_net_cut(long long nets, const int64_t* __restrict__ net_ptr,
                                                 const int32_t* __restrict__ pins, const uint8_t* __restrict__ side,
                                                 unsigned long long* __restrict__ count) {
    const long long e = blockIdx.x * 256ll + threadIdx.x;
    bool cut = false;
    if (e < nets) {
        const int64_t p0 = net_ptr[e], p1 = net_ptr[e + 1];
        if (p1 - p0 >= 2) {
            const uint8_t s0 = side[pins[p0]];
            for (int64_t p = p0 + 1; p < p1 && !cut; ++p) cut = side[pins[p]] != s0;
        }
    }
    const u64 m = __ballot(cut);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(count, (unsigned long long)__popcll(m));
}

void kl_prepare(hipStream_t s, const KLDev& d) {
    const int nb = (d.n + 255) / 256;
    hipLaunchKernelGGL(k_gain_scan, dim3(nb), dim3(256), 0, s, d);
    hipLaunchKernelGGL(k_cut_final, dim3(1), dim3(256), 0, s, d, nb);
    const int waves = d.nck0 + d.nck1;
    hipLaunchKernelGGL(k_chunk_init, dim3((waves + 3) / 4), dim3(256), 0, s, d);
}

void kl_loop(hipStream_t s, const KLDev& d, int limit, ek_swap* log, long long cap, KLOut* out) {
    hipLaunchKernelGGL(k_kl_loop, dim3(1), dim3(KL_LOOP_THREADS), 0, s, d, limit, log, cap, out);
}

void kl_replay(hipStream_t s, int n, const uint8_t* side_init, const ek_swap* log, const long long* count,
               long long cap, uint8_t* sides_out) {
    const int nb = std::min(2048, (n + 255) / 256);
    hipLaunchKernelGGL(k_replay, dim3(nb), dim3(256), 0, s, n, side_init, sides_out);
    hipLaunchKernelGGL(k_replay_swaps, dim3(64), dim3(256), 0, s, log, count, cap, sides_out);
}

void net_cut(hipStream_t s, int64_t nets, const int64_t* net_ptr, const int32_t* pins, const uint8_t* side,
             unsigned long long* count) {
    if (nets <= 0) return;
    hipLaunchKernelGGL(k_net_cut, dim3(unsigned((nets + 255) / 256)), dim3(256), 0, s, (long long)nets, net_ptr, pins,
                       side, count);
}

}  // namespace dev
}  // namespace ek
