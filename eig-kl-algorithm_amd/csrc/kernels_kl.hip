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
//   * k_chunk_init  : one wave64 per chunk (KL_CHUNK positions; KL_CHUNK_GB for the off-chip-bitmap loop) of each remain[]
//                     list; the chunk's best (gain, first position) packed in
//                     a 64-bit key whose unsigned max IS the cKL selection
//                     rule, so a wave64 shuffle max is an exact argmax.
//   * k_kl_swap_loop: the whole swap loop in ONE persistent 512-thread
//                     workgroup (no grid-wide sync, no host round trip per
//                     iteration — the reference gKL paid 2 launches + PCIe
//                     copies of remain and membership per iteration,
//                     gKL.cu:188-227).  Per iteration: argmax over chunk keys,
//                     edge weight lookup, swap, recompute the gains of
//                     N(node1) u N(node2) (one lane per row), re-key only the
//                     chunks those nodes live in.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>

#include "ek_internal.hpp"

#ifndef EK_KL_PREFETCH
#define EK_KL_PREFETCH 1  // provisional next pair's rows touched into L2 across barrier 2 (0: off, for A/B)
#endif
#ifndef EK_KL_NEXT
// 1: P selects the next pair exactly between the barriers and publishes it;
// the waves read it after barrier 2 instead of selecting.  Same swap logs,
// but 2.26 against 1.96 us/swap (profiles/r05/kl/kl_ab_next.txt): P's
// resolve holds barrier 2 back more than the selection it saves.
#define EK_KL_NEXT 0
#endif
#ifndef EK_E_TWO_TRIPS
#define EK_E_TWO_TRIPS 1  // early rescans: gains, then the winner's descriptor (0: both in one trip, A/B; 2.03 vs 2.00 us/swap)
#endif
#ifndef EK_G1_DRAIN
#define EK_G1_DRAIN 0  // lab: gain waves drain their stores at the loop top (vmcnt(0))
#endif
#ifndef EK_PIPE_SLEEP
#define EK_PIPE_SLEEP 1  // k_kl_swap_pipe: s_sleep units between the polls of a wait
#endif
#ifndef EK_E_SLEEP
#define EK_E_SLEEP 0  // early-rescan waves: s_sleep units before their loads (two-trip rescans: 0 best, 4: +0.01 us/swap)
#endif

namespace ek {
namespace dev {

typedef unsigned long long u64;
typedef int v4i __attribute__((ext_vector_type(4)));  // a clang vector: stays in registers where HIP's int4 struct may not
typedef float v2f __attribute__((ext_vector_type(2)));

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
// wave64 max of a 64-bit key without LDS traffic, in two 32-bit passes: the
// max of the high words, then the max of the low words of the lanes holding
// it.  Each pass is DPP quad_perm / row (half-)mirror steps inside each
// 16-lane row (v_max_u32 with a DPP source: one instruction per step), then
// gfx950's v_permlane16_swap (and v_permlane32_swap) across rows and halves.
// Every lane ends with the max.  (One 64-bit pass costs a compare and two
// selects per step.)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_max32(uint32_t v) {
    const uint32_t o = __builtin_amdgcn_update_dpp(0u, v, CTRL, 0xf, 0xf, false);  // 0: max's identity
    return o > v ? o : v;
}
__device__ __forceinline__ uint32_t row_max32(uint32_t v) {
    v = dpp_max32<0xB1>(v);   // quad_perm [1,0,3,2]
    v = dpp_max32<0x4E>(v);   // quad_perm [2,3,0,1]
    v = dpp_max32<0x141>(v);  // row_half_mirror
    return dpp_max32<0x140>(v);  // row_mirror
}
// max within each 32-lane half of the wave (lanes 0-31 and 32-63 separately)
__device__ __forceinline__ uint32_t half_max32(uint32_t v) {
    v = row_max32(v);
    const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return a[0] > a[1] ? a[0] : a[1];
}
__device__ __forceinline__ uint32_t wave_max32(uint32_t v) {
    v = half_max32(v);
    const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return a[0] > a[1] ? a[0] : a[1];
}
__device__ __forceinline__ u64 half_max_u64(u64 v) {
    const uint32_t hi = uint32_t(v >> 32), lo = uint32_t(v);
    const uint32_t H = half_max32(hi);
    return (u64(H) << 32) | half_max32(hi == H ? lo : 0u);
}
__device__ __forceinline__ u64 wave_max_u64(u64 v) {
    const uint32_t hi = uint32_t(v >> 32), lo = uint32_t(v);
    const uint32_t H = wave_max32(hi);
    return (u64(H) << 32) | wave_max32(hi == H ? lo : 0u);
}

// value of lane t of each 4-lane quad, in every lane of the quad (DPP
// quad_perm [t,t,t,t]; t a compile-time constant once the caller is unrolled)
__device__ __forceinline__ float quad_bcast(float v, int t) {
    switch (t) {
        case 0: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x00, 0xf, 0xf, false));
        case 1: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x55, 0xf, 0xf, false));
        case 2: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xAA, 0xf, 0xf, false));
        default: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xFF, 0xf, 0xf, false));
    }
}

// uniform broadcast of lane `l` (v_readlane: no LDS round trip, unlike __shfl)
__device__ __forceinline__ u64 readlane_u64(u64 v, int l) {
    const unsigned lo = __builtin_amdgcn_readlane(unsigned(v), l), hi = __builtin_amdgcn_readlane(unsigned(v >> 32), l);
    return (u64(hi) << 32) | lo;
}

// side of node v (0/1): LDS bitmap or global byte array
template <bool SMEM>
__device__ __forceinline__ uint32_t side_of(const uint32_t* s_side, const uint8_t* g_side, int v) {
    if constexpr (SMEM) return (s_side[v >> 5] >> (v & 31)) & 1u;
    else return g_side[v];
}

// bitmap word i of the side bytes (bit j = node 32i+j on side 1): a whole
// word is two 16-B loads (the byte array is hipMalloc'd, so 32i is 16-B
// aligned); the last, partial word reads clamped bytes unconditionally.  (A
// load behind a per-byte bounds branch waits for every load before it: the
// byte-at-a-time form issued 32 dependent round trips per word.)
__device__ __forceinline__ uint32_t side_word(const uint8_t* __restrict__ side, int n, int i) {
    const int base = i * 32;
    uint32_t b = 0;
    if (base + 32 <= n) {
        const uint4 a = *reinterpret_cast<const uint4*>(side + base);
        const uint4 c = *reinterpret_cast<const uint4*>(side + base + 16);
        const uint32_t w[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q) b |= uint32_t(((w[k] >> (8 * q)) & 0xffu) == 1u) << (4 * k + q);
    } else {
        uint8_t v[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j] = side[min(base + j, n - 1)];
#pragma unroll
        for (int j = 0; j < 32; ++j) b |= uint32_t(base + j < n && v[j] == 1) << j;
    }
    return b;
}

// connections(node), cKL.cpp:225-251, over the cKL-ordered row: two
// sequential fp32 accumulators, internal = neighbour on side 0.
template <bool SMEM>
__device__ __forceinline__ float row_gain(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                          const float* __restrict__ w, const uint32_t* s_side,
                                          const uint8_t* g_side, int u, float* ext_out) {
    float internal = 0.0f, external = 0.0f;
    const int p1 = rowptr[u + 1];
    for (int p = rowptr[u]; p < p1; ++p) {
        const float wt = w[p];
        if (side_of<SMEM>(s_side, g_side, col[p]) == 0) internal += wt;
        else external += wt;
    }
    if (ext_out) *ext_out = external;
    return external - internal;
}

// best key of KL_CHUNK consecutive positions of one remain[] list (gains by
// position).  The gain arrays are padded with NaN (invalid key) to a whole
// number of chunks, so every load is unconditional and all are in flight at once.
template <int CH = KL_CHUNK>
__device__ __forceinline__ u64 chunk_key(const float* __restrict__ gp, int s, int c, int lane) {
    float g[CH / 64];
#pragma unroll
    for (int q = 0; q < CH / 64; ++q) g[q] = gp[c * CH + q * 64 + lane];
    u64 k = 0ull;
#pragma unroll
    for (int q = 0; q < CH / 64; ++q) {
        const int p = c * CH + q * 64 + lane;
        const u64 kk = s ? key_min(g[q], p) : key_max(g[q], p);
        k = kk > k ? kk : k;
    }
    return wave_max_u64(k);
}

__global__ __launch_bounds__(256) void k_gain_scan(KLDev d) {
    __shared__ double lds4[4];
    const int u = blockIdx.x * 256 + threadIdx.x;
    double c = 0.0;
    if (u < d.n) {
        float ext = 0.0f;
        const float g = row_gain<false>(d.rowptr, d.col, d.w, nullptr, d.side_init, u, &ext);
        const uint32_t pl = d.plist[u];
        ((pl >> 31) ? d.gp1 : d.gp0)[pl & 0x7fffffffu] = g;
        if (d.side_init[u] == 0) c = double(ext);
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

// The lane's best of several positions p0 + 64 q (+ lane), compared as fp32
// gains: the same winner as the largest key_max / key_min, since within a lane
// positions rise with q, so a strict compare keeps the first of equal gains
// (+0 and -0 compare equal), NaN never compares true and the invalid ends
// (<= -FLT_MAX for list 0, >= FLT_MAX for list 1) never beat the initial
// value.  One compare and two selects per position instead of building and
// comparing a 64-bit key; the key is built once, for the lane's winner.
// Returns the winner's q in *bq (-1: none).
template <int NQ>
__device__ __forceinline__ u64 lane_best(const float* g, int s, int p0, int lane, int skip, int* bq) {
    float bg = s ? FLT_MAX : -FLT_MAX;
    int q0 = -1;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const float gq = p0 + q * 64 + lane == skip ? __builtin_nanf("") : g[q];
        const bool better = s ? gq < bg : gq > bg;
        bg = better ? gq : bg;
        q0 = better ? q : q0;
    }
    *bq = q0;
    if (q0 < 0) return 0ull;
    const int p = p0 + q0 * 64 + lane;
    return s ? key_min(bg, p) : key_max(bg, p);
}

// Best key of one chunk together with its winner's row descriptor.  Gains and
// descriptors are both read by position, so the winner needs no dependent
// load.  Returns the key in every lane; the winner lane (or lane 0 for an
// all-invalid chunk) has *mine = true and its descriptor in *info.
// (in blocks of 32 positions a lane: a 4096-position chunk's 64 gains and
// descriptors would not fit the registers at once; the keys carry their
// position, so the running max over blocks is the same winner)
template <int CH = KL_CHUNK>
__device__ __forceinline__ u64 chunk_best(const float* __restrict__ gp, const KLInfo* __restrict__ pinfo, int s,
                                          int c, int lane, KLInfo* info, bool* mine) {
    constexpr int NB = CH / 64 < 32 ? CH / 64 : 32;
    u64 k = 0ull;
    int4 bi = make_int4(0, 0, 0, 0);
    for (int q0 = 0; q0 < CH / 64; q0 += NB) {
        float g[NB];
        int4 pi[NB];
#pragma unroll
        for (int q = 0; q < NB; ++q) {  // padded arrays: unconditional, all in flight
            const int p = c * CH + (q0 + q) * 64 + lane;
            g[q] = gp[p];
            pi[q] = *reinterpret_cast<const int4*>(pinfo + p);
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const int p = c * CH + (q0 + q) * 64 + lane;
            const u64 kk = s ? key_min(g[q], p) : key_max(g[q], p);
            if (kk > k) {
                k = kk;
                bi = pi[q];
            }
        }
    }
    const u64 m = wave_max_u64(k);
    const u64 bal = __ballot(m != 0ull && k == m);
    *mine = bal ? (lane == __ffsll((long long)bal) - 1) : (lane == 0);
    info->a = bi.x;
    info->b = bi.y;
    info->c = bi.z;
    info->d = bi.w;
    return m;
}

template <int CH>
__global__ __launch_bounds__(256) void k_chunk_init(KLDev d) {
    const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (wv >= d.nck0 + d.nck1) return;
    const int s = wv < d.nck0 ? 0 : 1, c = s ? wv - d.nck0 : wv;
    if (d.pinfo0) {
        KLInfo info;
        bool mine;
        const u64 k = s ? chunk_best<CH>(d.gp1, d.pinfo1, 1, c, lane, &info, &mine)
                        : chunk_best<CH>(d.gp0, d.pinfo0, 0, c, lane, &info, &mine);
        if (mine) {
            (s ? d.ckey1 : d.ckey0)[c] = k;
            (s ? d.cinfo1 : d.cinfo0)[c] = info;
        }
    } else {
        const u64 k = s ? chunk_key<CH>(d.gp1, 1, c, lane) : chunk_key<CH>(d.gp0, 0, c, lane);
        if (lane == 0) (s ? d.ckey1 : d.ckey0)[c] = k;
    }
}

// chunk-key arrays the selection reads are padded with zero keys to a whole
// number of 32-lane passes (both lists to the same count): every wave reduces
// all of them itself, one half-wave per list
__host__ __device__ inline int kl_sel_pad(int nck0, int nck1) {
    const int m = nck0 > nck1 ? nck0 : nck1;
    return (m + 31) / 32 * 32;
}

// staging row stride in 16-B pieces: one piece of padding, so the 8 summing
// lanes of a wave (one per row) read 8 different bank groups instead of one
constexpr int KL_STAGE_ROW = KL_SEG_LANES + 1;
constexpr int KL_STAGE_ROWS = 16;  // rows a gain wave stages per pass (16 coded, 8 plain)
// updated rows that live in node1's / node2's own chunk, per list (more: the
// chunk is rescanned).  A chunk holds 1024 of the list's positions, so most
// swaps have none.
constexpr int KL_AB_CAP = 16;
// waves rescanning each of the two chunks node1 / node2 leave (E); the other
// waves but the pair-gain one run the gain updates (A/B: EK_KL_EPARTS=1)
#ifndef EK_KL_EPARTS
#define EK_KL_EPARTS 2
#endif
constexpr int KL_E_PARTS = EK_KL_EPARTS;
// chunks a list may have for k_kl_swap_loop's fixed LDS layout (FIX): 131,072
// positions a list
constexpr int KL_FIX_NCK = 131072 / KL_CHUNK;

size_t kl_loop_lds_bytes(const KLDev& d, bool bitmaps, bool fixed) {
    if (fixed && (d.nck0 > KL_FIX_NCK || d.nck1 > KL_FIX_NCK || d.nwd > KL_WDICT_CAP)) return 0;
    const size_t words = bitmaps ? (size_t(d.n) + 31) / 32 : 0;
    const size_t nck = fixed ? size_t(2 * KL_FIX_NCK) : size_t(d.nck0) + size_t(d.nck1);
    // staging for the gain waves: NG = waves - 1 (pair gain) - 2 * KL_E_PARTS (early rescans), as carved by the kernel
    constexpr size_t NG = KL_LOOP_THREADS / 64 - 1 - 2 * KL_E_PARTS;
    const size_t b = (nck + KL_ITEM_CAP + 4 + 2 * KL_AB_CAP + 2 + NG * KL_STAGE_ROWS * KL_STAGE_ROW) * sizeof(KLInfo) +
                     (2 * size_t(fixed ? KL_FIX_NCK : kl_sel_pad(d.nck0, d.nck1)) + nck + KL_ITEM_CAP + 4 + 2 * KL_AB_CAP + 2) * 8 +
                     (2 * nck + KL_ITEM_CAP + 4 + 4 + 4) * 4 + 2 * words * 4 +
                     (fixed ? size_t(KL_WDICT_CAP) : size_t(d.segc ? d.nwd : 0)) * 4 +
                     128;  // (+ k_kl_swap_pipe's speculative pair, 16-B aligned)
    return b <= 152 * 1024 ? b : 0;
}

// Best key of chunk c of one remain[] list over its positions other than
// `skip` (gains by position; the arrays are padded, so the loads are
// unconditional and all in flight at once).  Every lane gets the key; the
// winner lane (lane 0 for an all-invalid chunk) has *mine set and loads the
// winner's row descriptor into *info.
template <int CH = KL_CHUNK>
__device__ __forceinline__ u64 chunk_rescan(const float* __restrict__ gp, const KLInfo* __restrict__ pinfo, int s,
                                            int c, int skip, int lane, KLInfo* info, bool* mine) {
    float g[CH / 64];
#pragma unroll
    for (int q = 0; q < CH / 64; ++q) g[q] = gp[c * CH + q * 64 + lane];
    int bq;
    const u64 k = lane_best<CH / 64>(g, s, c * CH, lane, skip, &bq);
    const int bp = c * CH + (bq < 0 ? 0 : bq) * 64 + lane;
    const u64 m = wave_max_u64(k);
    const u64 bal = __ballot(m != 0ull && k == m);  // keys carry the position: one lane at most
    *mine = bal ? (lane == __ffsll((long long)bal) - 1) : (lane == 0);
    KLInfo inf{0, 0, 0, 0};
    if (bal && *mine) {
        const int4 x = *reinterpret_cast<const int4*>(pinfo + bp);
        inf = KLInfo{x.x, x.y, x.z, x.w};
    }
    // wait for that load here, on this (rare) path: left pending, the
    // compiler's wait tracking carries it past the join, and every later
    // write of those registers in the common path then waits vmcnt(0) —
    // i.e. for the acks of the gain stores of the swap
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) alone (gfx9 encoding)
    *info = inf;
    return m;
}

// chunk_rescan over one part: gains first, then the winner's descriptor (two
// round trips, 2 KB a wave instead of 10 KB beside the gain waves' loads)
template <int NQ>
__device__ __forceinline__ u64 chunk_rescan2(const float* __restrict__ gp, const KLInfo* __restrict__ pinfo, int s,
                                             int p0, int skip, int lane, KLInfo* info, bool* mine) {
    float g[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) g[q] = gp[p0 + q * 64 + lane];
    int bq;
    const u64 k = lane_best<NQ>(g, s, p0, lane, skip, &bq);
    const u64 m = wave_max_u64(k);
    const u64 bal = __ballot(m != 0ull && k == m);  // keys carry the position: one lane at most
    *mine = bal ? (lane == __ffsll((long long)bal) - 1) : (lane == 0);
    KLInfo inf{0, 0, 0, 0};
    if (bal && *mine) {
        const int4 x = *reinterpret_cast<const int4*>(pinfo + p0 + bq * 64 + lane);
        inf = KLInfo{x.x, x.y, x.z, x.w};
    }
    *info = inf;
    return m;
}

// chunk_rescan with every position's descriptor loaded beside its gain: one
// round trip instead of two (the early rescans run beside the gain updates and
// must not outlast them)
// (over positions [p0, p0 + 64*NQ), one of the chunk's parts)
template <int NQ>
__device__ __forceinline__ u64 chunk_rescan1(const float* __restrict__ gp, const KLInfo* __restrict__ pinfo, int s,
                                             int p0, int skip, int lane, KLInfo* info, bool* mine) {
    float g[NQ];
    int4 pi[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int p = p0 + q * 64 + lane;
        g[q] = gp[p];
        pi[q] = *reinterpret_cast<const int4*>(pinfo + p);
    }
    // lane_best's compare, carrying the winner's descriptor along (a select by
    // the winning index afterwards becomes a dynamically indexed array: scratch)
    float bg = s ? FLT_MAX : -FLT_MAX;
    int bq = -1;
    int4 bi = make_int4(0, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const float gq = p0 + q * 64 + lane == skip ? __builtin_nanf("") : g[q];
        const bool better = s ? gq < bg : gq > bg;
        bg = better ? gq : bg;
        bq = better ? q : bq;
        bi.x = better ? pi[q].x : bi.x;
        bi.y = better ? pi[q].y : bi.y;
        bi.z = better ? pi[q].z : bi.z;
        bi.w = better ? pi[q].w : bi.w;
    }
    const int bp = p0 + (bq < 0 ? 0 : bq) * 64 + lane;
    const u64 k = bq < 0 ? 0ull : (s ? key_min(bg, bp) : key_max(bg, bp));
    const u64 m = wave_max_u64(k);
    const u64 bal = __ballot(m != 0ull && k == m);
    *mine = bal ? (lane == __ffsll((long long)bal) - 1) : (lane == 0);
    *info = bal ? KLInfo{bi.x, bi.y, bi.z, bi.w} : KLInfo{0, 0, 0, 0};
    return m;
}

// The swap loop (cKL.cpp:334-390) in ONE persistent 512-thread workgroup,
// its state on chip: LDS holds the side/locked bitmaps, every chunk's best key
// and its winner's row descriptor {node, rowptr, rowlen}.  Per swap:
//   S   every wave selects node1 / node2 itself from the chunk keys (a few
//       keys per lane, DPP + permlane reductions per half-wave): no barrier;
//   W   the last wave: w(node1, node2), pair gain, running cut, log, stop rule;
//   E   two waves rescan the chunks node1 and node2 leave (they were those
//       chunks' winners) CONCURRENTLY with G1, off its dependency chain;
//   G1  the other waves recompute the gains of N(node1) u N(node2) (one lane
//       per row, the reference's sequential fp32 order) and merge the risen
//       keys of every other chunk into shadow keys (LDS atomicMax);
//   --- barrier ---
//   G2  resolve node1's / node2's chunk from the early rescan and the new keys
//       of the updated rows in it, publish merged keys, rescan the (rare)
//       chunks whose winner fell;
//   --- barrier ---
// Early-rescan rule: the rescan skips node1 (node2) and may read either the
// old or the new gain of a row G1 updates meanwhile.  If its winner R is not
// such a row, the chunk's key is exactly max(R, new keys of the updated rows
// in the chunk); if R is one whose new key is below R, R was a stale value and
// the chunk is rescanned after the barrier.
// SEGC: the rows' inline segments are the weight-coded ones (KLDev::segc),
// decoded through the weight table in LDS; the staged contributions and the
// sums are the same as from the plain segments.
// GB: the side / locked bitmaps live in global memory (in KLDev::locked: a graph
// whose n/4 bytes of bitmaps exceed the LDS budget while the rest still fits);
// they are read with agent-scope loads (performed at the L2, past the CU's
// vector L1) and flipped with agent-scope atomics, drained before barrier 2.
// The logic and the swap log are the on-chip form's.
// FIX: every LDS array at a compile-time offset, sized for KL_FIX_NCK chunks a
// list and KL_WDICT_CAP weight codes (the bitmaps last): the addresses fold
// into the LDS instructions' offsets instead of ~25 SGPRs of carve pointers,
// which the register allocator otherwise spills into VGPR lanes and reloads
// inside the loop.  Taken when both lists have at most KL_FIX_NCK chunks.
template <bool PROF, bool SEGC, bool GB = false, bool FIX = false>
__global__ __launch_bounds__(KL_LOOP_THREADS) void k_kl_swap_loop(KLDev d, int limit, ek_swap* __restrict__ log,
                                                                  long long cap, KLOut* __restrict__ out) {
    constexpr int NW = KL_LOOP_THREADS / 64;
    // positions per chunk key: larger chunks for the off-chip-bitmap form (fewer
    // keys for the selection to reduce; kl_loop_form)
    constexpr int CH = GB ? KL_CHUNK_GB : KL_CHUNK;
    // roles: W_W the pair gain; E_PARTS waves per chunk rescan node1's chunk
    // (waves W_EA, W_EA-1, ...) and E_PARTS node2's (W_EB, W_EB-1, ...);
    // waves 0 .. NG-1 run the gain updates
    constexpr int E_PARTS = KL_E_PARTS, NQ_E = CH / 64 / E_PARTS;
    constexpr int W_W = NW - 1, W_EA = NW - 2, W_EB = W_EA - E_PARTS, NG = W_EB - E_PARTS + 1;
    constexpr int W_PF = W_W;  // also runs P, the prefetch of the provisional next pair
    constexpr int W_FLIP = W_EA - 1;  // flips the side / lock bitmaps after barrier 1 (an early-rescan wave)
    static_assert(NG == KL_LOOP_THREADS / 64 - 1 - 2 * KL_E_PARTS, "kl_loop_lds_bytes reserves staging for NG gain waves");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // no static LDS: keeps it 16-B aligned
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int half = lane >> 5, hl = lane & 31;
    const int nsel = FIX ? KL_FIX_NCK : kl_sel_pad(d.nck0, d.nck1);
    const int words = (d.n + 31) / 32;
    const int lc0 = FIX ? KL_FIX_NCK : d.nck0, lc1 = FIX ? KL_FIX_NCK : d.nck1;  // the carve's chunk counts
    // LDS carve (kl_loop_lds_bytes): 16-B records first, then 8-B, then 4-B
    KLInfo* ci0 = reinterpret_cast<KLInfo*>(smem);  // chunk winners' descriptors
    KLInfo* ci1 = ci0 + lc0;
    KLInfo* it_info = ci1 + lc1;  // per updated row: {node, rowptr, len, position}
    KLInfo* er_info = it_info + KL_ITEM_CAP;  // [2][E_PARTS] early-rescan winners
    KLInfo* ab_info = er_info + 2 * E_PARTS;  // [2][KL_AB_CAP] updated rows in node1's / node2's chunk
    KLInfo* nx_info = ab_info + 2 * KL_AB_CAP;  // [2] the next pair's descriptors, published by P (EK_KL_NEXT)
    int4* sg_stage = reinterpret_cast<int4*>(nx_info + 2);  // [NG][KL_STAGE_ROWS][KL_STAGE_ROW] G1 staging
    u64* ck0 = reinterpret_cast<u64*>(sg_stage + NG * KL_STAGE_ROWS * KL_STAGE_ROW);  // chunk keys (zero-padded to nsel)
    u64* ck1 = ck0 + nsel;
    u64* ckn0 = ck1 + nsel;  // shadow keys: G1 merges risen keys here, G2 publishes them
    u64* ckn1 = ckn0 + lc0;
    u64* it_key = ckn1 + lc1;           // per updated row: its new key
    u64* er_key = it_key + KL_ITEM_CAP;     // [2][E_PARTS] early-rescan keys
    u64* ab_key = er_key + 2 * E_PARTS;     // [2][KL_AB_CAP] their new keys
    u64* nx_key = ab_key + 2 * KL_AB_CAP;   // [2] the next pair's keys, published by P
    int* dtag0 = reinterpret_cast<int*>(nx_key + 2);  // iteration that tagged a late rescan
    int* dtag1 = dtag0 + lc0;
    int* ctag0 = dtag1 + lc1;  // iteration that claimed it
    int* ctag1 = ctag0 + lc0;
    int* it_cs = ctag1 + lc1;  // per updated row: list << 31 | chunk (-1: locked)
    int* s_stop = it_cs + KL_ITEM_CAP;  // [4], by iteration parity
    // rows appended to ab_* by this swap's G1, per list: [0..1], reset by
    // G2a after its read.  With EK_KL_NEXT, [2][2] by iteration parity: G2a
    // (and P) read this swap's pair and G2a zeroes the other, which the next
    // swap's G1 fills (so P never reads a reset count)
    int* ab_cnt = s_stop + 4;
    int* nx_ok = ab_cnt + 4;  // [4]: [0] = 1 when P published the next pair
    // (FIX: the weight table at its fixed offset, then the bitmaps)
    uint32_t* s_side = GB ? reinterpret_cast<uint32_t*>(d.locked)
                     : FIX ? reinterpret_cast<uint32_t*>(nx_ok + 4 + KL_WDICT_CAP)
                           : reinterpret_cast<uint32_t*>(nx_ok + 4);
    uint32_t* s_lock = s_side + words;
    float* s_wd = (GB || FIX) ? reinterpret_cast<float*>(nx_ok + 4) : reinterpret_cast<float*>(s_lock + words);  // weight table (SEGC)
    auto bits_at = [&](const uint32_t* p) -> uint32_t {  // a bitmap word (GB: at the L2)
        if constexpr (GB) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else return *p;
    };
    if constexpr (SEGC)
        for (int i = tid; i < d.nwd; i += KL_LOOP_THREADS) s_wd[i] = d.wdict[i];
    for (int i = tid; i < nsel; i += KL_LOOP_THREADS) {
        ck0[i] = i < d.nck0 ? d.ckey0[i] : 0ull;
        ck1[i] = i < d.nck1 ? d.ckey1[i] : 0ull;
    }
    for (int i = tid; i < d.nck0; i += KL_LOOP_THREADS) {
        ckn0[i] = d.ckey0[i];
        ci0[i] = d.cinfo0[i];
        dtag0[i] = ctag0[i] = -1;
    }
    for (int i = tid; i < d.nck1; i += KL_LOOP_THREADS) {
        ckn1[i] = d.ckey1[i];
        ci1[i] = d.cinfo1[i];
        dtag1[i] = ctag1[i] = -1;
    }
    for (int i = tid; i < words; i += KL_LOOP_THREADS) {
        if constexpr (GB) {
            __hip_atomic_store(s_side + i, side_word(d.side_init, d.n, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(s_lock + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            s_side[i] = side_word(d.side_init, d.n, i);
            s_lock[i] = 0u;
        }
    }
    if constexpr (GB) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the bitmaps stored before the barrier
    if (tid < 4) s_stop[tid] = tid == 3 ? -1 : 0;
    if (tid < 4) ab_cnt[tid] = 0;
    if (tid < 4) nx_ok[tid] = 0;  // the first swap selects
    __syncthreads();
    float cut = *d.cut0, best = cut;  // loop-carried scalars: the W wave's lane 0 only
    long long best_it = 0, it = 0;
    unsigned term = 0;
    unsigned long long tph[12] = {}, tstamp = 0;  // diagnostic build only (PROF)
    // P (wave W_PF): the provisional next pair's descriptor, read before
    // barrier 2, and the lines its rows' loads touched (consumed one swap
    // later, after that wave's own rescan loads, so nothing waits for them)
    int4 pf_inf = make_int4(0, 0, 0, 0);
    int4 pf_seg = make_int4(0, 0, 0, 0), pf_seg2 = make_int4(0, 0, 0, 0), pf_aux = make_int4(0, 0, 0, 0);
    int pf_col = 0;
    float pf_w = 0.0f;
    uint32_t pf_sink = 0u;
    unsigned long long pf_hit_a = 0, pf_hit_b = 0;  // PROF
    const unsigned long long c_start = PROF ? __builtin_amdgcn_s_memtime() : 0ull;
    const unsigned long long r_start = PROF ? __builtin_amdgcn_s_memrealtime() : 0ull;
    auto stamp = [&](int ph) {
        if constexpr (PROF) {
            if (tid == 0) {
                const unsigned long long t = __builtin_amdgcn_s_memrealtime();
                if (ph >= 0) tph[ph] += t - tstamp;
                tstamp = t;
            }
        }
    };
    unsigned long long w_top = 0, w_arr1 = 0, w_arr2 = 0, w_g2a = 0, w_sel = 0, w_g2r = 0;  // PROF: this wave's timeline
    for (;; ++it) {
        stamp(-1);
        if constexpr (PROF) w_top = __builtin_amdgcn_s_memtime();
        if constexpr (EK_KL_PREFETCH) {
            if (wv == W_PF) {
                // P. touch the provisional pair's rows (one lane per row line:
                // lanes 0-31 node1's, 32-63 node2's; clamped addresses): the
                // W wave's weight lookup and the gain waves' segment and
                // descriptor loads after the selection then hit L2 instead
                // of the MALL
                const int rp = __builtin_amdgcn_readlane(pf_inf.y, 0), ln = __builtin_amdgcn_readlane(pf_inf.z, 0);
                const int rq = __builtin_amdgcn_readlane(pf_inf.y, 32), lq = __builtin_amdgcn_readlane(pf_inf.z, 32);
                const int r0 = half ? rq : rp, l0 = half ? lq : ln;
                if (l0 > 0) {
                    const int last = r0 + l0 - 1;
                    const int rs = min(r0 + hl, last);
                    if constexpr (SEGC) {
                        pf_seg = *reinterpret_cast<const int4*>(d.segc + size_t(rs) * KL_SEGC_PIECES);
                    } else if (d.seg) {
                        pf_seg = *reinterpret_cast<const int4*>(d.seg + size_t(rs) * KL_SEG_LANES);
                        pf_seg2 = *reinterpret_cast<const int4*>(d.seg + size_t(rs) * KL_SEG_LANES + KL_SEG_LANES / 2);
                    }
                    pf_aux = *reinterpret_cast<const int4*>(d.aux + min(r0 + 8 * hl, last));
                    pf_col = d.col[min(r0 + 32 * hl, last)];
                    pf_w = d.w[min(r0 + 32 * hl, last)];
                }
            }
        }
#if EK_G1_DRAIN
        // (lab) the gain waves wait for their previous gain stores here, beside
        // the selection, so the row loads after it wait for nothing older
        if (wv < NG) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#endif
        // S. selection (cKL.cpp:341-355): the pair P published before barrier
        // 2 (one LDS round trip), or else lanes 0-31 reduce remain[0]'s keys,
        // 32-63 remain[1]'s; identical in every wave
        u64 k0 = 0ull, k1 = 0ull;
        v4i dA = v4i{0, 0, 0, 0}, dB = v4i{0, 0, 0, 0};
        bool sel = true;
        if constexpr (EK_KL_NEXT) {
            const int ok = nx_ok[0];
            const u64 nk0 = nx_key[0], nk1 = nx_key[1];
            const v4i ni0 = *reinterpret_cast<const v4i*>(nx_info), ni1 = *reinterpret_cast<const v4i*>(nx_info + 1);
            if (__builtin_amdgcn_readfirstlane(ok)) {
                sel = false;
                k0 = readlane_u64(nk0, 0);
                k1 = readlane_u64(nk1, 0);
                dA = v4i{__builtin_amdgcn_readfirstlane(ni0.x), __builtin_amdgcn_readfirstlane(ni0.y),
                         __builtin_amdgcn_readfirstlane(ni0.z), 0};
                dB = v4i{__builtin_amdgcn_readfirstlane(ni1.x), __builtin_amdgcn_readfirstlane(ni1.y),
                         __builtin_amdgcn_readfirstlane(ni1.z), 0};
            }
        }
        if (sel) {
            u64 k = 0ull;
            // 8 keys per lane read together (clamped index: duplicates do not
            // change a max); one read per trip waited for each LDS round trip
            const u64* ck = half ? ck1 : ck0;
            if (nsel <= 4 * 32) {  // up to 128 chunks a list (~130k positions): 4 keys a lane
                u64 kv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) kv[u] = ck[min(hl + 32 * u, nsel - 1)];
#pragma unroll
                for (int u = 0; u < 4; ++u) k = kv[u] > k ? kv[u] : k;
            } else {
                for (int c0 = hl; c0 < nsel; c0 += 8 * 32) {
                    u64 kv[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) kv[u] = ck[min(c0 + 32 * u, nsel - 1)];
#pragma unroll
                    for (int u = 0; u < 8; ++u) k = kv[u] > k ? kv[u] : k;
                }
            }
            k = half_max_u64(k);
            k0 = readlane_u64(k, 0);
            k1 = readlane_u64(k, 32);
        }
        if (k0 == 0ull || k1 == 0ull) break;  // cKL.cpp:357,387-388 (identical in every wave)
        const int posA = int(~uint32_t(k0 & 0xffffffffull)), posB = int(~uint32_t(k1 & 0xffffffffull));
        const int cA = posA / CH, cB = posB / CH;
        if (sel) {
            dA = *reinterpret_cast<const v4i*>(ci0 + cA);
            dB = *reinterpret_cast<const v4i*>(ci1 + cB);
        }
        const int A = dA.x, pa = dA.y, la = dA.z, B = dB.x, pb = dB.y, lb = dB.z;
        if constexpr (PROF && EK_KL_PREFETCH) {  // how often the provisional pair was the pair
            if (wv == W_PF) {
                pf_hit_a += __builtin_amdgcn_readlane(pf_inf.x, 0) == A && __builtin_amdgcn_readlane(pf_inf.z, 0) > 0;
                pf_hit_b += __builtin_amdgcn_readlane(pf_inf.x, 32) == B && __builtin_amdgcn_readlane(pf_inf.z, 32) > 0;
            }
        }
        stamp(0);
        if constexpr (PROF) {
            if (A == -7) s_stop[2] = 0;  // keeps the descriptor read ahead of the stamp
            w_sel += __builtin_amdgcn_s_memtime() - w_top;
        }
        // swap + erase (swip, cKL.cpp:274-286): the bitmaps are flipped after
        // the first barrier (G2, W wave); until then every lookup reads the
        // pre-swap bitmaps and applies the swap itself: node1 and node2 (never
        // equal) change side and become locked.
        auto side_now = [&](int x) -> bool {
            return (((bits_at(s_side + (x >> 5)) >> (x & 31)) & 1u) != 0) ^ (x == A) ^ (x == B);
        };
        auto locked_now = [&](int x) -> bool {
            return ((bits_at(s_lock + (x >> 5)) >> (x & 31)) & 1u) || x == A || x == B;
        };
        const int tot = la + lb;
        const int tag = int(it);
        const int abp = EK_KL_NEXT ? (tag & 1) * 2 : 0;  // this swap's short-list counts (ab_cnt)
        if (wv == W_W) {
            // W. w(A,B) (getEdgeWeight, cKL.cpp:75-82) and the pair gain (cKL.cpp:360-386)
            float gA = 0.f, gB = 0.f;
            if (lane == 0) {
                gA = d.gp0[posA];
                gB = d.gp1[posB];
            }
            float wab = 0.0f;
            bool found = false;
            for (int i = lane; i < la; i += 64)
                if (d.col[pa + i] == B) {
                    wab = d.w[pa + i];
                    found = true;
                }
            const u64 bal = __ballot(found);
            if (bal) wab = __shfl(wab, __ffsll((long long)bal) - 1, 64);
            if (lane == 0) {
                d.gp0[posA] = __builtin_nanf("");
                d.gp1[posB] = __builtin_nanf("");
                const float gain = gA - gB - 2.0f * wab;
                cut -= gain;
                if (cut < best) {
                    best = cut;
                    best_it = it + 1;
                }
                if (it < cap)
                    log[it] = ek_swap{uint32_t(it + 1), uint32_t(A), uint32_t(B), gA, gB, gain, cut, 0u};
                int stop = 0;
                if (gain <= 0.0f) {
                    if (++term > unsigned(limit)) stop = 1;
                } else {
                    term = 0;
                }
                if (it + 1 >= d.n0 || it + 1 >= d.n1) stop = 1;  // a remain[] list is exhausted
                s_stop[it & 1] = stop;
            }
            if constexpr (EK_KL_PREFETCH)
                pf_sink ^= uint32_t(pf_seg.x ^ pf_seg.w ^ pf_seg2.x ^ pf_aux.x ^ pf_col) ^ __float_as_uint(pf_w);
        } else if (wv > W_EB - E_PARTS) {
            // E. early rescan of the chunk node1 (node2) leaves, E_PARTS waves
            // each taking a contiguous part of it
            const int s = wv <= W_EB ? 1 : 0, part = (s ? W_EB : W_EA) - wv;
            const int p0 = (s ? cB : cA) * CH + part * NQ_E * 64;
            // (with both trips' 2 KB a wave instead of 10 KB, the gain-update
            // waves' row loads no longer need a head start: EK_E_SLEEP 0)
            if constexpr (EK_E_SLEEP > 0) __builtin_amdgcn_s_sleep(EK_E_SLEEP);
            KLInfo info;
            bool mine;
#if EK_E_TWO_TRIPS
            const u64 kk = s ? chunk_rescan2<NQ_E>(d.gp1, d.pinfo1, 1, p0, posB, lane, &info, &mine)
                             : chunk_rescan2<NQ_E>(d.gp0, d.pinfo0, 0, p0, posA, lane, &info, &mine);
#else
            const u64 kk = s ? chunk_rescan1<NQ_E>(d.gp1, d.pinfo1, 1, p0, posB, lane, &info, &mine)
                             : chunk_rescan1<NQ_E>(d.gp0, d.pinfo0, 0, p0, posA, lane, &info, &mine);
#endif
            if (mine) {
                er_key[s * E_PARTS + part] = kk;
                er_info[s * E_PARTS + part] = info;
            }
        } else {
            // G1. gains of N(A) u N(B) (updateAffectedNodeGains, cKL.cpp:253-272):
            // one lane per row; the neighbour's descriptor {node, rowptr, len,
            // plist} (aux) and its first 32 {col, w} entries (seg) are both
            // addressed by the CSR position alone, so every load of the row is
            // issued at once; the sums run strictly in row order, the
            // zero-weight padding of short segments adds exact zeros
            // lanes per row: 8 for plain segments (2 pieces each), 4 for coded
            // ones (2 pieces each): 16 rows per wave, 48 per pass over the
            // three gain waves, so 0.1 % of the swaps (tot > 48) need a second
            // pass instead of 11 % (tot > 24) at ibm18 shape
            constexpr int LPR = SEGC ? 4 : 8, RPW = 64 / LPR;
            int4* stage = sg_stage + wv * KL_STAGE_ROWS * KL_STAGE_ROW;  // this wave's rows x KL_SEG_LANES pieces (+1 pad)
            for (int i0 = wv * RPW; i0 < tot; i0 += NG * RPW) {
                // LPR lanes per row, each loading 16-B pieces j8, j8 + LPR, ... of
                // the row's inline segment: each instruction touches each 128-B
                // line once.  (One lane loading all pieces of a line issues them
                // as separate instructions on the same line, and each waits for
                // the previous one's miss: serial L2 trips.)
                constexpr int PPL = (SEGC ? KL_SEGC_PIECES : KL_SEG_LANES) / LPR;  // pieces per lane
                const int gi = i0 + lane / LPR, j8 = lane % LPR, srow = lane / LPR;
                const int pg = gi < tot ? (gi < la ? pa + gi : pb + gi - la) : pa;
                int4 piece[PPL];
                if constexpr (SEGC) {  // pieces of 4 coded entries
#pragma unroll
                    for (int r = 0; r < PPL; ++r)
                        piece[r] = *reinterpret_cast<const int4*>(d.segc + size_t(pg) * KL_SEGC_PIECES + j8 + LPR * r);
                } else {
#pragma unroll
                    for (int r = 0; r < PPL; ++r)
                        piece[r] = d.seg ? *reinterpret_cast<const int4*>(d.seg + size_t(pg) * KL_SEG_LANES + j8 + LPR * r)
                                         : make_int4(0, 0, 0, 0);
                }
                const int4 a = j8 == 0 ? *reinterpret_cast<const int4*>(d.aux + pg) : make_int4(0, 0, 0, 0);
                if constexpr (PROF) {
                    if (tid == 0 && (piece[0].x == -12345 || a.x == -12345)) s_stop[2] = 0;  // waits for the loads
                }
                stamp(10);
                v2f ie_seg = {0.0f, 0.0f};  // SEGC: the row's inline-segment sums (internal, external)
                if constexpr (SEGC) {
                    // piece q = j8 + LPR*r holds entries 4q .. 4q+3.  Each lane
                    // decodes its entries' (internal, external) contributions;
                    // the sums then run strictly in row order through the row's
                    // quad of lanes: at step t (entries 4t .. 4t+3) the lane
                    // holding them adds its four, and a DPP quad broadcast hands
                    // the pair to the next step.  No LDS staging round trip.
                    const uint32_t cmask = (1u << d.wcolbits) - 1u;
                    v2f cc[PPL][4];
#pragma unroll
                    for (int r = 0; r < PPL; ++r) {
                        const uint32_t wv4[4] = {uint32_t(piece[r].x), uint32_t(piece[r].y), uint32_t(piece[r].z),
                                                 uint32_t(piece[r].w)};
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const float wk = s_wd[wv4[k] >> d.wcolbits];
                            const bool ek = side_now(int(wv4[k] & cmask));
                            cc[r][k] = v2f{ek ? 0.0f : wk, ek ? wk : 0.0f};
                        }
                    }
                    // a block of 4 entries no row of this wave reaches ends the
                    // chain (the zero padding would add exact zeros)
                    const int lenq = a.z;  // (the row's first lane; 0 in the others)
#pragma unroll
                    for (int st = 0; st < 4 * PPL; ++st) {
                        if (!__ballot(lenq > 4 * st)) break;
                        v2f x = ie_seg;
#pragma unroll
                        for (int k = 0; k < 4; ++k) x += cc[st / 4][k];  // v_pk_add_f32, in row order
                        ie_seg.x = quad_bcast(x.x, st % 4);
                        ie_seg.y = quad_bcast(x.y, st % 4);
                    }
                } else if (d.seg) {
                    // each lane looks up the sides of its own entries (4 LDS reads
                    // per wave instead of 32 serial ones by the summing lane) and
                    // stages every entry's (internal, external) contribution
#pragma unroll
                    for (int r = 0; r < PPL; ++r) {
                        const int4 pc = piece[r];
                        const bool e0 = side_now(pc.x);
                        const bool e1 = side_now(pc.z);
                        const float w0 = __int_as_float(pc.y), w1 = __int_as_float(pc.w);
                        stage[srow * KL_STAGE_ROW + j8 + LPR * r] =
                            make_int4(__float_as_int(e0 ? 0.0f : w0), __float_as_int(e0 ? w0 : 0.0f),
                                      __float_as_int(e1 ? 0.0f : w1), __float_as_int(e1 ? w1 : 0.0f));
                    }
                }
                stamp(11);
                if (j8 != 0 || gi >= tot) continue;  // the row's first lane sums it
                const int i = gi;
                int4 sg[KL_SEG_LANES];  // per entry pair: (internal, external) contributions
                if (!SEGC && d.seg) {
#pragma unroll
                    for (int j = 0; j < KL_SEG_LANES; ++j) sg[j] = stage[srow * KL_STAGE_ROW + j];
                }
                const int u = a.x, rp = a.y, len = a.z;
                const bool act = !locked_now(u);
                // the row's list, position, chunk and that chunk's current key
                // depend on the descriptor only: read ahead of the sums
                const uint32_t pl = uint32_t(a.w);
                const int ls = int(pl >> 31), pp = int(pl & 0x7fffffffu), c = pp / CH;
                const bool ab = ls ? c == cB : c == cA;  // node1's / node2's chunk: resolved in G2
                const u64 K = (ls ? ck1 : ck0)[c];       // stable until the barrier
                stamp(6);
                float internal = 0.0f, external = 0.0f;
                {  // summed whether or not u is locked: a branch on `act` would let the
                   // compiler sink the segment loads behind the descriptor's round trip
                    int q = 0;
                    if constexpr (SEGC) {
                        internal = ie_seg.x;
                        external = ie_seg.y;
                        q = 2 * KL_SEG_LANES;
                    } else if (d.seg) {
                        // 8 entries per block; a block no row of this wave reaches
                        // is skipped as a whole (wave-uniform branch): the loop is
                        // issue-bound, and the zero padding would add exact zeros.
                        // (internal, external) advance together in one packed fp32
                        // add per entry (v_pk_add_f32: two IEEE fp32 adds, the same
                        // bits as two v_add_f32), each strictly in row order
                        v2f ie = {0.0f, 0.0f};
#pragma unroll
                        for (int b = 0; b < KL_SEG_LANES / 4; ++b) {
                            if (!__ballot(len > 8 * b)) break;
#pragma unroll
                            for (int j = 4 * b; j < 4 * b + 4; ++j) {  // strictly in row order
                                ie += v2f{__int_as_float(sg[j].x), __int_as_float(sg[j].y)};
                                ie += v2f{__int_as_float(sg[j].z), __int_as_float(sg[j].w)};
                            }
                        }
                        internal = ie.x;
                        external = ie.y;
                        q = 2 * KL_SEG_LANES;
                    }
                    if constexpr (PROF) {
                        if (q < len) atomicAdd(&s_stop[2], 1);
                    }
                    for (; q < len; q += 16) {  // beyond the inline segment: 16 loads in flight per pass
                        int cc[16];
                        float ww[16];
#pragma unroll
                        for (int k2 = 0; k2 < 16; ++k2) {  // col/w carry 16 zero entries of tail padding
                            cc[k2] = d.col[rp + q + k2];
                            ww[k2] = q + k2 < len ? d.w[rp + q + k2] : 0.0f;
                        }
#pragma unroll
                        for (int k2 = 0; k2 < 16; ++k2) {
                            cc[k2] = q + k2 < len ? cc[k2] : 0;
                            const bool e = side_now(cc[k2]);
                            internal += e ? 0.0f : ww[k2];
                            external += e ? ww[k2] : 0.0f;
                        }
                    }
                }
                if constexpr (PROF) {
                    if (tid == 0 && internal == -1.0f) s_stop[2] = 0;  // keeps the sums ahead of the stamp
                }
                stamp(7);
                int cs = -1;
                u64 kn = 0ull;
                KLInfo inf{0, 0, 0, 0};
                if (act) {
                    const float g = external - internal;
                    const int s = ls;
                    (s ? d.gp1 : d.gp0)[pp] = g;
                    kn = key_max(s ? -g : g, pp);  // = key_min(g, pp) for list 1, without a branch
                    if (ab) {  // node1's / node2's chunk: resolved by G2a from this short list
                        const int slot = atomicAdd(&ab_cnt[abp + s], 1);
                        if (slot < KL_AB_CAP) {
                            ab_key[s * KL_AB_CAP + slot] = kn;
                            ab_info[s * KL_AB_CAP + slot] = KLInfo{u, rp, len, pp};
                        }
                    } else {
                        if (uint32_t(~uint32_t(K & 0xffffffffull)) == uint32_t(pp) && kn < K) {
                            (s ? dtag1 : dtag0)[c] = tag;  // the winner fell: rescan
                            s_stop[3] = tag;
                        } else if (kn > K) {
                            atomicMax(&(s ? ckn1 : ckn0)[c], kn);
                            if (i >= KL_ITEM_CAP) {  // no LDS slot for its descriptor
                                (s ? dtag1 : dtag0)[c] = tag;
                                s_stop[3] = tag;
                            }
                        }
                    }
                    cs = int((pl & 0x80000000u) | uint32_t(c));
                    inf = KLInfo{u, rp, len, pp};
                }
                if (i < KL_ITEM_CAP) {
                    it_key[i] = kn;
                    it_cs[i] = cs;
                    it_info[i] = inf;
                }
            }
        }
        stamp(1);
        if constexpr (PROF) w_arr1 += __builtin_amdgcn_s_memtime() - w_top;
        __syncthreads();  // (1) gains, early rescans, merged keys and tags visible
        stamp(2);
        // the last iteration that tagged a chunk, read first so its round trip
        // overlaps the G2a / P / G2b reads (G2c runs only when it is this one)
        const bool any_tag = s_stop[3] == tag;
        // G2a. node1's and node2's chunks: one wave (lanes 0-31 list 0, 32-63
        // list 1), beside G2b/G2c in the others
        if (wv == W_EA) {
            const int s = half, cS = s ? cB : cA;
            // one LDS round trip: the early rescan's parts (keys and winners),
            // the list of updated rows in the chunk and their count
            u64 rk[E_PARTS];
            v4i rf[E_PARTS];
#pragma unroll
            for (int q = 0; q < E_PARTS; ++q) {
                rk[q] = er_key[s * E_PARTS + q];
                rf[q] = *reinterpret_cast<const v4i*>(er_info + s * E_PARTS + q);
            }
            // (the list entries are read whatever the count, so all of it is one
            // round trip; slots beyond the count hold stale rows and are masked)
            const int cnt = ab_cnt[abp + s];
            const int hs = hl < KL_AB_CAP ? hl : KL_AB_CAP - 1;
            const u64 bk_raw = ab_key[s * KL_AB_CAP + hs];
            const v4i bf = *reinterpret_cast<const v4i*>(ab_info + s * KL_AB_CAP + hs);
            const bool have = hl < cnt && hl < KL_AB_CAP;
            const u64 bk = have ? bk_raw : 0ull;
            if (hl == 0) ab_cnt[(EK_KL_NEXT ? 2 - abp : 0) + s] = 0;  // after the read (in order within the wave), or the next swap's pair; G1 appends after barrier 2
            u64 R = rk[0];  // the early rescan's key: the best of its parts
            v4i Rf = rf[0];
#pragma unroll
            for (int q = 1; q < E_PARTS; ++q) {  // component selects (a conditional vector copy went to scratch)
                const bool b = rk[q] > R;
                R = b ? rk[q] : R;
                Rf.x = b ? rf[q].x : Rf.x;
                Rf.y = b ? rf[q].y : Rf.y;
                Rf.z = b ? rf[q].z : Rf.z;
                Rf.w = b ? rf[q].w : Rf.w;
            }
            const int Rpos = int(~uint32_t(R & 0xffffffffull));  // meaningless when R == 0 (never matched)
            // the early rescan saw the old gain of an updated row that then fell
            const bool stale = have && R != 0ull && bf.w == Rpos && bk < R;
            if constexpr (PROF) {
                if (stale && bf.x == -7) s_stop[2] = 0;  // keeps the reads ahead of the stamp
                w_g2r += __builtin_amdgcn_s_memtime() - w_top;
            }
            const u64 hmask = s ? 0xffffffff00000000ull : 0x00000000ffffffffull;
            const bool st = (__ballot(stale) & hmask) != 0ull || cnt > KL_AB_CAP;
            u64 m = 0ull;
            if (__ballot(cnt > 0)) m = half_max_u64(bk);  // (most swaps: no updated row in either chunk)
            if (!st) {
                // keys carry the position: at most one lane holds m
                if (m > R) {
                    if (have && bk == m) {
                        (s ? ck1 : ck0)[cS] = m;
                        (s ? ckn1 : ckn0)[cS] = m;
                        *reinterpret_cast<v4i*>((s ? ci1 : ci0) + cS) = bf;
                    }
                } else if (hl == 0) {
                    (s ? ck1 : ck0)[cS] = R;
                    (s ? ckn1 : ckn0)[cS] = R;
                    *reinterpret_cast<v4i*>((s ? ci1 : ci0) + cS) = Rf;
                }
            }
            // a stale early rescan (or more updated rows than the list
            // holds): full rescan now that every new gain (and node1/node2's NaN) is stored
            const bool stA = __builtin_amdgcn_readlane(int(st), 0) != 0, stB = __builtin_amdgcn_readlane(int(st), 32) != 0;
            if constexpr (PROF) {
                if (lane == 0) atomicAdd(&s_stop[2], 1000000 * (int(stA) + int(stB)));  // stale counts in the high digits
            }
            for (int q = 0; q < 2; ++q) {
                if (!(q ? stB : stA)) continue;
                KLInfo info;
                bool mine;
                const u64 kk = q ? chunk_rescan<CH>(d.gp1, d.pinfo1, 1, cB, -1, lane, &info, &mine)
                                 : chunk_rescan<CH>(d.gp0, d.pinfo0, 0, cA, -1, lane, &info, &mine);
                if (mine) {
                    (q ? ck1 : ck0)[q ? cB : cA] = kk;
                    (q ? ckn1 : ckn0)[q ? cB : cA] = kk;
                    (q ? ci1 : ci0)[q ? cB : cA] = info;
                }
            }
        }
        stamp(3);
        if constexpr (PROF) w_g2a += __builtin_amdgcn_s_memtime() - w_top;
        if (wv == W_FLIP && lane == 0) {  // the swap itself, for the next swap's lookups (barrier 2)
            // LDS atomics without return: four independent operations instead
            // of four dependent read-modify-write round trips
            if constexpr (GB) {  // at the L2, drained before barrier 2
                __hip_atomic_fetch_or(s_side + (A >> 5), 1u << (A & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_and(s_side + (B >> 5), ~(1u << (B & 31)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_or(s_lock + (A >> 5), 1u << (A & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_or(s_lock + (B >> 5), 1u << (B & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            } else {
                atomicOr(&s_side[A >> 5], 1u << (A & 31));
                atomicAnd(&s_side[B >> 5], ~(1u << (B & 31)));
                atomicOr(&s_lock[A >> 5], 1u << (A & 31));
                atomicOr(&s_lock[B >> 5], 1u << (B & 31));
            }
        }
        if constexpr (EK_KL_NEXT) {
            if (wv == W_PF) {
                // P. the next pair, exactly, from the state G2 is publishing
                // (beside it): per list the best of
                //  * the shadow keys of the chunks other than node1's /
                //    node2's: an untagged chunk's key IS its shadow key (G2b
                //    copies it), as every raise was merged into it by G1;
                //  * node1's / node2's chunk resolved as G2a resolves it: the
                //    early rescan against the updated rows in the chunk.
                // The winner's descriptor: the updated row holding the winning
                // key (the one G2b publishes), else the early rescan's winner,
                // else the chunk table's entry (neither G2a nor G2b writes it
                // this swap).  A tagged chunk, a stale early rescan, an
                // overflowing short list or more than 64 updated rows: nothing
                // published, the waves select after barrier 2.
                const int s = half, cS = s ? cB : cA, nck = s ? d.nck1 : d.nck0;
                const u64* ckn = s ? ckn1 : ckn0;
                u64 k = 0ull;
                for (int c0 = hl; c0 < nck; c0 += 4 * 32) {
                    u64 kv[4];  // all four reads in flight, then masked (no per-read branch)
#pragma unroll
                    for (int u = 0; u < 4; ++u) kv[u] = ckn[min(c0 + 32 * u, nck - 1)];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const u64 v = kv[u] & (min(c0 + 32 * u, nck - 1) == cS ? 0ull : ~0ull);
                        k = v > k ? v : k;
                    }
                }
                // the same round trip: the early rescan's parts, the short
                // list and its count, the updated rows (lane l: row l)
                u64 rk[E_PARTS];
                v4i rf[E_PARTS];
#pragma unroll
                for (int q = 0; q < E_PARTS; ++q) {
                    rk[q] = er_key[s * E_PARTS + q];
                    rf[q] = *reinterpret_cast<const v4i*>(er_info + s * E_PARTS + q);
                }
                const int cnt = ab_cnt[abp + s];
                const int hs = hl < KL_AB_CAP ? hl : KL_AB_CAP - 1;
                const u64 bk_raw = ab_key[s * KL_AB_CAP + hs];
                const v4i bf = *reinterpret_cast<const v4i*>(ab_info + s * KL_AB_CAP + hs);
                const int il = lane < tot ? lane : 0;
                const u64 ik = it_key[il];
                const int ics = it_cs[il];
                const v4i iinf = *reinterpret_cast<const v4i*>(it_info + il);
                const bool have = hl < cnt && hl < KL_AB_CAP;
                const u64 bk = have ? bk_raw : 0ull;
                u64 R = rk[0];
                v4i Rf = rf[0];
#pragma unroll
                for (int q = 1; q < E_PARTS; ++q) {
                    const bool b = rk[q] > R;
                    R = b ? rk[q] : R;
                    Rf.x = b ? rf[q].x : Rf.x;
                    Rf.y = b ? rf[q].y : Rf.y;
                    Rf.z = b ? rf[q].z : Rf.z;
                    Rf.w = b ? rf[q].w : Rf.w;
                }
                const int Rpos = int(~uint32_t(R & 0xffffffffull));
                const bool stale = have && R != 0ull && bf.w == Rpos && bk < R;
                const bool bad = any_tag || tot > 64 || __ballot(stale || cnt > KL_AB_CAP) != 0ull;
                const u64 m = __ballot(cnt > 0) ? half_max_u64(bk) : 0ull;
                const u64 kS = m > R ? m : R;
                k = kS > k ? kS : k;
                k = half_max_u64(k);
                const u64 kA = readlane_u64(k, 0), kB = readlane_u64(k, 32);
                // list-1 rows have bit 31 of it_cs set; -1 is a locked row
                const bool own = lane < tot && ics != -1;
                const u64 mA = __ballot(own && ics >= 0 && ik == kA), mB = __ballot(own && ics < 0 && ik == kB);
                const u64 mS = s ? mB : mA;
                v4i desc = Rf;
                if (mA) {
                    const int l = __ffsll((long long)mA) - 1;
                    const v4i t = v4i{__builtin_amdgcn_readlane(iinf.x, l), __builtin_amdgcn_readlane(iinf.y, l),
                                      __builtin_amdgcn_readlane(iinf.z, l), 0};
                    if (!s) desc = t;
                }
                if (mB) {
                    const int l = __ffsll((long long)mB) - 1;
                    const v4i t = v4i{__builtin_amdgcn_readlane(iinf.x, l), __builtin_amdgcn_readlane(iinf.y, l),
                                      __builtin_amdgcn_readlane(iinf.z, l), 0};
                    if (s) desc = t;
                }
                if (!mS && k != R && k != 0ull)  // an unchanged chunk's winner
                    desc = *reinterpret_cast<const v4i*>((s ? ci1 : ci0) + int(~uint32_t(k & 0xffffffffull)) / CH);
                if (hl == 0) {
                    nx_key[s] = k;
                    *reinterpret_cast<v4i*>(nx_info + s) = desc;
                }
                if (lane == 0) nx_ok[0] = bad ? 0 : 1;
                if constexpr (EK_KL_PREFETCH) pf_inf = make_int4(desc.x, desc.y, desc.z, 0);
            }
        } else if constexpr (EK_KL_PREFETCH) {
            if (wv == W_PF) {
                // P. provisional next pair (a prefetch hint, never a result):
                // per list the best shadow key outside node1's / node2's chunk
                // against that chunk's early rescan.  Its descriptor is read
                // now and used after barrier 2 (the bitmap flip runs in another
                // wave: the wait the compiler puts ahead of its LDS reads would
                // hold this one at barrier 2 for the load)
                const u64* ckn = half ? ckn1 : ckn0;
                const int nck = half ? d.nck1 : d.nck0, cS = half ? cB : cA;
                u64 k = 0ull;
                for (int c0 = hl; c0 < nck; c0 += 4 * 32) {
                    u64 kv[4];  // all four reads in flight, then masked (no per-read branch)
#pragma unroll
                    for (int u = 0; u < 4; ++u) kv[u] = ckn[min(c0 + 32 * u, nck - 1)];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const u64 v = kv[u] & (min(c0 + 32 * u, nck - 1) == cS ? 0ull : ~0ull);
                        k = v > k ? v : k;
                    }
                }
#pragma unroll
                for (int q = 0; q < E_PARTS; ++q) {
                    const u64 v = er_key[half * E_PARTS + q];
                    k = v > k ? v : k;
                }
                k = half_max_u64(k);
                pf_inf = make_int4(0, 0, 0, 0);
                if (k != 0ull && hl == 0)
                    pf_inf = *reinterpret_cast<const int4*>((half ? d.pinfo1 : d.pinfo0) + int(~uint32_t(k & 0xffffffffull)));
            }
        }
        // G2b. publish merged keys of the other untagged chunks (every item of
        // a chunk writes the same value) and the descriptor of the item that
        // won: the two early-rescan waves of list 1, from the item list (two
        // LDS round trips: the item, then the merged key and the chunk's tag).
        // Not the gain waves: the compiler puts waits for their gain stores'
        // acks ahead of register writes in this code (measured 2.20 -> 2.13 us
        // per swap at ibm18 shape).
        if (wv == W_EB || wv == W_EB - 1) {
            for (int i = (W_EB - wv) * 64 + lane; i < tot && i < KL_ITEM_CAP; i += 128) {
                const int cs = it_cs[i];
                const u64 kn = it_key[i];
                // a vector, not a KLInfo: the struct copied under a condition went
                // through scratch (and a vmcnt(0) wait) in every swap
                const int4 inf = *reinterpret_cast<const int4*>(it_info + i);
                if (cs == -1) continue;  // (list-1 chunk ids have bit 31 set: negative as int)
                const int s = int(uint32_t(cs) >> 31), c = cs & 0x7fffffff;
                const u64 kmerged = (s ? ckn1 : ckn0)[c];
                const int dt = (s ? dtag1 : dtag0)[c];
                if ((s ? c == cB : c == cA) || dt == tag) continue;
                (s ? ck1 : ck0)[c] = kmerged;
                if (kmerged == kn) *reinterpret_cast<int4*>((s ? ci1 : ci0) + c) = inf;
            }
        }
        // G2c. full rescans of the tagged chunks (one wave each, claimed once)
        for (int i = wv; any_tag && i < tot; i += NW) {
            int cs;
            if (i < KL_ITEM_CAP) cs = it_cs[i];
            else {  // beyond the LDS item list (hubs): rederive
                const int u = i < la ? d.col[pa + i] : d.col[pb + i - la];
                cs = locked_now(u) ? -1 : int((uint32_t(d.nd[u].c) & 0x80000000u) |
                                                                     ((uint32_t(d.nd[u].c) & 0x7fffffffu) / CH));
            }
            if (cs == -1) continue;
            const int s = int(uint32_t(cs) >> 31), c = cs & 0x7fffffff;
            if ((s ? dtag1 : dtag0)[c] != tag) continue;  // node1's / node2's chunks are never tagged
            int claimed = 0;
            if (lane == 0) claimed = atomicMax(&(s ? ctag1 : ctag0)[c], tag) < tag;
            if (!__shfl(claimed, 0, 64)) continue;
            if constexpr (PROF) {
                if (lane == 0) atomicAdd(&s_stop[2], 1);  // late rescans in the low digits
            }
            KLInfo info;
            bool mine;
            const u64 kk = s ? chunk_rescan<CH>(d.gp1, d.pinfo1, 1, c, -1, lane, &info, &mine)
                             : chunk_rescan<CH>(d.gp0, d.pinfo0, 0, c, -1, lane, &info, &mine);
            if (mine) {
                (s ? ck1 : ck0)[c] = kk;
                (s ? ckn1 : ckn0)[c] = kk;
                (s ? ci1 : ci0)[c] = info;
            }
        }
        stamp(4);
        if constexpr (PROF) w_arr2 += __builtin_amdgcn_s_memtime() - w_top;
        __syncthreads();  // (2) keys visible to the next selection
        stamp(5);
        if (s_stop[it & 1]) {
            ++it;
            break;
        }
    }
    __syncthreads();
    for (int u = tid; u < d.n; u += KL_LOOP_THREADS) d.side[u] = uint8_t((bits_at(s_side + (u >> 5)) >> (u & 31)) & 1u);
    if (EK_KL_PREFETCH && wv == W_PF && lane == 0 && pf_sink == 0x5a5a5a5au) out->prof[12] = 1ull;  // keeps P's loads
    if (lane == 0 && (NW <= 8 || wv < 8)) {  // (KLOut::warr holds 8 waves' stamps)
        out->warr[wv] = w_arr1;
        out->warr[8 + wv] = w_arr2;
        out->warr[16 + wv] = w_g2a;
        out->warr[24 + wv] = w_sel;
        out->warr[32 + wv] = w_g2r;
        if (wv == W_PF) {
            out->warr[40] = pf_hit_a;
            out->warr[41] = pf_hit_b;
        }
    }
    if (wv == W_W && lane == 0) {
        out->iterations = it;
        out->best_iter = best_it;
        out->initial_cut = *d.cut0;
        out->best_cut = best;
        out->final_cut = cut;
        out->status = 2u;
    }
    if (tid == 0) {  // phase stamps are taken by thread 0
        if constexpr (PROF) {
            tph[8] = 100ull * (unsigned long long)(s_stop[2] / 1000000);
            tph[9] = 100ull * (unsigned long long)(s_stop[2] % 1000000);
        }
        for (int i = 0; i < 12; ++i) out->prof[i] = tph[i];
        out->prof[14] = PROF ? __builtin_amdgcn_s_memtime() - c_start : 0ull;
        out->prof[15] = PROF ? __builtin_amdgcn_s_memrealtime() - r_start : 0ull;
    }
}


// ---------------------------------------------------------------------------
// The swap loop with consecutive swaps overlapped (k_kl_swap_pipe; VERDICT r5
// next-1).  The per-swap work, the LDS state and the parity rules are those of
// k_kl_swap_loop; the schedule differs:
//  * barrier 2 is a counter in LDS, not s_barrier.  The gain waves only arrive
//    at it (once their reads of this swap's state are done) and never wait at
//    it; the other waves wait for all eight arrivals before the selection;
//  * right after barrier 1 each gain wave takes the next pair exactly from
//    the state G2 is publishing (the EK_KL_NEXT rule above: the shadow keys of
//    the other chunks, node1's / node2's chunks resolved as G2a resolves them,
//    the winners' descriptors from the updated rows, the early rescan or the
//    chunk table), loads that pair's neighbour rows and sums their gains into
//    registers — while G2 and the next selection run in the other waves;
//  * the W wave publishes the selection's pair (keys and descriptors, one LDS
//    flag); a gain wave whose pair has the same keys commits its sums (gain
//    stores, key merges, item lists) at once, otherwise it runs G1 on the
//    published pair (a tagged chunk, a stale early rescan, an overflowing short
//    list or more rows than one pass: no speculation).
// A node's gain is recomputed from its row and the current sides alone
// (cKL.cpp:253-272), so the sums are the same fp32 bits whenever they run:
// the sides are the bitmaps after this swap (its flip applied by hand, as it
// may still be in flight in the W_FLIP wave) with the next pair's two nodes
// swapped.  The keys carry the positions, so equal keys are the same pair.
// Every wait is a bounded poll: a wave that gives up raises an abort word the
// others poll as well, and the launch ends with status 3 (EK_EHIP on the host)
// instead of hanging.
// PROF: per-swap counters and shader-clock spans of gain wave 0, the W wave
// and the G2a wave (KLOut::prof, marker 0x9199 in [13]; printed by the host).
template <bool PROF, bool SEGC>
__global__ __launch_bounds__(KL_LOOP_THREADS) void k_kl_swap_pipe(KLDev d, int limit, ek_swap* __restrict__ log,
                                                                  long long cap, KLOut* __restrict__ out) {
    constexpr int NW = KL_LOOP_THREADS / 64;
    constexpr int E_PARTS = KL_E_PARTS, NQ_E = KL_CHUNK / 64 / E_PARTS;
    constexpr int W_W = NW - 1, W_EA = NW - 2, W_EB = W_EA - E_PARTS, NG = W_EB - E_PARTS + 1;
    constexpr int W_FLIP = W_EA - 1;
    constexpr int LPR = SEGC ? 4 : 8, RPW = 64 / LPR;
    constexpr int PPL = (SEGC ? KL_SEGC_PIECES : KL_SEG_LANES) / LPR;  // 16-B pieces per lane
    constexpr unsigned POLL_CAP = 1u << 22;                              // polls before a wait gives up
    static_assert(NG == KL_LOOP_THREADS / 64 - 1 - 2 * KL_E_PARTS, "kl_loop_lds_bytes reserves staging for NG gain waves");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int half = lane >> 5, hl = lane & 31;
    const int nsel = kl_sel_pad(d.nck0, d.nck1);
    const int words = (d.n + 31) / 32;
    // LDS carve: k_kl_swap_loop's (kl_loop_lds_bytes); nx_info / nx_key hold
    // the published pair, nx_ok the waits' words
    KLInfo* ci0 = reinterpret_cast<KLInfo*>(smem);
    KLInfo* ci1 = ci0 + d.nck0;
    KLInfo* it_info = ci1 + d.nck1;
    KLInfo* er_info = it_info + KL_ITEM_CAP;
    KLInfo* ab_info = er_info + 2 * E_PARTS;
    KLInfo* nx_info = ab_info + 2 * KL_AB_CAP;
    int4* sg_stage = reinterpret_cast<int4*>(nx_info + 2);
    u64* ck0 = reinterpret_cast<u64*>(sg_stage + NG * KL_STAGE_ROWS * KL_STAGE_ROW);
    u64* ck1 = ck0 + nsel;
    u64* ckn0 = ck1 + nsel;
    u64* ckn1 = ckn0 + d.nck0;
    u64* it_key = ckn1 + d.nck1;
    u64* er_key = it_key + KL_ITEM_CAP;
    u64* ab_key = er_key + 2 * E_PARTS;
    u64* nx_key = ab_key + 2 * KL_AB_CAP;
    int* dtag0 = reinterpret_cast<int*>(nx_key + 2);
    int* dtag1 = dtag0 + d.nck0;
    int* ctag0 = dtag1 + d.nck1;
    int* ctag1 = ctag0 + d.nck0;
    int* it_cs = ctag1 + d.nck1;
    int* s_stop = it_cs + KL_ITEM_CAP;  // [0..1] stop by parity, [3] the last tag
    int* ab_cnt = s_stop + 4;           // [2][2]: short-list counts by swap parity
    int* sync = ab_cnt + 4;  // [0] barrier-2 arrivals, [1] W's pair, [2] abort, [3] wave 0's speculative pair (iteration + 1)
    uint32_t* s_side = reinterpret_cast<uint32_t*>(sync + 4);
    uint32_t* s_lock = s_side + words;
    float* s_wd = reinterpret_cast<float*>(s_lock + words);
    // gain wave 0's speculative pair for waves 1 .. NG-1: [0..1] keys (0: none), [2..5] the two descriptors
    u64* sp = reinterpret_cast<u64*>((reinterpret_cast<uintptr_t>(s_wd + (SEGC ? d.nwd : 0)) + 15) & ~uintptr_t(15));
    if constexpr (SEGC)
        for (int i = tid; i < d.nwd; i += KL_LOOP_THREADS) s_wd[i] = d.wdict[i];
    for (int i = tid; i < nsel; i += KL_LOOP_THREADS) {
        ck0[i] = i < d.nck0 ? d.ckey0[i] : 0ull;
        ck1[i] = i < d.nck1 ? d.ckey1[i] : 0ull;
    }
    for (int i = tid; i < d.nck0; i += KL_LOOP_THREADS) {
        ckn0[i] = d.ckey0[i];
        ci0[i] = d.cinfo0[i];
        dtag0[i] = ctag0[i] = -1;
    }
    for (int i = tid; i < d.nck1; i += KL_LOOP_THREADS) {
        ckn1[i] = d.ckey1[i];
        ci1[i] = d.cinfo1[i];
        dtag1[i] = ctag1[i] = -1;
    }
    for (int i = tid; i < words; i += KL_LOOP_THREADS) {
        s_side[i] = side_word(d.side_init, d.n, i);
        s_lock[i] = 0u;
    }
    if (tid < 4) s_stop[tid] = tid == 3 ? -1 : 0;
    if (tid < 4) ab_cnt[tid] = 0;
    if (tid < 4) sync[tid] = 0;
    __syncthreads();
    float cut = *d.cut0, best = cut;  // loop-carried scalars: the W wave's lane 0 only
    long long best_it = 0, it = 0;
    unsigned term = 0;
    unsigned long long pc[12] = {};  // PROF counters / spans (this wave's)
    unsigned long long t_a = 0, t_b = 0;
    auto now = [&]() -> unsigned long long { return PROF ? __builtin_amdgcn_s_memtime() : 0ull; };
    const unsigned long long t_start = now();

    // ---- waits (bounded; the abort word ends every other wait too)
    auto aborted = [&]() -> bool { return __hip_atomic_load(&sync[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0; };
    auto give_up = [&]() { __hip_atomic_store(&sync[2], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    // barrier 2: this wave's LDS reads and writes of the swap are done
    auto arrive = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_fetch_add(&sync[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto wait_word = [&](int w, int target) -> bool {
        for (unsigned p = 0;; ++p) {
            const int v = __hip_atomic_load(&sync[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (__builtin_amdgcn_readfirstlane(v) >= target) break;
            if constexpr (EK_PIPE_SLEEP > 0) __builtin_amdgcn_s_sleep(EK_PIPE_SLEEP);  // (spare the CU's scalar issue)
            if ((p & 255u) == 255u) {  // (the abort word every 256 polls: one LDS round trip a poll)
                if (__builtin_amdgcn_readfirstlane(int(aborted()))) return false;
                if (p >= POLL_CAP) {
                    give_up();
                    return false;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        return true;
    };

    // ---- G1, split: the rows' loads and sums (no shared writes), then their commit.
    // One pass over rows i0 + lane / LPR of the pair's neighbour lists; side_fn /
    // lock_fn give the sides and locks the gains are computed under.  The row's
    // first lane (gi >= 0 on return) holds its descriptor and sums.
    auto g1_rows = [&](int i0, int pa, int la, int pb, int lb, auto&& side_fn, auto&& lock_fn, int& gi_o, int4& a_o,
                       float& in_o, float& ex_o, bool& act_o) {
        const int tot = la + lb;
        const int gi = i0 + lane / LPR, j8 = lane % LPR, srow = lane / LPR;
        int pg = gi < tot ? (gi < la ? pa + gi : pb + gi - la) : pa;
        pg = min(max(pg, 0), int(d.nnz) - 1);  // (a speculative descriptor never addresses outside the CSR)
        int4 piece[PPL];
        if constexpr (SEGC) {
#pragma unroll
            for (int r = 0; r < PPL; ++r)
                piece[r] = *reinterpret_cast<const int4*>(d.segc + size_t(pg) * KL_SEGC_PIECES + j8 + LPR * r);
        } else {
#pragma unroll
            for (int r = 0; r < PPL; ++r)
                piece[r] = d.seg ? *reinterpret_cast<const int4*>(d.seg + size_t(pg) * KL_SEG_LANES + j8 + LPR * r)
                                 : make_int4(0, 0, 0, 0);
        }
        const int4 a = j8 == 0 ? *reinterpret_cast<const int4*>(d.aux + pg) : make_int4(0, 0, 0, 0);
        v2f ie_seg = {0.0f, 0.0f};
        int4* stage = sg_stage + wv * KL_STAGE_ROWS * KL_STAGE_ROW;
        if constexpr (SEGC) {
            const uint32_t cmask = (1u << d.wcolbits) - 1u;
            v2f cc[PPL][4];
#pragma unroll
            for (int r = 0; r < PPL; ++r) {
                const uint32_t wv4[4] = {uint32_t(piece[r].x), uint32_t(piece[r].y), uint32_t(piece[r].z),
                                         uint32_t(piece[r].w)};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float wk = s_wd[wv4[k] >> d.wcolbits];
                    const bool ek = side_fn(int(wv4[k] & cmask));
                    cc[r][k] = v2f{ek ? 0.0f : wk, ek ? wk : 0.0f};
                }
            }
            const int lenq = a.z;
#pragma unroll
            for (int st = 0; st < 4 * PPL; ++st) {
                if (!__ballot(lenq > 4 * st)) break;
                v2f x = ie_seg;
#pragma unroll
                for (int k = 0; k < 4; ++k) x += cc[st / 4][k];  // in row order
                ie_seg.x = quad_bcast(x.x, st % 4);
                ie_seg.y = quad_bcast(x.y, st % 4);
            }
        } else if (d.seg) {
#pragma unroll
            for (int r = 0; r < PPL; ++r) {
                const int4 pc = piece[r];
                const bool e0 = side_fn(pc.x);
                const bool e1 = side_fn(pc.z);
                const float w0 = __int_as_float(pc.y), w1 = __int_as_float(pc.w);
                stage[srow * KL_STAGE_ROW + j8 + LPR * r] =
                    make_int4(__float_as_int(e0 ? 0.0f : w0), __float_as_int(e0 ? w0 : 0.0f),
                              __float_as_int(e1 ? 0.0f : w1), __float_as_int(e1 ? w1 : 0.0f));
            }
        }
        gi_o = -1;
        if (j8 != 0 || gi >= tot) return;  // the row's first lane sums it
        const int len = a.z, rp = a.y;
        float internal = 0.0f, external = 0.0f;
        int q = 0;
        if constexpr (SEGC) {
            internal = ie_seg.x;
            external = ie_seg.y;
            q = 2 * KL_SEG_LANES;
        } else if (d.seg) {
            int4 sg[KL_SEG_LANES];
#pragma unroll
            for (int j = 0; j < KL_SEG_LANES; ++j) sg[j] = stage[srow * KL_STAGE_ROW + j];
            v2f ie = {0.0f, 0.0f};
#pragma unroll
            for (int b = 0; b < KL_SEG_LANES / 4; ++b) {
                if (!__ballot(len > 8 * b)) break;
#pragma unroll
                for (int j = 4 * b; j < 4 * b + 4; ++j) {
                    ie += v2f{__int_as_float(sg[j].x), __int_as_float(sg[j].y)};
                    ie += v2f{__int_as_float(sg[j].z), __int_as_float(sg[j].w)};
                }
            }
            internal = ie.x;
            external = ie.y;
            q = 2 * KL_SEG_LANES;
        }
        for (; q < len; q += 16) {  // beyond the inline segment: 16 loads in flight per pass
            int cc[16];
            float ww[16];
            const int lim = int(d.nnz) - 1;  // (a speculative row stays inside the CSR)
#pragma unroll
            for (int k2 = 0; k2 < 16; ++k2) {
                cc[k2] = d.col[min(rp + q + k2, lim + 16)];  // col/w carry 16 zero entries of tail padding
                ww[k2] = q + k2 < len ? d.w[min(rp + q + k2, lim)] : 0.0f;
            }
#pragma unroll
            for (int k2 = 0; k2 < 16; ++k2) {
                cc[k2] = q + k2 < len ? cc[k2] : 0;
                const bool e = side_fn(cc[k2]);
                internal += e ? 0.0f : ww[k2];
                external += e ? ww[k2] : 0.0f;
            }
        }
        gi_o = gi;
        a_o = a;
        in_o = internal;
        ex_o = external;
        act_o = !lock_fn(a.x);
    };
    // the commit of one row (G1's writes): its gain, and its new key merged
    // into its chunk's shadow key, node1's / node2's short list or a tag
    auto g1_commit = [&](int gi, int4 a, float internal, float external, bool act, int cA, int cB, int tag,
                         int abp) {
        if (gi < 0) return;
        const int u = a.x, rp = a.y, len = a.z;
        const uint32_t pl = uint32_t(a.w);
        const int ls = int(pl >> 31), pp = int(pl & 0x7fffffffu), c = pp / KL_CHUNK;
        const bool ab = ls ? c == cB : c == cA;
        const u64 K = (ls ? ck1 : ck0)[c];
        int cs = -1;
        u64 kn = 0ull;
        KLInfo inf{0, 0, 0, 0};
        if (act) {
            const float g = external - internal;
            const int s = ls;
            (s ? d.gp1 : d.gp0)[pp] = g;
            kn = key_max(s ? -g : g, pp);
            if (ab) {
                const int slot = atomicAdd(&ab_cnt[abp + s], 1);
                if (slot < KL_AB_CAP) {
                    ab_key[s * KL_AB_CAP + slot] = kn;
                    ab_info[s * KL_AB_CAP + slot] = KLInfo{u, rp, len, pp};
                }
            } else {
                if (uint32_t(~uint32_t(K & 0xffffffffull)) == uint32_t(pp) && kn < K) {
                    (s ? dtag1 : dtag0)[c] = tag;
                    s_stop[3] = tag;
                } else if (kn > K) {
                    atomicMax(&(s ? ckn1 : ckn0)[c], kn);
                    if (gi >= KL_ITEM_CAP) {
                        (s ? dtag1 : dtag0)[c] = tag;
                        s_stop[3] = tag;
                    }
                }
            }
            cs = int((pl & 0x80000000u) | uint32_t(c));
            inf = KLInfo{u, rp, len, pp};
        }
        if (gi < KL_ITEM_CAP) {
            it_key[gi] = kn;
            it_cs[gi] = cs;
            it_info[gi] = inf;
        }
    };

    bool fail = false;
    if (wv < NG) {
        // ================= gain waves
        bool spec = false;
        u64 sk0 = 0ull, sk1 = 0ull;
        int s_gi = -1;
        int4 s_a = make_int4(0, 0, 0, 0);
        float s_in = 0.0f, s_ex = 0.0f;
        bool s_act = false;
        int pA = -1, pB = -1;  // the previous swap's pair (its flip may still be in flight)
        for (;; ++it) {
            if constexpr (PROF) t_a = now();
            if (!wait_word(1, int(it) + 1)) {  // the selection's pair, published by W
                fail = true;
                break;
            }
            if constexpr (PROF) {
                t_b = now();
                pc[3] += t_b - t_a;  // waiting for the pair
            }
            const u64 k0 = nx_key[0], k1 = nx_key[1];
            const v4i dA = *reinterpret_cast<const v4i*>(nx_info), dB = *reinterpret_cast<const v4i*>(nx_info + 1);
            const u64 K0 = readlane_u64(k0, 0), K1 = readlane_u64(k1, 0);
            if (K0 == 0ull || K1 == 0ull) break;
            const int posA = int(~uint32_t(K0 & 0xffffffffull)), posB = int(~uint32_t(K1 & 0xffffffffull));
            const int cA = posA / KL_CHUNK, cB = posB / KL_CHUNK;
            const int A = __builtin_amdgcn_readfirstlane(dA.x), pa = __builtin_amdgcn_readfirstlane(dA.y),
                      la = __builtin_amdgcn_readfirstlane(dA.z);
            const int B = __builtin_amdgcn_readfirstlane(dB.x), pb = __builtin_amdgcn_readfirstlane(dB.y),
                      lb = __builtin_amdgcn_readfirstlane(dB.z);
            const int tot = la + lb, tag = int(it), abp = (tag & 1) * 2;
            const int qA = pA, qB = pB;
            // sides / locks after the previous swap (flip applied by hand), then this pair swapped
            auto side_cur = [&](int x) -> bool {
                const bool b = x == qA ? true : x == qB ? false : ((s_side[x >> 5] >> (x & 31)) & 1u) != 0;
                return b ^ (x == A) ^ (x == B);
            };
            auto lock_cur = [&](int x) -> bool {
                return ((s_lock[x >> 5] >> (x & 31)) & 1u) || x == qA || x == qB || x == A || x == B;
            };
            if constexpr (PROF) {
                pc[2] += 1;
                pc[1] += spec && sk0 == K0 && sk1 == K1;
            }
            if (spec && sk0 == K0 && sk1 == K1) {
                g1_commit(s_gi, s_a, s_in, s_ex, s_act, cA, cB, tag, abp);
            } else {
                for (int i0 = wv * RPW; i0 < tot; i0 += NG * RPW) {
                    int gi;
                    int4 a;
                    float in_, ex_;
                    bool act;
                    g1_rows(i0, pa, la, pb, lb, side_cur, lock_cur, gi, a, in_, ex_, act);
                    g1_commit(gi, a, in_, ex_, act, cA, cB, tag, abp);
                }
            }
            if constexpr (PROF) {
                if (tid == 0 && s_in == -12345.0f) s_stop[2] = 0;  // keeps the commit's LDS writes ahead of the stamp
                t_a = now();
                pc[6] += t_a - t_b;  // pair -> barrier 1 (commit or G1)
            }
            __syncthreads();  // (1) gains, early rescans, merged keys and tags visible
            if constexpr (PROF) t_a = now();
            if (s_stop[it & 1]) {
                ++it;
                break;
            }
            // P. the next pair, exactly, from the state G2 is publishing
            // (gain wave 0; it hands the pair to the other gain waves)
            spec = false;
            u64 kA = 0ull, kB = 0ull;
            int nA = 0, npa = 0, nla = 0, nB = 0, npb = 0, nlb = 0;
            bool okp = false;
            if (wv == 0) {
                const bool any_tag = s_stop[3] == tag;
                const int s = half, cS = s ? cB : cA, nck = s ? d.nck1 : d.nck0;
                const u64* ckn = s ? ckn1 : ckn0;
                u64 k = 0ull;
                for (int c0 = hl; c0 < nck; c0 += 4 * 32) {
                    u64 kv[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) kv[u] = ckn[min(c0 + 32 * u, nck - 1)];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const u64 v = kv[u] & (min(c0 + 32 * u, nck - 1) == cS ? 0ull : ~0ull);
                        k = v > k ? v : k;
                    }
                }
                u64 rk[E_PARTS];
                v4i rf[E_PARTS];
#pragma unroll
                for (int q = 0; q < E_PARTS; ++q) {
                    rk[q] = er_key[s * E_PARTS + q];
                    rf[q] = *reinterpret_cast<const v4i*>(er_info + s * E_PARTS + q);
                }
                const int cnt = ab_cnt[abp + s];
                const int hs = hl < KL_AB_CAP ? hl : KL_AB_CAP - 1;
                const u64 bk_raw = ab_key[s * KL_AB_CAP + hs];
                const v4i bf = *reinterpret_cast<const v4i*>(ab_info + s * KL_AB_CAP + hs);
                const int il = lane < tot ? lane : 0;
                const u64 ik = it_key[il];
                const int ics = it_cs[il];
                const v4i iinf = *reinterpret_cast<const v4i*>(it_info + il);
                const bool have = hl < cnt && hl < KL_AB_CAP;
                const u64 bk = have ? bk_raw : 0ull;
                u64 R = rk[0];
                v4i Rf = rf[0];
#pragma unroll
                for (int q = 1; q < E_PARTS; ++q) {
                    const bool b = rk[q] > R;
                    R = b ? rk[q] : R;
                    Rf.x = b ? rf[q].x : Rf.x;
                    Rf.y = b ? rf[q].y : Rf.y;
                    Rf.z = b ? rf[q].z : Rf.z;
                    Rf.w = b ? rf[q].w : Rf.w;
                }
                const int Rpos = int(~uint32_t(R & 0xffffffffull));
                const bool stale = have && R != 0ull && bf.w == Rpos && bk < R;
                const bool bad = any_tag || tot > 64 || __ballot(stale || cnt > KL_AB_CAP) != 0ull;
                const u64 m = __ballot(cnt > 0) ? half_max_u64(bk) : 0ull;
                const u64 kS = m > R ? m : R;
                k = kS > k ? kS : k;
                k = half_max_u64(k);
                kA = readlane_u64(k, 0);
                kB = readlane_u64(k, 32);
                const bool own = lane < tot && ics != -1;
                const u64 mA = __ballot(own && ics >= 0 && ik == kA), mB = __ballot(own && ics < 0 && ik == kB);
                const u64 mS = s ? mB : mA;
                v4i desc = Rf;
                if (mA) {
                    const int l = __ffsll((long long)mA) - 1;
                    const v4i t = v4i{__builtin_amdgcn_readlane(iinf.x, l), __builtin_amdgcn_readlane(iinf.y, l),
                                      __builtin_amdgcn_readlane(iinf.z, l), 0};
                    if (!s) desc = t;
                }
                if (mB) {
                    const int l = __ffsll((long long)mB) - 1;
                    const v4i t = v4i{__builtin_amdgcn_readlane(iinf.x, l), __builtin_amdgcn_readlane(iinf.y, l),
                                      __builtin_amdgcn_readlane(iinf.z, l), 0};
                    if (s) desc = t;
                }
                if (!mS && k != R && k != 0ull)  // an unchanged chunk's winner (no G2 wave writes its entry)
                    desc = *reinterpret_cast<const v4i*>((s ? ci1 : ci0) + int(~uint32_t(k & 0xffffffffull)) / KL_CHUNK);
                // every read of this swap's state is done: barrier 2's arrival
                arrive();
                nA = __builtin_amdgcn_readlane(desc.x, 0);
                npa = __builtin_amdgcn_readlane(desc.y, 0);
                nla = __builtin_amdgcn_readlane(desc.z, 0);
                nB = __builtin_amdgcn_readlane(desc.x, 32);
                npb = __builtin_amdgcn_readlane(desc.y, 32);
                nlb = __builtin_amdgcn_readlane(desc.z, 32);
                okp = !bad && kA != 0ull && kB != 0ull && nla >= 0 && nlb >= 0 && nla + nlb <= NG * RPW && nA != nB;
                if (lane == 0) {  // (to the other gain waves)
                    sp[0] = okp ? kA : 0ull;
                    sp[1] = kB;
                    reinterpret_cast<v4i*>(sp + 2)[0] = v4i{nA, npa, nla, 0};
                    reinterpret_cast<v4i*>(sp + 2)[1] = v4i{nB, npb, nlb, 0};
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __hip_atomic_store(&sync[3], int(it) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            } else {
                arrive();  // (this wave reads none of the swap's shared state)
                if (!wait_word(3, int(it) + 1)) {
                    fail = true;
                    break;
                }
                kA = sp[0];
                kB = sp[1];
                const v4i a0 = reinterpret_cast<const v4i*>(sp + 2)[0], b0 = reinterpret_cast<const v4i*>(sp + 2)[1];
                kA = readlane_u64(kA, 0);
                kB = readlane_u64(kB, 0);
                okp = kA != 0ull;
                nA = __builtin_amdgcn_readfirstlane(a0.x);
                npa = __builtin_amdgcn_readfirstlane(a0.y);
                nla = __builtin_amdgcn_readfirstlane(a0.z);
                nB = __builtin_amdgcn_readfirstlane(b0.x);
                npb = __builtin_amdgcn_readfirstlane(b0.y);
                nlb = __builtin_amdgcn_readfirstlane(b0.z);
            }
            if constexpr (PROF) {
                t_b = now();
                pc[4] += t_b - t_a;  // barrier 1 -> the speculative pair
            }
            {
                if (okp) {
                    // the rows of the next pair under the sides after this swap and that pair's
                    auto side_nx = [&](int x) -> bool {
                        const bool b = x == A ? true : x == B ? false : ((s_side[x >> 5] >> (x & 31)) & 1u) != 0;
                        return b ^ (x == nA) ^ (x == nB);
                    };
                    auto lock_nx = [&](int x) -> bool {
                        return ((s_lock[x >> 5] >> (x & 31)) & 1u) || x == A || x == B || x == nA || x == nB;
                    };
                    s_gi = -1;
                    if (wv * RPW < nla + nlb)  // (rows for this wave)
                        g1_rows(wv * RPW, npa, nla, npb, nlb, side_nx, lock_nx, s_gi, s_a, s_in, s_ex, s_act);
                    spec = true;
                    if constexpr (PROF) {
                        pc[0] += 1;
                        if (s_gi >= 0 && s_in == -12345.0f) s_stop[2] = 0;  // keeps the sums ahead of the stamp
                        pc[5] += now() - t_b;  // the speculative rows
                    }
                    sk0 = kA;
                    sk1 = kB;
                }
            }
            pA = A;
            pB = B;
        }
    } else {
        // ================= W, early rescans, G2
        for (;; ++it) {
            if constexpr (PROF) t_a = now();
            if (it > 0 && !wait_word(0, 8 * int(it))) {  // barrier 2 of the previous swap
                fail = true;
                break;
            }
            if constexpr (PROF) {
                t_b = now();
                pc[7] += t_b - t_a;  // waiting at barrier 2
            }
            // S. selection (cKL.cpp:341-355) by the W wave alone (lanes 0-31 remain[0]'s
            // keys, 32-63 remain[1]'s), published to every other wave
            u64 k0, k1;
            v4i dA = v4i{0, 0, 0, 0}, dB = v4i{0, 0, 0, 0};
            if (wv == W_W) {
                u64 k = 0ull;
                const u64* ck = half ? ck1 : ck0;
                if (nsel <= 4 * 32) {
                    u64 kv[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) kv[u] = ck[min(hl + 32 * u, nsel - 1)];
#pragma unroll
                    for (int u = 0; u < 4; ++u) k = kv[u] > k ? kv[u] : k;
                } else {
                    for (int c0 = hl; c0 < nsel; c0 += 8 * 32) {
                        u64 kv[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) kv[u] = ck[min(c0 + 32 * u, nsel - 1)];
#pragma unroll
                        for (int u = 0; u < 8; ++u) k = kv[u] > k ? kv[u] : k;
                    }
                }
                k = half_max_u64(k);
                k0 = readlane_u64(k, 0);
                k1 = readlane_u64(k, 32);
                if (k0 != 0ull && k1 != 0ull) {
                    dA = *reinterpret_cast<const v4i*>(ci0 + int(~uint32_t(k0 & 0xffffffffull)) / KL_CHUNK);
                    dB = *reinterpret_cast<const v4i*>(ci1 + int(~uint32_t(k1 & 0xffffffffull)) / KL_CHUNK);
                }
                if (lane == 0) {
                    nx_key[0] = k0;
                    nx_key[1] = k1;
                    *reinterpret_cast<v4i*>(nx_info) = dA;
                    *reinterpret_cast<v4i*>(nx_info + 1) = dB;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __hip_atomic_store(&sync[1], int(it) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            } else {
                if (!wait_word(1, int(it) + 1)) {
                    fail = true;
                    break;
                }
                k0 = readlane_u64(nx_key[0], 0);
                k1 = readlane_u64(nx_key[1], 0);
                const v4i a0 = *reinterpret_cast<const v4i*>(nx_info), b0 = *reinterpret_cast<const v4i*>(nx_info + 1);
                dA = v4i{__builtin_amdgcn_readfirstlane(a0.x), __builtin_amdgcn_readfirstlane(a0.y),
                         __builtin_amdgcn_readfirstlane(a0.z), 0};
                dB = v4i{__builtin_amdgcn_readfirstlane(b0.x), __builtin_amdgcn_readfirstlane(b0.y),
                         __builtin_amdgcn_readfirstlane(b0.z), 0};
            }
            const int posA = int(~uint32_t(k0 & 0xffffffffull)), posB = int(~uint32_t(k1 & 0xffffffffull));
            const int cA = posA / KL_CHUNK, cB = posB / KL_CHUNK;
            if constexpr (PROF) {
                t_a = now();
                pc[8] += t_a - t_b;  // barrier 2 -> the pair (selection)
            }
            if (k0 == 0ull || k1 == 0ull) break;  // cKL.cpp:357,387-388 (identical in every wave)
            const int A = dA.x, pa = dA.y, la = dA.z, B = dB.x, pb = dB.y, lb = dB.z;
            auto locked_now = [&](int x) -> bool { return ((s_lock[x >> 5] >> (x & 31)) & 1u) || x == A || x == B; };
            const int tot = la + lb;
            const int tag = int(it);
            const int abp = (tag & 1) * 2;
            if (wv == W_W) {
                // W. w(A,B) (getEdgeWeight, cKL.cpp:75-82) and the pair gain (cKL.cpp:360-386)
                float gA = 0.f, gB = 0.f;
                if (lane == 0) {
                    gA = d.gp0[posA];
                    gB = d.gp1[posB];
                }
                float wab = 0.0f;
                bool found = false;
                for (int i = lane; i < la; i += 64)
                    if (d.col[pa + i] == B) {
                        wab = d.w[pa + i];
                        found = true;
                    }
                const u64 bal = __ballot(found);
                if (bal) wab = __shfl(wab, __ffsll((long long)bal) - 1, 64);
                if (lane == 0) {
                    d.gp0[posA] = __builtin_nanf("");
                    d.gp1[posB] = __builtin_nanf("");
                    const float gain = gA - gB - 2.0f * wab;
                    cut -= gain;
                    if (cut < best) {
                        best = cut;
                        best_it = it + 1;
                    }
                    if (it < cap) log[it] = ek_swap{uint32_t(it + 1), uint32_t(A), uint32_t(B), gA, gB, gain, cut, 0u};
                    int stop = 0;
                    if (gain <= 0.0f) {
                        if (++term > unsigned(limit)) stop = 1;
                    } else {
                        term = 0;
                    }
                    if (it + 1 >= d.n0 || it + 1 >= d.n1) stop = 1;
                    s_stop[it & 1] = stop;
                }
            } else {
                // E. early rescan of the chunk node1 (node2) leaves
                const int s = wv <= W_EB ? 1 : 0, part = (s ? W_EB : W_EA) - wv;
                const int p0 = (s ? cB : cA) * KL_CHUNK + part * NQ_E * 64;
                KLInfo info;
                bool mine;
                const u64 kk = s ? chunk_rescan2<NQ_E>(d.gp1, d.pinfo1, 1, p0, posB, lane, &info, &mine)
                                 : chunk_rescan2<NQ_E>(d.gp0, d.pinfo0, 0, p0, posA, lane, &info, &mine);
                if (mine) {
                    er_key[s * E_PARTS + part] = kk;
                    er_info[s * E_PARTS + part] = info;
                }
            }
            if constexpr (PROF) {
                t_b = now();
                pc[9] += t_b - t_a;  // the pair -> barrier 1 (W / early rescans)
            }
            __syncthreads();  // (1)
            if constexpr (PROF) t_a = now();
            if (s_stop[it & 1]) {
                if (wv == W_FLIP && lane == 0) {  // the last swap's flip, for the sides written below
                    atomicOr(&s_side[A >> 5], 1u << (A & 31));
                    atomicAnd(&s_side[B >> 5], ~(1u << (B & 31)));
                }
                ++it;
                break;
            }
            const bool any_tag = s_stop[3] == tag;
            if (wv == W_EA) {  // G2a, as in k_kl_swap_loop
                const int s = half, cS = s ? cB : cA;
                u64 rk[E_PARTS];
                v4i rf[E_PARTS];
#pragma unroll
                for (int q = 0; q < E_PARTS; ++q) {
                    rk[q] = er_key[s * E_PARTS + q];
                    rf[q] = *reinterpret_cast<const v4i*>(er_info + s * E_PARTS + q);
                }
                const int cnt = ab_cnt[abp + s];
                const int hs = hl < KL_AB_CAP ? hl : KL_AB_CAP - 1;
                const u64 bk_raw = ab_key[s * KL_AB_CAP + hs];
                const v4i bf = *reinterpret_cast<const v4i*>(ab_info + s * KL_AB_CAP + hs);
                const bool have = hl < cnt && hl < KL_AB_CAP;
                const u64 bk = have ? bk_raw : 0ull;
                if (hl == 0) ab_cnt[2 - abp + s] = 0;  // the next swap's list (its G1 appends after barrier 2)
                u64 R = rk[0];
                v4i Rf = rf[0];
#pragma unroll
                for (int q = 1; q < E_PARTS; ++q) {
                    const bool b = rk[q] > R;
                    R = b ? rk[q] : R;
                    Rf.x = b ? rf[q].x : Rf.x;
                    Rf.y = b ? rf[q].y : Rf.y;
                    Rf.z = b ? rf[q].z : Rf.z;
                    Rf.w = b ? rf[q].w : Rf.w;
                }
                const int Rpos = int(~uint32_t(R & 0xffffffffull));
                const bool stale = have && R != 0ull && bf.w == Rpos && bk < R;
                const u64 hmask = s ? 0xffffffff00000000ull : 0x00000000ffffffffull;
                const bool st = (__ballot(stale) & hmask) != 0ull || cnt > KL_AB_CAP;
                u64 m = 0ull;
                if (__ballot(cnt > 0)) m = half_max_u64(bk);
                if (!st) {
                    if (m > R) {
                        if (have && bk == m) {
                            (s ? ck1 : ck0)[cS] = m;
                            (s ? ckn1 : ckn0)[cS] = m;
                            *reinterpret_cast<v4i*>((s ? ci1 : ci0) + cS) = bf;
                        }
                    } else if (hl == 0) {
                        (s ? ck1 : ck0)[cS] = R;
                        (s ? ckn1 : ckn0)[cS] = R;
                        *reinterpret_cast<v4i*>((s ? ci1 : ci0) + cS) = Rf;
                    }
                }
                const bool stA = __builtin_amdgcn_readlane(int(st), 0) != 0, stB = __builtin_amdgcn_readlane(int(st), 32) != 0;
                for (int q = 0; q < 2; ++q) {
                    if (!(q ? stB : stA)) continue;
                    KLInfo info;
                    bool mine;
                    const u64 kk = q ? chunk_rescan(d.gp1, d.pinfo1, 1, cB, -1, lane, &info, &mine)
                                     : chunk_rescan(d.gp0, d.pinfo0, 0, cA, -1, lane, &info, &mine);
                    if (mine) {
                        (q ? ck1 : ck0)[q ? cB : cA] = kk;
                        (q ? ckn1 : ckn0)[q ? cB : cA] = kk;
                        (q ? ci1 : ci0)[q ? cB : cA] = info;
                    }
                }
            }
            if (wv == W_FLIP && lane == 0) {  // the swap itself, for the next swap's lookups
                atomicOr(&s_side[A >> 5], 1u << (A & 31));
                atomicAnd(&s_side[B >> 5], ~(1u << (B & 31)));
                atomicOr(&s_lock[A >> 5], 1u << (A & 31));
                atomicOr(&s_lock[B >> 5], 1u << (B & 31));
            }
            if (wv == W_EB || wv == W_EB - 1) {  // G2b
                for (int i = (W_EB - wv) * 64 + lane; i < tot && i < KL_ITEM_CAP; i += 128) {
                    const int cs = it_cs[i];
                    const u64 kn = it_key[i];
                    const int4 inf = *reinterpret_cast<const int4*>(it_info + i);
                    if (cs == -1) continue;
                    const int s = int(uint32_t(cs) >> 31), c = cs & 0x7fffffff;
                    const u64 kmerged = (s ? ckn1 : ckn0)[c];
                    const int dt = (s ? dtag1 : dtag0)[c];
                    if ((s ? c == cB : c == cA) || dt == tag) continue;
                    (s ? ck1 : ck0)[c] = kmerged;
                    if (kmerged == kn) *reinterpret_cast<int4*>((s ? ci1 : ci0) + c) = inf;
                }
            }
            // G2c. full rescans of the tagged chunks (the waves of this group, each claimed once)
            for (int i = wv - NG; any_tag && i < tot; i += NW - NG) {
                int cs;
                if (i < KL_ITEM_CAP) cs = it_cs[i];
                else {
                    const int u = i < la ? d.col[pa + i] : d.col[pb + i - la];
                    cs = locked_now(u) ? -1 : int((uint32_t(d.nd[u].c) & 0x80000000u) |
                                                  ((uint32_t(d.nd[u].c) & 0x7fffffffu) / KL_CHUNK));
                }
                if (cs == -1) continue;
                const int s = int(uint32_t(cs) >> 31), c = cs & 0x7fffffff;
                if ((s ? dtag1 : dtag0)[c] != tag) continue;
                int claimed = 0;
                if (lane == 0) claimed = atomicMax(&(s ? ctag1 : ctag0)[c], tag) < tag;
                if (!__shfl(claimed, 0, 64)) continue;
                KLInfo info;
                bool mine;
                const u64 kk = s ? chunk_rescan(d.gp1, d.pinfo1, 1, c, -1, lane, &info, &mine)
                                 : chunk_rescan(d.gp0, d.pinfo0, 0, c, -1, lane, &info, &mine);
                if (mine) {
                    (s ? ck1 : ck0)[c] = kk;
                    (s ? ckn1 : ckn0)[c] = kk;
                    (s ? ci1 : ci0)[c] = info;
                }
            }
            arrive();  // (2), as a counter
            if constexpr (PROF) pc[10] += now() - t_a;  // barrier 1 -> G2 done
        }
    }
    if (fail) give_up();
    __syncthreads();
    for (int u = tid; u < d.n; u += KL_LOOP_THREADS) d.side[u] = uint8_t((s_side[u >> 5] >> (u & 31)) & 1u);
    if (wv == W_W && lane == 0) {
        out->iterations = it;
        out->best_iter = best_it;
        out->initial_cut = *d.cut0;
        out->best_cut = best;
        out->final_cut = cut;
        out->status = sync[2] ? 3u : 2u;
    }
    if constexpr (PROF) {
        // [0] speculations, [1] hits, [2] swaps, [3] gain wave 0 waiting for the pair, [4] its P, [5] its
        // speculative rows, [6] pair -> barrier 1; W: [7] barrier-2 wait, [8] selection, [9] pair -> barrier 1;
        // [10] W's G2 span, [11] G2a's; [12] loop cycles, [13] marker
        if (wv == 0 && lane == 0)
            for (int i = 0; i < 7; ++i) out->prof[i] = pc[i];
        if (wv == W_W && lane == 0) {
            for (int i = 7; i < 11; ++i) out->prof[i] = pc[i];
            out->prof[12] = now() - t_start;
            out->prof[13] = 0x9199ull;
        }
        if (wv == W_EA && lane == 0) out->prof[11] = pc[10];
    } else if (tid == 0) {
        for (int i = 0; i < 16; ++i) out->prof[i] = 0ull;
    }
}


// The swap loop with its state in global memory: the fallback for graphs
// whose bitmaps and chunk tables do not fit in LDS (and the A/B reference,
// EK_KL_GLOBAL_STATE=1).  Four barriers per swap.  Only SMEM=false is launched.
template <bool SMEM, bool PROF>
__global__ __launch_bounds__(KL_LOOP_THREADS) void k_kl_loop(KLDev d, int limit, ek_swap* __restrict__ log,
                                                             long long cap, KLOut* __restrict__ out) {
    constexpr int NW = KL_LOOP_THREADS / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ u64 red0[NW], red1[NW];
    __shared__ float s_w;
    __shared__ int s_stop;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int words = (d.n + 31) / 32;
    u64* ck0 = d.ckey0;
    u64* ck1 = d.ckey1;
    uint32_t* s_side = nullptr;
    uint32_t* s_lock = nullptr;
    if constexpr (SMEM) {
        ck0 = reinterpret_cast<u64*>(smem);
        ck1 = ck0 + d.nck0;
        s_side = reinterpret_cast<uint32_t*>(ck1 + d.nck1);
        s_lock = s_side + words;
        for (int i = tid; i < d.nck0; i += KL_LOOP_THREADS) ck0[i] = d.ckey0[i];
        for (int i = tid; i < d.nck1; i += KL_LOOP_THREADS) ck1[i] = d.ckey1[i];
        for (int i = tid; i < words; i += KL_LOOP_THREADS) {
            s_side[i] = side_word(d.side_init, d.n, i);
            s_lock[i] = 0u;
        }
    }
    if (tid == 0) s_w = 0.0f;
    __syncthreads();
    // loop-carried scalars live in thread 0 only
    float cut = *d.cut0, best = cut;
    long long best_it = 0, it = 0;
    unsigned term = 0;
    unsigned long long tph[4] = {0, 0, 0, 0}, tstamp = 0;  // diagnostic build only (PROF)
    auto stamp = [&](int ph) {
        if constexpr (PROF) {
            if (tid == 0) {
                const unsigned long long t = __builtin_amdgcn_s_memrealtime();
                if (ph >= 0) tph[ph] += t - tstamp;
                tstamp = t;
            }
        }
    };
    for (;;) {
        stamp(-1);
        // S. selection (cKL.cpp:341-355): max key over both lists' chunks
        u64 k0 = 0ull, k1 = 0ull;
        for (int c = tid; c < d.nck0; c += KL_LOOP_THREADS) k0 = ck0[c] > k0 ? ck0[c] : k0;
        for (int c = tid; c < d.nck1; c += KL_LOOP_THREADS) k1 = ck1[c] > k1 ? ck1[c] : k1;
        k0 = wave_max_u64(k0);
        k1 = wave_max_u64(k1);
        if (lane == 0) {
            red0[wv] = k0;
            red1[wv] = k1;
        }
        __syncthreads();  // (1)
        stamp(0);
        k0 = red0[0];
        k1 = red1[0];
#pragma unroll
        for (int i = 1; i < NW; ++i) {
            k0 = red0[i] > k0 ? red0[i] : k0;
            k1 = red1[i] > k1 ? red1[i] : k1;
        }
        if (k0 == 0ull || k1 == 0ull) break;  // cKL.cpp:357,387-388 (uniform)
        const int posA = int(~uint32_t(k0 & 0xffffffffull)), posB = int(~uint32_t(k1 & 0xffffffffull));
        const int A = d.order0[posA], B = d.order1[posB];
        const int pa = d.rowptr[A], la = d.rowptr[A + 1] - pa;
        const int pb = d.rowptr[B], lb = d.rowptr[B + 1] - pb;
        // W. w(A,B) (getEdgeWeight, cKL.cpp:75-82); swap + erase (swip, cKL.cpp:274-286)
        float gA = 0.f, gB = 0.f;
        if (tid == 0) {
            gA = d.gp0[posA];
            gB = d.gp1[posB];
            d.gp0[posA] = __builtin_nanf("");
            d.gp1[posB] = __builtin_nanf("");
            if constexpr (SMEM) {
                s_side[A >> 5] |= 1u << (A & 31);
                s_side[B >> 5] &= ~(1u << (B & 31));
                s_lock[A >> 5] |= 1u << (A & 31);
                s_lock[B >> 5] |= 1u << (B & 31);
            } else {
                d.side[A] = 1;
                d.side[B] = 0;
                d.locked[A] = 1;
                d.locked[B] = 1;
            }
        }
        for (int i = tid; i < la; i += KL_LOOP_THREADS)
            if (d.col[pa + i] == B) s_w = d.w[pa + i];  // B occurs at most once in A's row
        __syncthreads();  // (2)
        stamp(1);
        if (tid == 0) {   // pair gain, running cut, log, termination (cKL.cpp:358-386)
            const float gain = gA - gB - 2.0f * s_w;
            cut -= gain;
            ++it;
            if (cut < best) {
                best = cut;
                best_it = it;
            }
            if (it <= cap) log[it - 1] = ek_swap{uint32_t(it), uint32_t(A), uint32_t(B), gA, gB, gain, cut, 0u};
            int stop = 0;
            if (gain <= 0.0f) {
                if (++term > unsigned(limit)) stop = 1;
            } else {
                term = 0;
            }
            if (it >= d.n0 || it >= d.n1) stop = 1;  // a remain[] list is exhausted
            s_stop = stop;
        }
        // G. gains of N(A) u N(B) (updateAffectedNodeGains, cKL.cpp:253-272)
        for (int i = tid; i < la + lb; i += KL_LOOP_THREADS) {
            const int u = i < la ? d.col[pa + i] : d.col[pb + i - la];
            bool lk;
            if constexpr (SMEM) lk = (s_lock[u >> 5] >> (u & 31)) & 1u;
            else lk = d.locked[u] != 0;
            if (!lk) {
                const float g = row_gain<SMEM>(d.rowptr, d.col, d.w, s_side, d.side, u, nullptr);
                const uint32_t pl = d.plist[u];
                ((pl >> 31) ? d.gp1 : d.gp0)[pl & 0x7fffffffu] = g;
            }
        }
        __syncthreads();  // (3)
        stamp(2);
        // K. re-key the chunks holding A, B and every affected node
        for (int i = wv; i < la + lb + 2; i += NW) {
            const int u = i < la ? d.col[pa + i] : i < la + lb ? d.col[pb + i - la] : (i == la + lb ? A : B);
            const uint32_t pl = d.plist[u];
            const int s = int(pl >> 31), c = int(pl & 0x7fffffffu) / KL_CHUNK;
            const u64 k = s ? chunk_key(d.gp1, 1, c, lane) : chunk_key(d.gp0, 0, c, lane);
            if (lane == 0) (s ? ck1 : ck0)[c] = k;
        }
        if (tid == 0) s_w = 0.0f;
        __syncthreads();  // (4)
        stamp(3);
        if (s_stop) break;
    }
    if constexpr (SMEM) {
        __syncthreads();
        for (int u = tid; u < d.n; u += KL_LOOP_THREADS) d.side[u] = uint8_t((s_side[u >> 5] >> (u & 31)) & 1u);
    }
    if (tid == 0) {
        out->iterations = it;
        out->best_iter = best_it;
        out->initial_cut = *d.cut0;
        out->best_cut = best;
        out->final_cut = cut;
        out->status = SMEM ? 1u : 0u;
        for (int i = 0; i < 4; ++i) out->prof[i] = tph[i];  // global-state loop: 4 phases
        for (int i = 4; i < 16; ++i) out->prof[i] = 0ull;
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

// integer hyperedge cuts of three partitions at once (initial, best prefix,
// final): nets whose pins are not all on one side.  One thread per net; its
// pins' ids are loaded four at a time, then their three sides.  Each
// workgroup stores its three counts (part[k * gridDim.x + block]) and the
// host adds them: one atomic add per wave on a single counter serialised at
// the memory side (~13 ns each: 49 us a launch for one cut at the headline's
// 240k nets, 144 us for three)
__global__ __launch_bounds__(256) void k_net_cut(long long nets, const int64_t* __restrict__ net_ptr,
                                                 const int32_t* __restrict__ pins, const uint8_t* __restrict__ sa,
                                                 const uint8_t* __restrict__ sb, const uint8_t* __restrict__ sc,
                                                 unsigned* __restrict__ part) {
    __shared__ unsigned wcnt[3][4];
    const long long e = blockIdx.x * 256ll + threadIdx.x;
    bool ca = false, cb = false, cc = false;
    if (e < nets) {
        const int64_t p0 = net_ptr[e], p1 = net_ptr[e + 1];
        if (p1 - p0 >= 2) {
            const int v0 = pins[p0];
            const uint8_t a0 = sa[v0], b0 = sb[v0], c0 = sc[v0];
            for (int64_t p = p0 + 1; p < p1 && !(ca && cb && cc); p += 4) {
                int v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = p + u < p1 ? pins[p + u] : v0;  // past the net: the first pin
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    ca |= sa[v[u]] != a0;
                    cb |= sb[v[u]] != b0;
                    cc |= sc[v[u]] != c0;
                }
            }
        }
    }
    const u64 ma = __ballot(ca), mb = __ballot(cb), mc = __ballot(cc);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        wcnt[0][w] = unsigned(__popcll(ma));
        wcnt[1][w] = unsigned(__popcll(mb));
        wcnt[2][w] = unsigned(__popcll(mc));
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const unsigned* c = wcnt[threadIdx.x];
        part[threadIdx.x * gridDim.x + blockIdx.x] = c[0] + c[1] + c[2] + c[3];
    }
}

__global__ __launch_bounds__(256) void k_build_aux(long long nnz, const int32_t* __restrict__ col,
                                                   const KLInfo* __restrict__ nd, KLInfo* __restrict__ aux) {
    const long long p = blockIdx.x * 256ll + threadIdx.x;
    if (p >= nnz) return;
    const int v = col[p];
    const int4 x = *reinterpret_cast<const int4*>(nd + v);
    *reinterpret_cast<int4*>(aux + p) = make_int4(v, x.x, x.y, x.z);
}

// seg[p*KL_SEG_LANES + j] = entries 2j, 2j+1 of row col[p] as {col, w bits, col, w bits} (0 past its end)
__global__ __launch_bounds__(256) void k_build_seg(long long nnz, const int32_t* __restrict__ rowptr,
                                                   const int32_t* __restrict__ col, const float* __restrict__ w,
                                                   KLInfo* __restrict__ seg) {
    const long long t = blockIdx.x * 256ll + threadIdx.x;
    const long long p = t / KL_SEG_LANES;
    if (p >= nnz) return;
    const int j = int(t % KL_SEG_LANES), v = col[p];
    const int rp = rowptr[v], len = rowptr[v + 1] - rp;
    const int e0 = 2 * j, e1 = 2 * j + 1;
    int4 o = make_int4(0, 0, 0, 0);
    if (e0 < len) {
        o.x = col[rp + e0];
        o.y = __float_as_int(w[rp + e0]);
    }
    if (e1 < len) {
        o.z = col[rp + e1];
        o.w = __float_as_int(w[rp + e1]);
    }
    *reinterpret_cast<int4*>(seg + t) = o;
}

void kl_build_aux(hipStream_t s, int64_t nnz, const int32_t* col, const KLInfo* nd, KLInfo* aux) {
    if (nnz <= 0) return;
    hipLaunchKernelGGL(k_build_aux, dim3(unsigned((nnz + 255) / 256)), dim3(256), 0, s, (long long)nnz, col, nd, aux);
}

void kl_build_seg(hipStream_t s, int64_t nnz, const int32_t* rowptr, const int32_t* col, const float* w, KLInfo* seg) {
    if (nnz <= 0) return;
    hipLaunchKernelGGL(k_build_seg, dim3(unsigned((nnz * KL_SEG_LANES + 255) / 256)), dim3(256), 0, s, (long long)nnz, rowptr,
                       col, w, seg);
}

// segc[p*KL_SEGC_PIECES + j] = coded entries 4j .. 4j+3 of row col[p] (word 0 past its end)
__global__ __launch_bounds__(256) void k_build_segc(long long nnz, const int32_t* __restrict__ rowptr,
                                                    const int32_t* __restrict__ col, const uint32_t* __restrict__ kw,
                                                    KLInfo* __restrict__ segc) {
    const long long t = blockIdx.x * 256ll + threadIdx.x;
    const long long p = t / KL_SEGC_PIECES;
    if (p >= nnz) return;
    const int j = int(t % KL_SEGC_PIECES), v = col[p];
    const int rp = rowptr[v], len = rowptr[v + 1] - rp;
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = 4 * j + k < len ? kw[rp + 4 * j + k] : 0u;
    segc[t] = KLInfo{int32_t(o[0]), int32_t(o[1]), int32_t(o[2]), int32_t(o[3])};
}

void kl_build_segc(hipStream_t s, int64_t nnz, const int32_t* rowptr, const int32_t* col, const uint32_t* kw,
                   KLInfo* segc) {
    if (nnz <= 0) return;
    hipLaunchKernelGGL(k_build_segc, dim3(unsigned((nnz * KL_SEGC_PIECES + 255) / 256)), dim3(256), 0, s,
                       (long long)nnz, rowptr, col, kw, segc);
}

// Exact fp32 weights by bit pattern: code 0 is 0.0f (the padding), the rest
// in first-seen order.  Open addressing over the few distinct values (sums of
// 1/(k-1) over shared nets: tens at ibm18 shape).
bool kl_weight_codes(int64_t n, int64_t nnz, const int32_t* col, const float* w, std::vector<uint32_t>& kw,
                     std::vector<float>& wdict, int& wcolbits) {
    wcolbits = 1;
    while (wcolbits < 31 && (int64_t(1) << wcolbits) < n) ++wcolbits;
    if (wcolbits > 28) return false;
    const size_t max_codes = std::min<size_t>(size_t(1) << (32 - wcolbits), size_t(KL_WDICT_CAP));
    const size_t cap = 2 * size_t(KL_WDICT_CAP);  // power of two, at least twice the codes
    struct Table {  // open addressing over the fp32 bit patterns
        std::vector<uint32_t> keys;
        std::vector<int32_t> slot;
        size_t cap;
        explicit Table(size_t c) : keys(c), slot(c, -1), cap(c) {}
        size_t find(uint32_t k) const {
            size_t h = size_t((k * 0x9E3779B1u) >> 19) & (cap - 1);
            while (slot[h] >= 0 && keys[h] != k) h = (h + 1) & (cap - 1);
            return h;
        }
    };
    // 1. each thread's distinct weights (in first-occurrence order), in
    // parallel; 2. their union, code 0 = 0.0f then in thread order; 3. every
    // entry encoded in parallel.  The codes only index the table the swap
    // loop decodes through, so their order does not change any result.
    const int T = int(std::min<int64_t>(host_threads(), std::max<int64_t>(1, nnz / 65536)));
    std::vector<std::vector<uint32_t>> seen(static_cast<size_t>(T));
    std::atomic<bool> over{false};
    run_threads(T, [&](int t) {
        Table loc(cap);
        auto& sv = seen[size_t(t)];
        for (int64_t p = nnz * t / T; p < nnz * (t + 1) / T && !over.load(std::memory_order_relaxed); ++p) {
            uint32_t k;
            std::memcpy(&k, &w[p], 4);
            const size_t h = loc.find(k);
            if (loc.slot[h] < 0) {
                if (sv.size() >= max_codes) {
                    over = true;
                    break;
                }
                loc.slot[h] = int32_t(sv.size());
                loc.keys[h] = k;
                sv.push_back(k);
            }
        }
    });
    if (over) return false;
    Table glob(cap);
    wdict.assign(1, 0.0f);
    {
        const size_t h = glob.find(0u);
        glob.slot[h] = 0;
        glob.keys[h] = 0u;
    }
    for (const auto& sv : seen)
        for (const uint32_t k : sv) {
            const size_t h = glob.find(k);
            if (glob.slot[h] >= 0) continue;
            if (wdict.size() >= max_codes) return false;
            glob.slot[h] = int32_t(wdict.size());
            glob.keys[h] = k;
            float f;
            std::memcpy(&f, &k, 4);
            wdict.push_back(f);
        }
    kw.resize(size_t(std::max<int64_t>(nnz, 0)));
    run_threads(T, [&](int t) {
        for (int64_t p = nnz * t / T; p < nnz * (t + 1) / T; ++p) {
            uint32_t k;
            std::memcpy(&k, &w[p], 4);
            kw[size_t(p)] = (uint32_t(glob.slot[glob.find(k)]) << wcolbits) | uint32_t(col[p]);
        }
    });
    return true;
}

// Row descriptors of a partition, from the uploaded lists (integers only):
// by position in each list {node, rowptr, rowlen, 0}, zero past the list up to
// the chunk padding; by node {rowptr, rowlen, plist, 0}.
__global__ __launch_bounds__(256) void k_build_desc(int n, int n0, int n1, int pad0, int pad1,
                                                    const int32_t* __restrict__ order0,
                                                    const int32_t* __restrict__ order1,
                                                    const uint32_t* __restrict__ plist,
                                                    const int32_t* __restrict__ rowptr, KLInfo* __restrict__ p0,
                                                    KLInfo* __restrict__ p1, KLInfo* __restrict__ nd) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < pad0) {
        KLInfo v{0, 0, 0, 0};
        if (i < n0) {
            const int u = order0[i];
            v = KLInfo{u, rowptr[u], rowptr[u + 1] - rowptr[u], 0};
        }
        p0[i] = v;
    }
    if (i < pad1) {
        KLInfo v{0, 0, 0, 0};
        if (i < n1) {
            const int u = order1[i];
            v = KLInfo{u, rowptr[u], rowptr[u + 1] - rowptr[u], 0};
        }
        p1[i] = v;
    }
    if (i < n) nd[i] = KLInfo{rowptr[i], rowptr[i + 1] - rowptr[i], int32_t(plist[i]), 0};
}

void kl_build_desc(hipStream_t s, int n, int n0, int n1, int pad0, int pad1, const int32_t* order0,
                   const int32_t* order1, const uint32_t* plist, const int32_t* rowptr, KLInfo* p0, KLInfo* p1,
                   KLInfo* nd) {
    const int m = std::max(n, std::max(pad0, pad1));
    if (m <= 0) return;
    hipLaunchKernelGGL(k_build_desc, dim3((m + 255) / 256), dim3(256), 0, s, n, n0, n1, pad0, pad1, order0, order1,
                       plist, rowptr, p0, p1, nd);
}

namespace {
KLDev with_chunk(KLDev d, int ch) {
    d.nck0 = (d.n0 + ch - 1) / ch;
    d.nck1 = (d.n1 + ch - 1) / ch;
    return d;
}
// Which swap loop runs, decided on the KL_CHUNK chunk counts: LDS bytes of
// the on-chip form (0: does not fit / not taken), of the off-chip-bitmap form,
// and the chunk size the chosen form and its chunk keys use.  kl_prepare and
// kl_loop both ask, so the keys are built for the loop that reads them.
struct LoopForm {
    size_t lds, lds_gb;
    int ch;
};
LoopForm loop_form(const KLDev& d_in) {
    const KLDev d = with_chunk(d_in, KL_CHUNK);
    const bool force_gb = std::getenv("EK_KL_GBITS") && std::getenv("EK_KL_GBITS")[0] == '1';
    const size_t lds = force_gb ? 0 : kl_loop_lds_bytes(d);
    const size_t lds_gb = d.locked && !std::getenv("EK_KL_GLOBAL_STATE") ? kl_loop_lds_bytes(d, false) : 0;
    if (!lds && lds_gb) return {0, kl_loop_lds_bytes(with_chunk(d, KL_CHUNK_GB), false), KL_CHUNK_GB};
    return {lds, lds_gb, KL_CHUNK};
}
}  // namespace

void kl_prepare(hipStream_t s, const KLDev& d_in) {
    const KLDev d = with_chunk(d_in, loop_form(d_in).ch);
    const int nb = (d.n + 255) / 256;
    hipLaunchKernelGGL(k_gain_scan, dim3(nb), dim3(256), 0, s, d);
    hipLaunchKernelGGL(k_cut_final, dim3(1), dim3(256), 0, s, d, nb);
    const int waves = d.nck0 + d.nck1;
    if (loop_form(d_in).ch == KL_CHUNK_GB)
        hipLaunchKernelGGL(k_chunk_init<KL_CHUNK_GB>, dim3((waves + 3) / 4), dim3(256), 0, s, d);
    else
        hipLaunchKernelGGL(k_chunk_init<KL_CHUNK>, dim3((waves + 3) / 4), dim3(256), 0, s, d);
}

// Streams `n16` 16-B pieces through the caches (nothing kept): after it the
// array's lines sit in the Infinity Cache (MALL) as far as it holds them.
__global__ __launch_bounds__(256) void k_touch(const int4* __restrict__ p, long long n16, int* __restrict__ sink) {
    int acc = 0;
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n16; i += 256ll * gridDim.x) acc ^= p[i].x;
    if (acc == 0x7fffabcd) sink[0] = acc;
}

void kl_loop(hipStream_t s, const KLDev& d_in, int limit, ek_swap* log, long long cap, KLOut* out) {
    // the on-chip loop with its bitmaps in LDS; else (a larger graph) with
    // them in global memory while the rest fits (EK_KL_GBITS=1 forces that
    // form: tests), over KL_CHUNK_GB-position chunks; else the global-state loop
    const LoopForm form = loop_form(d_in);
    const KLDev d = with_chunk(d_in, form.ch);
    const size_t lds = form.lds, lds_gb = form.lds_gb;
    // Warm the Infinity Cache with the per-entry arrays the swap loop reads at
    // random (inline segments, then descriptors, so the descriptors are the
    // most recent): most of its one dependent round trip per swap then hits
    // the MALL instead of HBM.  ibm18 shape: 59.3 -> 57.9 ms for the swap
    // loop, the two streams included (~50 us); the chunk scans' descriptors
    // as well: no further gain.  EK_KL_NOTOUCH=1: off (A/B).
    if (!std::getenv("EK_KL_NOTOUCH")) {
        int* sink = reinterpret_cast<int*>(&out->prof[13]);  // never written in practice
        if (d.segc)
            hipLaunchKernelGGL(k_touch, dim3(4096), dim3(256), 0, s, reinterpret_cast<const int4*>(d.segc),
                               (long long)d.nnz * KL_SEGC_PIECES, sink);
        else if (d.seg)
            hipLaunchKernelGGL(k_touch, dim3(4096), dim3(256), 0, s, reinterpret_cast<const int4*>(d.seg),
                               (long long)d.nnz * KL_SEG_LANES, sink);
        hipLaunchKernelGGL(k_touch, dim3(1024), dim3(256), 0, s, reinterpret_cast<const int4*>(d.aux), (long long)d.nnz,
                           sink);
    }
    const bool prof = std::getenv("EK_KL_PROF") != nullptr;  // phase stamps: diagnostic instantiation
    // the overlapped schedule (k_kl_swap_pipe); EK_KL_PIPE=0/1 forces it off/on
    const char* pe = std::getenv("EK_KL_PIPE");
    const bool pipe = pe && pe[0] ? pe[0] != '0' : false;
    if (lds && pipe && !std::getenv("EK_KL_GLOBAL_STATE")) {
        if (prof && d.segc)
            hipLaunchKernelGGL((k_kl_swap_pipe<true, true>), dim3(1), dim3(KL_LOOP_THREADS), lds, s, d, limit, log, cap, out);
        else if (prof)
            hipLaunchKernelGGL((k_kl_swap_pipe<true, false>), dim3(1), dim3(KL_LOOP_THREADS), lds, s, d, limit, log, cap, out);
        else if (d.segc)
            hipLaunchKernelGGL((k_kl_swap_pipe<false, true>), dim3(1), dim3(KL_LOOP_THREADS), lds, s, d, limit, log, cap, out);
        else
            hipLaunchKernelGGL((k_kl_swap_pipe<false, false>), dim3(1), dim3(KL_LOOP_THREADS), lds, s, d, limit, log, cap, out);
        return;
    }
    const bool global_state = std::getenv("EK_KL_GLOBAL_STATE") != nullptr;  // A/B: force the global-state loop
    if (!lds && lds_gb) {
        if (prof && d.segc)  // (phase stamps of the off-chip-bitmap form: diagnostic)
            hipLaunchKernelGGL((k_kl_swap_loop<true, true, true>), dim3(1), dim3(KL_LOOP_THREADS), lds_gb, s, d, limit,
                               log, cap, out);
        else if (d.segc)
            hipLaunchKernelGGL((k_kl_swap_loop<false, true, true>), dim3(1), dim3(KL_LOOP_THREADS), lds_gb, s, d, limit,
                               log, cap, out);
        else
            hipLaunchKernelGGL((k_kl_swap_loop<false, false, true>), dim3(1), dim3(KL_LOOP_THREADS), lds_gb, s, d, limit,
                               log, cap, out);
        return;
    }
    // the fixed LDS layout when the chunk lists allow it (EK_KL_FIXLDS=0: off, A/B)
    const char* fx = std::getenv("EK_KL_FIXLDS");
    const size_t lds_fix = lds && !global_state && !prof && !(fx && fx[0] == '0') ? kl_loop_lds_bytes(d, true, true) : 0;
    if (lds_fix) {
        if (d.segc)
            hipLaunchKernelGGL((k_kl_swap_loop<false, true, false, true>), dim3(1), dim3(KL_LOOP_THREADS), lds_fix, s, d,
                               limit, log, cap, out);
        else
            hipLaunchKernelGGL((k_kl_swap_loop<false, false, false, true>), dim3(1), dim3(KL_LOOP_THREADS), lds_fix, s, d,
                               limit, log, cap, out);
        return;
    }
    if (lds && !global_state && prof && d.segc)
        hipLaunchKernelGGL((k_kl_swap_loop<true, true>), dim3(1), dim3(KL_LOOP_THREADS), lds, s, d, limit, log, cap, out);
    else if (lds && !global_state && prof)
        hipLaunchKernelGGL((k_kl_swap_loop<true, false>), dim3(1), dim3(KL_LOOP_THREADS), lds, s, d, limit, log, cap, out);
    else if (lds && !global_state && d.segc)
        hipLaunchKernelGGL((k_kl_swap_loop<false, true>), dim3(1), dim3(KL_LOOP_THREADS), lds, s, d, limit, log, cap,
                           out);
    else if (lds && !global_state)
        hipLaunchKernelGGL((k_kl_swap_loop<false, false>), dim3(1), dim3(KL_LOOP_THREADS), lds, s, d, limit, log, cap,
                           out);
    else if (prof)
        hipLaunchKernelGGL((k_kl_loop<false, true>), dim3(1), dim3(KL_LOOP_THREADS), 0, s, d, limit, log, cap, out);
    else
        hipLaunchKernelGGL((k_kl_loop<false, false>), dim3(1), dim3(KL_LOOP_THREADS), 0, s, d, limit, log, cap, out);
}

void kl_replay(hipStream_t s, int n, const uint8_t* side_init, const ek_swap* log, const long long* count,
               long long cap, uint8_t* sides_out) {
    const int nb = std::min(2048, (n + 255) / 256);
    hipLaunchKernelGGL(k_replay, dim3(nb), dim3(256), 0, s, n, side_init, sides_out);
    hipLaunchKernelGGL(k_replay_swaps, dim3(64), dim3(256), 0, s, log, count, cap, sides_out);
}

int net_cut_blocks(int64_t nets) { return int((nets + 255) / 256); }

void net_cut(hipStream_t s, int64_t nets, const int64_t* net_ptr, const int32_t* pins, const uint8_t* side_a,
             const uint8_t* side_b, const uint8_t* side_c, unsigned* part) {
    if (nets <= 0) return;
    hipLaunchKernelGGL(k_net_cut, dim3(unsigned(net_cut_blocks(nets))), dim3(256), 0, s, (long long)nets, net_ptr,
                       pins, side_a, side_b, side_c, part);
}


// ---------------------------------------------------------------------------
// Median split of the Fiedler vector on the device (ek_kl_set_partition_fiedler):
// the same values ek_median_split and the remain[] lists of ek_solve_file give
// on the host (io.cpp, solve.cpp), without the vector's round trip.

// out = x * sgn: the normalised, sign-fixed Ritz vector, the same IEEE
// products as the host's v_out[i] = v[i] * sgn (ctx.cpp)
__global__ __launch_bounds__(256) void k_fiedler_scale(const double* __restrict__ x, double sgn, int n,
                                                       double* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = x[i] * sgn;
}

// The median's two ranks by a radix select (no sort): the fp64 values as the
// ordered 64-bit keys of a radix sort (sign flipped, negatives inverted: -0
// before +0, exactly a radix sort's order), eight passes of one byte from the
// top.  A pass histograms the byte of the keys that match the prefix found so
// far (LDS bins, then agent-scope adds into that pass's 256 global bins); its
// last block to finish (two-level arrival counter) scans the bins, extends the
// prefix by the byte holding the rank and subtracts the keys below it.  Both
// ranks (n/2 - 1 and n/2 of an even n) are selected in the same passes.  The
// keys come out identical to a full sort's entries at those ranks.
constexpr int SEL_THREADS = 256, SEL_PER = 8, SEL_PASSES = 8;
constexpr int SEL_SUB = 16;  // first-level arrival counters, 64 uints apart
struct SelState {
    unsigned long long prefix[2], mask[2];
    unsigned k[2];
    unsigned pad[2];
    unsigned hist[SEL_PASSES][2][256];
    unsigned ctr[(SEL_SUB + 1) * 64];
};

__device__ __forceinline__ unsigned long long ord_key(double v) {
    const unsigned long long u = static_cast<unsigned long long>(__double_as_longlong(v));
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__global__ __launch_bounds__(SEL_THREADS) void k_select_init(SelState* st, unsigned k0, unsigned k1) {
    // (the histograms and counters are zeroed by the host's memset)
    if (threadIdx.x < 2) {
        st->prefix[threadIdx.x] = 0ull;
        st->mask[threadIdx.x] = 0ull;
        st->k[threadIdx.x] = threadIdx.x ? k1 : k0;
    }
}

__global__ __launch_bounds__(SEL_THREADS) void k_select_pass(const double* __restrict__ v, int n, SelState* st,
                                                             int pass, unsigned long long* keys_out) {
    __shared__ unsigned h[2][256];
    __shared__ int s_last;
    const int t = threadIdx.x;
    h[0][t] = 0u;
    h[1][t] = 0u;
    const unsigned long long p0 = st->prefix[0], m0 = st->mask[0], p1 = st->prefix[1], m1 = st->mask[1];
    const int shift = 56 - 8 * pass;
    __syncthreads();
    const int base = int(blockIdx.x) * SEL_THREADS * SEL_PER;
#pragma unroll
    for (int u = 0; u < SEL_PER; ++u) {
        const int i = base + u * SEL_THREADS + t;
        if (i < n) {
            const unsigned long long key = ord_key(v[i]);
            const unsigned d = unsigned(key >> shift) & 255u;
            if ((key & m0) == p0) atomicAdd(&h[0][d], 1u);
            if ((key & m1) == p1) atomicAdd(&h[1][d], 1u);
        }
    }
    __syncthreads();
    for (int r = 0; r < 2; ++r)
        if (h[r][t]) __hip_atomic_fetch_add(&st->hist[pass][r][t], h[r][t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every thread's adds performed before the block arrives
    __syncthreads();
    if (t == 0) {
        const unsigned nb = gridDim.x, g = blockIdx.x % SEL_SUB;
        const unsigned gsize = (nb - g + SEL_SUB - 1) / SEL_SUB, ngroups = nb < SEL_SUB ? nb : SEL_SUB;
        s_last = 0;
        if (__hip_atomic_fetch_add(st->ctr + g * 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1u)
            s_last = __hip_atomic_fetch_add(st->ctr + SEL_SUB * 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                     ngroups - 1u;
    }
    __syncthreads();
    if (!s_last) return;
    // the last block: every bin's total, then the byte holding each rank (one
    // wave per rank: an inclusive scan of its 256 bins, 4 per lane)
    if (t < SEL_SUB + 1) st->ctr[t * 64] = 0u;  // re-armed for the next pass
    const int w = t >> 6, l = t & 63;
    if (w < 2) {
        unsigned c[4], sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            c[q] = __hip_atomic_load(&st->hist[pass][w][4 * l + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sum += c[q];
        }
        unsigned incl = sum;  // inclusive scan of the lanes' sums
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned y = __shfl_up(incl, o, 64);
            if (l >= o) incl += y;
        }
        const unsigned k = st->k[w];
        unsigned below = incl - sum;  // keys in the bins of the lanes before this one
        int dsel = -1;
        unsigned bsel = 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (dsel < 0 && k >= below && k < below + c[q]) {
                dsel = 4 * l + q;
                bsel = below;
            }
            below += c[q];
        }
        if (dsel >= 0) {  // exactly one lane holds the rank
            const unsigned long long pf = st->prefix[w] | (static_cast<unsigned long long>(dsel) << shift);
            st->prefix[w] = pf;
            st->mask[w] |= 255ull << shift;
            st->k[w] = k - bsel;
            if (pass == SEL_PASSES - 1) keys_out[w] = pf;
        }
    }
}

size_t split_tmp_bytes(int n) {
    const size_t blocks = size_t((n + 1023) / 1024) + 1;
    return sizeof(SelState) + 256 + blocks * 4 + 64;
}

void fiedler_scale(hipStream_t s, const double* x, double sgn, int n, double* out) {
    hipLaunchKernelGGL(k_fiedler_scale, dim3((n + 255) / 256), dim3(256), 0, s, x, sgn, n, out);
}

void split_select(hipStream_t s, void* tmp, const double* v, int n, unsigned k0, unsigned k1,
                  unsigned long long* keys_out) {
    SelState* st = static_cast<SelState*>(tmp);
    const hipError_t e = hipMemsetAsync(st, 0, sizeof(SelState), s);
    if (e != hipSuccess) ek::fail(EK_EHIP, "split_select: %s", hipGetErrorString(e));
    hipLaunchKernelGGL(k_select_init, dim3(1), dim3(SEL_THREADS), 0, s, st, k0, k1);
    const int nb = (n + SEL_THREADS * SEL_PER - 1) / (SEL_THREADS * SEL_PER);
    for (int p = 0; p < SEL_PASSES; ++p)
        hipLaunchKernelGGL(k_select_pass, dim3(nb), dim3(SEL_THREADS), 0, s, v, n, st, p, keys_out);
}

double key_value(unsigned long long key) {
    const unsigned long long u = (key >> 63) ? (key & 0x7fffffffffffffffull) : ~key;
    double d;
    std::memcpy(&d, &u, 8);
    return d;
}

// remain[] lists in node order (cKL.cpp:155-174): side 0 holds the nodes with
// !(med > v[i]) (bit 0 of ek_median_split).  k_split_count counts them per
// 1024-node block; k_split_place gives each node its position (the blocks
// before it, summed by every block, plus an in-block exclusive scan) in list
// 0, or i - that in list 1, and writes plist and the initial sides as
// ek_kl_set_partition builds them; the last block also writes n0.
constexpr int PART_THREADS = 256, PART_PER = 4, PART_BLOCK = PART_THREADS * PART_PER;
__global__ __launch_bounds__(PART_THREADS) void k_split_count(const double* __restrict__ v, int n, double med,
                                                              unsigned* __restrict__ bcount) {
    __shared__ unsigned ws[PART_THREADS / 64];
    const int t = threadIdx.x, base = int(blockIdx.x) * PART_BLOCK;
    unsigned c = 0;
#pragma unroll
    for (int u = 0; u < PART_PER; ++u) {
        const int i = base + t * PART_PER + u;
        if (i < n && !(med > v[i])) ++c;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((t & 63) == 0) ws[t >> 6] = c;
    __syncthreads();
    if (t == 0) bcount[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(PART_THREADS) void k_split_place(const double* __restrict__ v, int n, double med,
                                                              const unsigned* __restrict__ bcount,
                                                              int32_t* __restrict__ order0, int32_t* __restrict__ order1,
                                                              uint32_t* __restrict__ plist, uint8_t* __restrict__ side,
                                                              unsigned* __restrict__ n0_out) {
    __shared__ unsigned ws[PART_THREADS / 64];
    __shared__ unsigned wscan[PART_THREADS / 64];
    const int t = threadIdx.x, base = int(blockIdx.x) * PART_BLOCK;
    // side-0 nodes in the blocks before this one
    unsigned before = 0;
    for (int b = t; b < int(blockIdx.x); b += PART_THREADS) before += bcount[b];
    for (int o = 32; o > 0; o >>= 1) before += __shfl_xor(before, o, 64);
    if ((t & 63) == 0) ws[t >> 6] = before;
    bool f[PART_PER];
    unsigned c = 0;
#pragma unroll
    for (int u = 0; u < PART_PER; ++u) {
        const int i = base + t * PART_PER + u;
        f[u] = i < n && !(med > v[i]);
        c += f[u] ? 1u : 0u;
    }
    // exclusive scan of the threads' counts over the block (wave scan, then
    // the waves' totals)
    const int l = t & 63, w = t >> 6;
    unsigned incl = c;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(incl, o, 64);
        if (l >= o) incl += y;
    }
    if (l == 63) wscan[w] = incl;
    __syncthreads();
    unsigned off = ws[0] + ws[1] + ws[2] + ws[3];
    for (int q = 0; q < w; ++q) off += wscan[q];
    unsigned p0 = off + incl - c;
#pragma unroll
    for (int u = 0; u < PART_PER; ++u) {
        const int i = base + t * PART_PER + u;
        if (i >= n) break;
        if (f[u]) {
            order0[p0] = i;
            plist[i] = p0;
            side[i] = 0;
            ++p0;
        } else {
            const uint32_t p1 = uint32_t(i) - p0;
            order1[p1] = i;
            plist[i] = p1 | 0x80000000u;
            side[i] = 1;
        }
    }
    if (blockIdx.x == gridDim.x - 1 && t == PART_THREADS - 1) *n0_out = p0;
}

void split_partition(hipStream_t s, void* tmp, const double* v, int n, double med, int32_t* order0, int32_t* order1,
                     uint32_t* plist, uint8_t* side, unsigned* n0_out) {
    unsigned* bcount = reinterpret_cast<unsigned*>(static_cast<char*>(tmp) + sizeof(SelState) + 256);
    const int nb = (n + PART_BLOCK - 1) / PART_BLOCK;
    hipLaunchKernelGGL(k_split_count, dim3(nb), dim3(PART_THREADS), 0, s, v, n, med, bcount);
    hipLaunchKernelGGL(k_split_place, dim3(nb), dim3(PART_THREADS), 0, s, v, n, med, bcount, order0, order1, plist,
                       side, n0_out);
}

}  // namespace dev
}  // namespace ek
