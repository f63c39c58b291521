// The clique Laplacian built on the device, straight from the hypergraph's
// pins into the SpMV's dictionary-coded segments (initializeMatrix,
// cEIG.cpp:86-133, restated for gfx950).  Same values, bit for bit, as the
// host build (graph_build.cpp build_laplacian_rows): every (row, col) sum
// runs over the row's nets in ascending order, the diagonal is minus the
// row's sum in ascending column order, and the row blocks come from the
// same greedy partition — so the SpMV and the Lanczos run are bit-identical
// to the ones on host-built rows (tests/test_gpu_build.py).  Rows longer
// than a workgroup's LDS sort and value sets larger than the dictionary
// table fall back to the host build (ek_spmv_setup_pins reports which).
//
// Kernels (integer work and fixed-order fp64 sums):
//   k_net_count   per net: incidence and raw-entry counts of its rows
//   k_scan_*      exclusive scans (tile sums, one-block scan of them, tiles)
//   k_net_fill    per net: (net, position) incidences into their rows' slots
//   k_rows        per row: incidences sorted, raw entries gathered, stable
//                 insertion sort by column, duplicates summed, diagonal
//   k_rows_long   one workgroup per row past k_rows' limit (LDS bitonic sort
//                 of (column, index) keys: stable)
//   k_row_write   per row: CSR columns / values, the diagonal in place
//   k_dict_insert open-addressing set of the values' fp64 bit patterns
//   k_dict_codes  occupied slots -> codes (scanned flags), the value table
//   k_encode      per row block: coded words into its segment, row starts
#include <hip/hip_runtime.h>

#include "ek_internal.hpp"

namespace ek {
namespace dev {

namespace {

constexpr int BT = 256;
constexpr int ROW_SHORT = 256;  // raw entries a thread sorts in place; longer rows go to k_rows_long
constexpr int LONG_CAP = 8192;  // raw entries k_rows_long sorts in LDS (64 KB of keys)
constexpr unsigned long long EMPTY_KEY = ~0ull;  // a NaN payload: never a Laplacian value

inline unsigned grid_of(long long n) { return unsigned((n + BT - 1) / BT); }

__global__ __launch_bounds__(BT) void k_net_count(long long nets, const int64_t* __restrict__ net_ptr,
                                                  const int32_t* __restrict__ pins, long long r0, long long r1,
                                                  int* __restrict__ icnt, int* __restrict__ rcnt) {
    const long long e = (long long)blockIdx.x * BT + threadIdx.x;
    if (e >= nets) return;
    const long long p0 = net_ptr[e], p1 = net_ptr[e + 1], k = p1 - p0;
    if (k < 2) return;
    for (long long p = p0; p < p1; ++p) {
        const long long v = pins[p];
        if (v >= r0 && v < r1) {
            atomicAdd(&icnt[v - r0], 1);
            atomicAdd(&rcnt[v - r0], int(k - 1));
        }
    }
}

// ---- exclusive scan: int in[n] -> long long out[n + 1] (out[n] = total)
constexpr int SCAN_TILE = 1024, SCAN_PER = SCAN_TILE / BT;

__device__ __forceinline__ long long block_incl_scan(long long v, long long* lds) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    if (lane == 63) lds[w] = v;
    __syncthreads();
    long long add = 0;
    for (int i = 0; i < w; ++i) add += lds[i];
    __syncthreads();
    return v + add;
}

__global__ __launch_bounds__(BT) void k_scan_tiles(const int* __restrict__ in, long long n,
                                                   long long* __restrict__ tile_sum) {
    __shared__ long long lds[4];
    long long s = 0;
    const long long base = (long long)blockIdx.x * SCAN_TILE;
#pragma unroll
    for (int u = 0; u < SCAN_PER; ++u) {
        const long long i = base + u * BT + threadIdx.x;
        s += i < n ? in[i] : 0;
    }
    s = block_incl_scan(s, lds);
    if (threadIdx.x == BT - 1) tile_sum[blockIdx.x] = s;
}

__global__ __launch_bounds__(BT) void k_scan_sums(long long* __restrict__ tile_sum, int ntiles) {
    __shared__ long long lds[4];
    __shared__ long long tot;
    long long carry = 0;
    for (int b0 = 0; b0 < ntiles; b0 += BT) {
        const int i = b0 + threadIdx.x;
        const long long v = i < ntiles ? tile_sum[i] : 0;
        const long long inc = block_incl_scan(v, lds);
        if (i < ntiles) tile_sum[i] = carry + inc - v;
        if (threadIdx.x == BT - 1) tot = inc;
        __syncthreads();
        carry += tot;
        __syncthreads();
    }
}

__global__ __launch_bounds__(BT) void k_scan_apply(const int* __restrict__ in, long long n,
                                                   const long long* __restrict__ tile_off, long long* __restrict__ out) {
    __shared__ long long lds[4];
    const long long base = (long long)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_PER;
    int v[SCAN_PER];
    long long s = 0;
#pragma unroll
    for (int u = 0; u < SCAN_PER; ++u) {
        v[u] = base + u < n ? in[base + u] : 0;
        s += v[u];
    }
    long long run = tile_off[blockIdx.x] + block_incl_scan(s, lds) - s;
#pragma unroll
    for (int u = 0; u < SCAN_PER; ++u) {
        if (base + u < n) out[base + u] = run;
        run += v[u];
        if (base + u == n - 1) out[n] = run;
    }
}

__global__ __launch_bounds__(BT) void k_net_fill(long long nets, const int64_t* __restrict__ net_ptr,
                                                 const int32_t* __restrict__ pins, long long r0, long long r1,
                                                 const long long* __restrict__ ip, int* __restrict__ cur,
                                                 int2* __restrict__ inc) {
    const long long e = (long long)blockIdx.x * BT + threadIdx.x;
    if (e >= nets) return;
    const long long p0 = net_ptr[e], p1 = net_ptr[e + 1];
    if (p1 - p0 < 2) return;
    for (long long p = p0; p < p1; ++p) {
        const long long v = pins[p];
        if (v >= r0 && v < r1) inc[ip[v - r0] + atomicAdd(&cur[v - r0], 1)] = make_int2(int(e), int(p - p0));
    }
}

// raw entries of row i in the host build's order: its incidences by (net,
// position) ascending, each net's other pins in order; returns their count
__device__ int gather_row(long long i, const long long* __restrict__ ip, int2* __restrict__ inc,
                          const int64_t* __restrict__ net_ptr, const int32_t* __restrict__ pins, int* __restrict__ scol,
                          double* __restrict__ sval, long long at) {
    const long long a = ip[i], b = ip[i + 1];
    for (long long x = a + 1; x < b; ++x) {  // atomics filled the slots in any order
        const int2 key = inc[x];
        long long y = x;
        while (y > a && (inc[y - 1].x > key.x || (inc[y - 1].x == key.x && inc[y - 1].y > key.y))) {
            inc[y] = inc[y - 1];
            --y;
        }
        inc[y] = key;
    }
    int m = 0;
    for (long long x = a; x < b; ++x) {
        const int2 q = inc[x];
        const long long p0 = net_ptr[q.x], p1 = net_ptr[q.x + 1];
        const double w = -(2.0 / double(p1 - p0));
        for (long long p = p0; p < p1; ++p)
            if (p - p0 != q.y) {
                scol[at + m] = pins[p];
                sval[at + m] = w;
                ++m;
            }
    }
    return m;
}

// column-sorted raw entries at [at, at + m): duplicates summed in order,
// merged entries written back from `at`; the row sum in ascending column
// order gives the diagonal (-sum)
__device__ void merge_row(long long i, long long r, int* __restrict__ scol, double* __restrict__ sval, long long at,
                          int m, int* __restrict__ ulen, int* __restrict__ len, double* __restrict__ diag) {
    int u = 0;
    for (int x = 0; x < m; ++x) {
        if (u > 0 && scol[at + u - 1] == scol[at + x]) sval[at + u - 1] += sval[at + x];
        else {
            scol[at + u] = scol[at + x];
            sval[at + u] = sval[at + x];
            ++u;
        }
    }
    double s = 0.0;
    bool hd = false;
    for (int x = 0; x < u; ++x) {
        s += sval[at + x];
        hd |= scol[at + x] == r;
    }
    ulen[i] = u;
    len[i] = u + (hd ? 0 : 1);
    diag[i] = -s;
}

__global__ __launch_bounds__(BT) void k_rows(long long nr, long long r0, const long long* __restrict__ ip,
                                             int2* __restrict__ inc, const long long* __restrict__ rp,
                                             const int64_t* __restrict__ net_ptr, const int32_t* __restrict__ pins,
                                             int* __restrict__ scol, double* __restrict__ sval, int* __restrict__ ulen,
                                             int* __restrict__ len, double* __restrict__ diag,
                                             int* __restrict__ long_rows, int* __restrict__ n_long) {
    const long long i = (long long)blockIdx.x * BT + threadIdx.x;
    if (i >= nr) return;
    const long long at = rp[i];
    if (rp[i + 1] - at > ROW_SHORT) {  // a workgroup of its own (k_rows_long)
        long_rows[atomicAdd(n_long, 1)] = int(i);
        return;
    }
    const int m = gather_row(i, ip, inc, net_ptr, pins, scol, sval, at);
    for (int x = 1; x < m; ++x) {  // stable insertion sort by column
        const int c = scol[at + x];
        const double v = sval[at + x];
        int y = x;
        while (y > 0 && scol[at + y - 1] > c) {
            scol[at + y] = scol[at + y - 1];
            sval[at + y] = sval[at + y - 1];
            --y;
        }
        scol[at + y] = c;
        sval[at + y] = v;
    }
    merge_row(i, r0 + i, scol, sval, at, m, ulen, len, diag);
}

__global__ __launch_bounds__(BT) void k_rows_long(long long r0, const int* __restrict__ long_rows,
                                                  const long long* __restrict__ ip, int2* __restrict__ inc,
                                                  const long long* __restrict__ rp, const int64_t* __restrict__ net_ptr,
                                                  const int32_t* __restrict__ pins, int* __restrict__ scol,
                                                  double* __restrict__ sval, double* __restrict__ tval,
                                                  int* __restrict__ ulen, int* __restrict__ len,
                                                  double* __restrict__ diag, int* __restrict__ too_long) {
    __shared__ unsigned long long key[LONG_CAP];
    __shared__ int m_s;
    const long long i = long_rows[blockIdx.x];
    const long long at = rp[i];
    if (rp[i + 1] - at > LONG_CAP) {
        if (threadIdx.x == 0) atomicAdd(too_long, 1);
        return;
    }
    if (threadIdx.x == 0) m_s = gather_row(i, ip, inc, net_ptr, pins, scol, sval, at);
    __syncthreads();
    const int m = m_s;
    int p2 = 1;
    while (p2 < m) p2 <<= 1;
    for (int x = threadIdx.x; x < p2; x += BT)
        key[x] = x < m ? (static_cast<unsigned long long>(uint32_t(scol[at + x])) << 32) | uint32_t(x) : ~0ull;
    __syncthreads();
    for (int k = 2; k <= p2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int x = threadIdx.x; x < p2; x += BT) {
                const int y = x ^ j;
                if (y > x) {
                    const unsigned long long a = key[x], b = key[y];
                    if ((a > b) == ((x & k) == 0)) {
                        key[x] = b;
                        key[y] = a;
                    }
                }
            }
            __syncthreads();
        }
    for (int x = threadIdx.x; x < m; x += BT) tval[at + x] = sval[at + int(uint32_t(key[x]))];
    __syncthreads();
    for (int x = threadIdx.x; x < m; x += BT) {
        scol[at + x] = int(key[x] >> 32);
        sval[at + x] = tval[at + x];
    }
    __syncthreads();
    if (threadIdx.x == 0) merge_row(i, r0 + i, scol, sval, at, m, ulen, len, diag);
}

__global__ __launch_bounds__(BT) void k_row_write(long long nr, long long r0, const long long* __restrict__ rp,
                                                  const long long* __restrict__ off, const int* __restrict__ ulen,
                                                  const int* __restrict__ len, const int* __restrict__ scol,
                                                  const double* __restrict__ sval, const double* __restrict__ diag,
                                                  int* __restrict__ rowptr, int* __restrict__ col,
                                                  double* __restrict__ val) {
    const long long i = (long long)blockIdx.x * BT + threadIdx.x;
    if (i >= nr) return;
    const long long at = rp[i], r = r0 + i;
    long long o = off[i];
    rowptr[i] = int(o);
    if (i == nr - 1) rowptr[nr] = int(off[nr]);
    const int u = ulen[i];
    const double dg = diag[i];
    bool placed = len[i] == u;  // the row holds (r, r) already (repeated pins): its value becomes -sum
    for (int x = 0; x < u; ++x) {
        const int c = scol[at + x];
        if (!placed && c > r) {
            col[o] = int(r);
            val[o++] = dg;
            placed = true;
        }
        col[o] = c;
        val[o++] = c == r ? dg : sval[at + x];
    }
    if (!placed) {
        col[o] = int(r);
        val[o] = dg;
    }
}

__device__ __forceinline__ unsigned dict_hash(unsigned long long k, unsigned mask) {
    return unsigned(((k ^ (k >> 29)) * 0x9E3779B97F4A7C15ull) >> 20) & mask;
}

__global__ __launch_bounds__(BT) void k_dict_insert(long long nnz, const double* __restrict__ val,
                                                    unsigned long long* __restrict__ table, unsigned mask,
                                                    int* __restrict__ overflow) {
    // The workgroup's values are first made distinct in an LDS set (a few
    // per workgroup: the Laplacian holds ~1e3 distinct values in 1e6
    // entries), and only those go to the global table: one global probe per
    // distinct value per workgroup instead of one per entry (k_dict_insert
    // took 1.0 ms at ibm18 shape on the hot values' lines).
    constexpr int LT = 4 * BT;  // power of two, 4x the workgroup's values: never full
    __shared__ unsigned long long lt[LT];
    for (int i = threadIdx.x; i < LT; i += BT) lt[i] = EMPTY_KEY;
    __syncthreads();
    const long long p = (long long)blockIdx.x * BT + threadIdx.x;
    if (p >= nnz) return;
    const unsigned long long k = static_cast<unsigned long long>(__double_as_longlong(val[p]));
    for (unsigned h = dict_hash(k, LT - 1);; h = (h + 1) & (LT - 1)) {
        const unsigned long long prev = atomicCAS(&lt[h], EMPTY_KEY, k);
        if (prev == k) return;  // another lane of the workgroup carries it
        if (prev == EMPTY_KEY) break;
    }
    unsigned h = dict_hash(k, mask);
    for (unsigned probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
        // a plain read first: the few hot values are in the table after their
        // first insert; a slot only goes EMPTY -> value, so a stale EMPTY just
        // costs the CAS that then reports the value
        const unsigned long long cur = table[h];
        if (cur == k) return;
        if (cur == EMPTY_KEY) {
            const unsigned long long prev = atomicCAS(&table[h], EMPTY_KEY, k);
            if (prev == EMPTY_KEY || prev == k) return;
        }
    }
    atomicAdd(overflow, 1);  // table full
}

__global__ __launch_bounds__(BT) void k_dict_flags(const unsigned long long* __restrict__ table, int tsize,
                                                   int* __restrict__ flag) {
    const int h = blockIdx.x * BT + threadIdx.x;
    if (h < tsize) flag[h] = table[h] != EMPTY_KEY ? 1 : 0;
}

__global__ __launch_bounds__(BT) void k_dict_codes(const unsigned long long* __restrict__ table, int tsize,
                                                   const long long* __restrict__ code_of_slot,
                                                   double* __restrict__ dict) {
    const int h = blockIdx.x * BT + threadIdx.x;
    if (h < tsize && table[h] != EMPTY_KEY) dict[code_of_slot[h]] = __longlong_as_double((long long)table[h]);
}

__device__ __forceinline__ uint32_t code_of(double v, const unsigned long long* __restrict__ table, unsigned mask,
                                            const long long* __restrict__ code_of_slot) {
    const unsigned long long k = static_cast<unsigned long long>(__double_as_longlong(v));
    unsigned h = dict_hash(k, mask);
    while (table[h] != k) h = (h + 1) & mask;  // every value was inserted
    return uint32_t(code_of_slot[h]);
}

// block b: seg[b*SEG + t] = coded word t (0 past cnt), rel[b*REL + t] = row
// start t inside the segment (t <= nr) or cnt; a long row's words go to the
// overflow area at desc.nnz0 and its segment and row starts stay 0
__global__ __launch_bounds__(BT) void k_encode(const int4* __restrict__ desc, const int* __restrict__ rowptr,
                                               const int* __restrict__ col, const double* __restrict__ val,
                                               const unsigned long long* __restrict__ table, unsigned mask,
                                               const long long* __restrict__ code_of_slot, int colbits,
                                               uint32_t* __restrict__ seg, uint16_t* __restrict__ rel) {
    const int b = blockIdx.x;
    const int4 d = desc[b];
    const int r0 = d.x, nr = d.y, cnt = d.w;
    const int p0 = rowptr[r0];
    uint32_t* s = seg + size_t(b) * SPMV_SEG_NNZ;
    uint16_t* rl = rel + size_t(b) * SPMV_REL_STRIDE;
    if (cnt > SPMV_SEG_NNZ) {
        for (int t = threadIdx.x; t < cnt; t += BT)
            seg[size_t(d.z) + t] = (code_of(val[p0 + t], table, mask, code_of_slot) << colbits) | uint32_t(col[p0 + t]);
        for (int t = threadIdx.x; t < SPMV_SEG_NNZ; t += BT) s[t] = 0u;
        for (int t = threadIdx.x; t < SPMV_REL_STRIDE; t += BT) rl[t] = 0;
        return;
    }
    for (int t = threadIdx.x; t < SPMV_SEG_NNZ; t += BT)
        s[t] = t < cnt ? (code_of(val[p0 + t], table, mask, code_of_slot) << colbits) | uint32_t(col[p0 + t]) : 0u;
    for (int t = threadIdx.x; t < SPMV_REL_STRIDE; t += BT) rl[t] = uint16_t(t <= nr ? rowptr[r0 + t] - p0 : cnt);
}

__global__ __launch_bounds__(BT) void k_encode_words(long long nnz, const int* __restrict__ col,
                                                     const double* __restrict__ val,
                                                     const unsigned long long* __restrict__ table, unsigned mask,
                                                     const long long* __restrict__ code_of_slot, int colbits,
                                                     uint32_t* __restrict__ pk) {
    const long long e = (long long)blockIdx.x * BT + threadIdx.x;
    if (e < nnz) pk[e] = (code_of(val[e], table, mask, code_of_slot) << colbits) | uint32_t(col[e]);
}

}  // namespace

void encode_words(hipStream_t s, long long nnz, const int* col, const double* val, const unsigned long long* table,
                  int tsize, const long long* code_of_slot, int colbits, uint32_t* pk) {
    if (nnz > 0)
        hipLaunchKernelGGL(k_encode_words, dim3(grid_of(nnz)), dim3(BT), 0, s, nnz, col, val, table, unsigned(tsize - 1),
                           code_of_slot, colbits, pk);
}

void exclusive_scan(hipStream_t s, const int* in, long long n, long long* out, long long* tiles) {
    const int ntiles = int((n + SCAN_TILE - 1) / SCAN_TILE);
    if (ntiles == 0) {
        (void)hipMemsetAsync(out, 0, sizeof(long long), s);
        return;
    }
    hipLaunchKernelGGL(k_scan_tiles, dim3(ntiles), dim3(BT), 0, s, in, n, tiles);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(BT), 0, s, tiles, ntiles);
    hipLaunchKernelGGL(k_scan_apply, dim3(ntiles), dim3(BT), 0, s, in, n, tiles, out);
}

void lap_count(hipStream_t s, const LapBuild& b) {
    hipLaunchKernelGGL(k_net_count, dim3(grid_of(b.nets)), dim3(BT), 0, s, b.nets, b.net_ptr, b.pins, b.r0, b.r1,
                       b.icnt, b.rcnt);
}

void lap_fill_rows(hipStream_t s, const LapBuild& b) {
    const long long nr = b.r1 - b.r0;
    int2* inc = reinterpret_cast<int2*>(b.inc);
    hipLaunchKernelGGL(k_net_fill, dim3(grid_of(b.nets)), dim3(BT), 0, s, b.nets, b.net_ptr, b.pins, b.r0, b.r1, b.ip,
                       b.cur, inc);
    hipLaunchKernelGGL(k_rows, dim3(grid_of(nr)), dim3(BT), 0, s, nr, b.r0, b.ip, inc, b.rp, b.net_ptr, b.pins,
                       b.scol, b.sval, b.ulen, b.len, b.diag, b.long_rows, b.counters);
}

void lap_long_rows(hipStream_t s, const LapBuild& b, int n_long) {
    if (n_long > 0)
        hipLaunchKernelGGL(k_rows_long, dim3(n_long), dim3(BT), 0, s, b.r0, b.long_rows, b.ip,
                           reinterpret_cast<int2*>(b.inc), b.rp, b.net_ptr,
                           b.pins, b.scol, b.sval, b.tval, b.ulen, b.len, b.diag, b.counters + 1);
}

void lap_write(hipStream_t s, const LapBuild& b, const long long* off, int* rowptr, int* col, double* val) {
    const long long nr = b.r1 - b.r0;
    hipLaunchKernelGGL(k_row_write, dim3(grid_of(nr)), dim3(BT), 0, s, nr, b.r0, b.rp, off, b.ulen, b.len, b.scol,
                       b.sval, b.diag, rowptr, col, val);
}

void dict_build(hipStream_t s, long long nnz, const double* val, unsigned long long* table, int tsize,
                int* overflow, int* flags, long long* code_of_slot, long long* tiles) {
    (void)hipMemsetAsync(table, 0xFF, size_t(tsize) * 8, s);
    hipLaunchKernelGGL(k_dict_insert, dim3(grid_of(nnz)), dim3(BT), 0, s, nnz, val, table, unsigned(tsize - 1),
                       overflow);
    hipLaunchKernelGGL(k_dict_flags, dim3(grid_of(tsize)), dim3(BT), 0, s, table, tsize, flags);
    exclusive_scan(s, flags, tsize, code_of_slot, tiles);  // code_of_slot[tsize] = number of distinct values
}

void dict_values(hipStream_t s, const unsigned long long* table, int tsize, const long long* code_of_slot,
                 double* dict) {
    hipLaunchKernelGGL(k_dict_codes, dim3(grid_of(tsize)), dim3(BT), 0, s, table, tsize, code_of_slot, dict);
}

void encode_segments(hipStream_t s, int nblocks, const int32_t* desc, const int* rowptr, const int* col,
                     const double* val, const unsigned long long* table, int tsize, const long long* code_of_slot,
                     int colbits, uint32_t* seg, uint16_t* rel) {
    if (nblocks > 0)
        hipLaunchKernelGGL(k_encode, dim3(nblocks), dim3(BT), 0, s, reinterpret_cast<const int4*>(desc), rowptr, col,
                           val, table, unsigned(tsize - 1), code_of_slot, colbits, seg, rel);
}

// The sharded Lanczos all-gathers each rank's slice of f into a slot of S
// doubles (rank-major, padded: the slices are nnz-balanced and unequal), so a
// global column c owned by rank r (off[r] <= c < off[r+1]) is read at
// r * S + (c - off[r]).  Monotone in c: sorted rows stay sorted.
__global__ __launch_bounds__(BT) void k_remap_cols(long long nnz, int* __restrict__ col,
                                                   const long long* __restrict__ off, int nranks, long long slot) {
    const long long p = (long long)blockIdx.x * BT + threadIdx.x;
    if (p >= nnz) return;
    const long long c = col[p];
    int lo = 0, hi = nranks - 1;  // largest r with off[r] <= c
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= c) lo = mid;
        else hi = mid - 1;
    }
    col[p] = int(lo * slot + (c - off[lo]));
}

void remap_cols(hipStream_t s, long long nnz, int* col, const long long* off, int nranks, long long slot) {
    if (nnz > 0)
        hipLaunchKernelGGL(k_remap_cols, dim3(grid_of(nnz)), dim3(BT), 0, s, nnz, col, off, nranks, slot);
}

// The owned-slot part of a sharded rank's rows (ctx.cpp factorize_mr: its
// SpMV runs while the all-gather of the other slots is in flight): per local
// row the entries whose slot-layout column lies in [lo, hi) — a contiguous
// run, the columns are sorted — counted, then copied with LOCAL column ids
// (col - lo: x is the rank's own f) after an exclusive scan of the counts.
__global__ __launch_bounds__(BT) void k_own_count(long long nr, const int* __restrict__ rowptr,
                                                  const int* __restrict__ col, int lo, int hi, int* __restrict__ cnt) {
    const long long r = (long long)blockIdx.x * BT + threadIdx.x;
    if (r >= nr) return;
    int k = 0;
    for (int p = rowptr[r]; p < rowptr[r + 1]; ++p) k += col[p] >= lo && col[p] < hi;
    cnt[r] = k;
}

__global__ __launch_bounds__(BT) void k_own_fill(long long nr, const int* __restrict__ rowptr,
                                                 const int* __restrict__ col, const double* __restrict__ val, int lo,
                                                 int hi, const long long* __restrict__ off, int* __restrict__ orp,
                                                 int* __restrict__ ocol, double* __restrict__ oval) {
    const long long r = (long long)blockIdx.x * BT + threadIdx.x;
    if (r > nr) return;
    orp[r] = int(off[r]);
    if (r == nr) return;
    long long q = off[r];
    for (int p = rowptr[r]; p < rowptr[r + 1]; ++p)
        if (col[p] >= lo && col[p] < hi) {
            ocol[q] = col[p] - lo;
            oval[q] = val[p];
            ++q;
        }
}

long long own_split(hipStream_t s, long long nr, const int* rowptr, const int* col, const double* val, int lo, int hi,
                    int* cnt, long long* off, long long* tiles, int* orp, int* ocol, double* oval) {
    if (nr <= 0) return 0;
    hipLaunchKernelGGL(k_own_count, dim3(grid_of(nr)), dim3(BT), 0, s, nr, rowptr, col, lo, hi, cnt);
    exclusive_scan(s, cnt, nr, off, tiles);
    long long tot = 0;
    (void)hipMemcpyAsync(&tot, off + nr, 8, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    if (ocol)
        hipLaunchKernelGGL(k_own_fill, dim3(grid_of(nr + 1)), dim3(BT), 0, s, nr, rowptr, col, val, lo, hi, off, orp,
                           ocol, oval);
    return tot;
}

// The halo exchange of the sharded step (ctx.cpp halo_build): one launch
// packs every peer's message and this rank's own block of the compact x.
// Messages: sbuf[t] = f[sidx[t]] for t < nsend (sidx = the rows each peer
// reads, each message closed by the index ldv: this rank's ||f||^2
// partial); own block: X[base + k] = f[k] for k < nrows, and P[0] = f[ldv].
__global__ __launch_bounds__(BT) void k_halo_pack(const double* __restrict__ f, int ldv, const int* __restrict__ sidx,
                                                  long long nsend, double* __restrict__ sbuf, double* __restrict__ X,
                                                  long long base, long long nrows, double* __restrict__ P) {
    const long long t = (long long)blockIdx.x * BT + threadIdx.x;
    if (t < nsend) {
        sbuf[t] = f[sidx[t]];
        return;
    }
    const long long k = t - nsend;
    if (k < nrows) X[base + k] = f[k];
    else if (k == nrows) P[0] = f[ldv];
}

void halo_pack(hipStream_t s, const double* f, int ldv, const int* sidx, long long nsend, double* sbuf, double* X,
               long long base, long long nrows, double* P) {
    const long long tot = nsend + nrows + 1;
    hipLaunchKernelGGL(k_halo_pack, dim3(grid_of(tot)), dim3(BT), 0, s, f, ldv, sidx, nsend, sbuf, X, base, nrows, P);
}

// X[t] = x[gidx[t]] (gidx < 0: 0.0): a global n-vector into the compact halo
// layout (ek_spmv / ek_spmv_host on a halo context)
__global__ __launch_bounds__(BT) void k_gather_idx(const double* __restrict__ x, const int* __restrict__ gidx,
                                                   long long len, double* __restrict__ X) {
    const long long t = (long long)blockIdx.x * BT + threadIdx.x;
    if (t < len) X[t] = gidx[t] >= 0 ? x[gidx[t]] : 0.0;
}

void gather_idx(hipStream_t s, const double* x, const int* gidx, long long len, double* X) {
    if (len > 0) hipLaunchKernelGGL(k_gather_idx, dim3(grid_of(len)), dim3(BT), 0, s, x, gidx, len, X);
}

}  // namespace dev
}  // namespace ek
