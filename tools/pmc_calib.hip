// PMC calibration lab (not shipped): kernels with a KNOWN byte count in the
// access widths the product's kernels use, one dispatch each, to be run
// under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes).
// The guide calibrates FETCH_SIZE only for 16-B/lane streaming reads (it
// reports half); this measures the widths of the Lanczos SpMV:
//   read16  : 16 B/lane coalesced stream           (the guide's case)
//   read8   : 8 B/lane coalesced stream            (f, the basis columns)
//   read4   : 4 B/lane coalesced stream            (the coded 32-bit words)
//   gatherX : 8 B random gathers into a table of X bytes, every line touched
//             by every XCD (the x gathers: one copy per XCD L2 = 8 X?)
//   write8  : 8 B/lane coalesced stores            (y, the basis column)
// Each read kernel folds its loads into one value per workgroup (a few KB of
// stores), so a dispatch's FETCH_SIZE is its reads.  The program prints the
// expected bytes per dispatch, in dispatch order.
// Build: make -C tools; run: tools/build/pmc_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

constexpr int T = 256;

template <class V>
__device__ __forceinline__ double as_d(const V& v);
template <>
__device__ __forceinline__ double as_d(const double2& v) { return v.x + v.y; }
template <>
__device__ __forceinline__ double as_d(const double& v) { return v; }
template <>
__device__ __forceinline__ double as_d(const unsigned& v) { return double(v); }

// grid-stride coalesced read of n elements of V; one double per block out
template <class V>
__global__ __launch_bounds__(T) void k_read(const V* __restrict__ a, size_t n, double* __restrict__ out) {
    double s = 0.0;
    for (size_t i = size_t(blockIdx.x) * T + threadIdx.x; i < n; i += size_t(gridDim.x) * T) s += as_d(a[i]);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __shared__ double w[T / 64];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = (w[0] + w[1]) + (w[2] + w[3]);
}

// `per` random 8-B gathers per thread into x[0:nx) (hash, no index loads)
__global__ __launch_bounds__(T) void k_gather(const double* __restrict__ x, unsigned nx, int per,
                                              double* __restrict__ out) {
    const unsigned t = blockIdx.x * T + threadIdx.x;
    double s = 0.0;
    for (int k = 0; k < per; ++k) {
        unsigned h = (t * 2654435761u) ^ (unsigned(k) * 40503u + 0x9E3779B9u);
        h ^= h >> 15;
        h *= 0x2c1b3c6du;
        h ^= h >> 12;
        s += x[h % nx];
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __shared__ double w[T / 64];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = (w[0] + w[1]) + (w[2] + w[3]);
}

__global__ __launch_bounds__(T) void k_write8(double* __restrict__ a, size_t n) {
    for (size_t i = size_t(blockIdx.x) * T + threadIdx.x; i < n; i += size_t(gridDim.x) * T) a[i] = double(i);
}

int main() {
    const size_t BYTES = size_t(64) << 20;  // 64 MiB streams: past every L2, inside the MALL
    void* a = nullptr;
    double* out = nullptr;
    CK(hipMalloc(&a, BYTES));
    CK(hipMalloc(reinterpret_cast<void**>(&out), size_t(1) << 20));
    CK(hipMemset(a, 0, BYTES));
    CK(hipDeviceSynchronize());
    const int grid = 4096;  // 16 waves per CU on 256 CUs
    std::printf("dispatch\tkernel\texpected_read_bytes\texpected_write_bytes\n");
    int d = 0;
    // streams (each twice: the second run's data may sit in the MALL; FETCH counts L2 misses either way)
    for (int rep = 0; rep < 2; ++rep) {
        k_read<double2><<<grid, T>>>(static_cast<const double2*>(a), BYTES / 16, out);
        std::printf("%d\tread16\t%zu\t%d\n", d++, BYTES, grid * 8);
        k_read<double><<<grid, T>>>(static_cast<const double*>(a), BYTES / 8, out);
        std::printf("%d\tread8\t%zu\t%d\n", d++, BYTES, grid * 8);
        k_read<unsigned><<<grid, T>>>(static_cast<const unsigned*>(a), BYTES / 4, out);
        std::printf("%d\tread4\t%zu\t%d\n", d++, BYTES, grid * 8);
    }
    // gathers: table sizes of x at 1x (1.6 MB), 2x (3.2 MB), 10x (16 MB); 1.3M gathers
    // like one SpMV at 1x (4 per thread over 1280 blocks), every line hit by every XCD
    for (size_t xb : {size_t(201920) * 8, size_t(403840) * 8, size_t(2019200) * 8}) {
        const int blocks = 1280, per = 4;
        k_gather<<<blocks, T>>>(static_cast<const double*>(a), unsigned(xb / 8), per, out);
        std::printf("%d\tgather_table_%zuB_x%d_gathers\t%zu (one copy)\t%d\n", d++, xb, blocks * T * per, xb,
                    blocks * 8);
    }
    k_write8<<<grid, T>>>(static_cast<double*>(a), BYTES / 8);
    std::printf("%d\twrite8\t0\t%zu\n", d++, BYTES);
    CK(hipDeviceSynchronize());
    CK(hipGetLastError());
    CK(hipFree(a));
    CK(hipFree(out));
    return 0;
}
