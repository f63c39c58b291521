// LDS round-trip lab (not part of the product): what one wave of the KL swap
// loop's 512-thread workgroup pays for a dependent LDS read while the other
// seven waves (a) sit in s_barrier, (b) poll one LDS word in a tight loop,
// (c) poll it with s_sleep between polls, (d) issue their own independent LDS
// reads, (e) run dependent VALU chains.  Wave 0 chases a pointer chain through
// LDS (one ds_read_b32 a step); the shader clock (s_memtime) around the chain.
// Build: hipcc --offload-arch=gfx950 -O3 tools/lds_lab.hip -o /tmp/lds_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

constexpr int WORDS = 8192;  // 32 KB chain table

template <int MODE>
__global__ __launch_bounds__(512) void lab(int steps, unsigned long long* out) {
    __shared__ int tab[WORDS];
    __shared__ int flag;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < WORDS; i += 512) tab[i] = (i * 2654435761u + 977) % WORDS;  // a scattered chain
    if (tid == 0) flag = 0;
    __syncthreads();
    if (wv == 0) {
        int r = lane * 37;
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        for (int s = 0; s < steps; ++s) r = tab[r];
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) {
            out[0] = t1 - t0;
            out[1] = unsigned(r);
        }
        __hip_atomic_store(&flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if constexpr (MODE == 1 || MODE == 2) {
        while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) == 0)
            if constexpr (MODE == 2) __builtin_amdgcn_s_sleep(1);
    } else if constexpr (MODE == 3) {
        int acc = 0;
        for (int k = 0; __builtin_amdgcn_readfirstlane(__hip_atomic_load(&flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) == 0; ++k) {
            int v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = tab[(lane * 64 + u * 512 + k * 7) % WORDS];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u];
        }
        if (acc == 12345) out[2] = 1;
    } else if constexpr (MODE == 4) {
        float x = float(lane);
        while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) == 0)
#pragma unroll
            for (int u = 0; u < 64; ++u) x = x * 1.0001f + 0.5f;
        if (x == 1.0f) out[2] = 1;
    }
    __syncthreads();
}

int main() {
    unsigned long long* d;
    CK(hipMalloc(&d, 64));
    unsigned long long h[3];
    const int steps = 4096;
    const char* names[5] = {"others in s_barrier", "others polling one LDS word", "others polling with s_sleep 1",
                            "others streaming independent LDS reads", "others running VALU chains"};
    for (int rep = 0; rep < 2; ++rep)
        for (int m = 0; m < 5; ++m) {
            switch (m) {
                case 0: hipLaunchKernelGGL(lab<0>, dim3(1), dim3(512), 0, 0, steps, d); break;
                case 1: hipLaunchKernelGGL(lab<1>, dim3(1), dim3(512), 0, 0, steps, d); break;
                case 2: hipLaunchKernelGGL(lab<2>, dim3(1), dim3(512), 0, 0, steps, d); break;
                case 3: hipLaunchKernelGGL(lab<3>, dim3(1), dim3(512), 0, 0, steps, d); break;
                default: hipLaunchKernelGGL(lab<4>, dim3(1), dim3(512), 0, 0, steps, d); break;
            }
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h, d, 24, hipMemcpyDeviceToHost));
            if (rep) std::printf("%-42s %.1f cycles per dependent ds_read_b32\n", names[m], double(h[0]) / steps);
        }
    return 0;
}
