// Device helpers shared by the SpMV kernels (kernels_spmv.hip, kernels_panel.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "ek_internal.hpp"

namespace ek {
namespace dev {

// Block 0 of the chunk's last SpMV (StepFin::chk_dst set): the Lanczos
// mid-cycle check's copy.  Every thread of the block calls it after the
// finalize's publish (thread 0: alpha[step], offd[step], fn2_out).  The copy
// goes to pinned host memory, each thread's stores are released to the system
// (vmcnt(0) + the system-scope fence), and then one system-scope store of the
// sequence number (read from the host's pinned word: graph replays carry only
// the pointer) tells the polling host the slot is complete.  It runs beside
// the other blocks' rows, so no launch of its own and no queue barrier.
__device__ __forceinline__ void chk_mirror(const StepFin& f, int t, int nthreads) {
    __threadfence_block();
    __syncthreads();
    for (int i = t; i < f.chk_b; i += nthreads) {
        f.chk_dst[i] = f.alpha[i];
        f.chk_dst[f.chk_m + i] = f.offd[i];
        f.chk_dst[2 * f.chk_m + i] = f.chk_fn2[i];
    }
    __threadfence_system();
    __syncthreads();
    if (t == 0) {
        const unsigned seq = __hip_atomic_load(f.chk_seq_src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(f.chk_word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace dev
}  // namespace ek

// (lab: EK_OUT_STORE, an A/B build switch) the Lanczos step's vector outputs
// (the SpMV's y and basis column, the three-term residual f) stored
// 0: plainly; 1: non-temporal; 2: agent-scope (sc1, written through the L2)
#ifndef EK_OUT_STORE
#define EK_OUT_STORE 0
#endif
__device__ __forceinline__ void out_store(double* p, double v) {
#if EK_OUT_STORE == 1
    __builtin_nontemporal_store(v, p);
#elif EK_OUT_STORE == 2
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), static_cast<unsigned long long>(__double_as_longlong(v)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    *p = v;
#endif
}
__device__ __forceinline__ void out_store(float* p, float v) {
#if EK_OUT_STORE == 1
    __builtin_nontemporal_store(v, p);
#elif EK_OUT_STORE == 2
    __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    *p = v;
#endif
}
__device__ __forceinline__ void out_store2(double* p, double2 v) {
#if EK_OUT_STORE == 1
    typedef double nd2 __attribute__((ext_vector_type(2)));
    nd2 x;
    x.x = v.x;
    x.y = v.y;
    __builtin_nontemporal_store(x, reinterpret_cast<nd2*>(p));
#elif EK_OUT_STORE == 2
    out_store(p, v.x);
    out_store(p + 1, v.y);
#else
    *reinterpret_cast<double2*>(p) = v;
#endif
}

