// Test helper (tests/test_sanitizers.py only): the GPU-side C-ABI entry points
// the host sources call (ctx.cpp is HIP code), as a machine without a usable
// gfx950 device sees them — every one fails with EK_EHIP like the real
// library there — so the host code (CLI argument and file handling, the
// solve pipeline up to the GPU, ingest, clique expansions, EIG I/O, the
// restart QR) can be built with -fsanitize=address,undefined by g++ alone.
#include "../../eig-kl-algorithm_amd/csrc/ek_internal.hpp"

namespace {
int absent(const char* what) {
    ek::set_error("%s: no HIP device available (sanitizer build)", what);
    return EK_EHIP;
}
}  // namespace

int ek::spmv_setup_hgr(ek_ctx*, const ek_hgr&, int32_t*) { return absent("ek_spmv_setup_pins"); }

void ek::ctx_ranks(ek_ctx*, int* rank, int* nranks) {
    if (rank) *rank = 0;
    if (nranks) *nranks = 1;
}

extern "C" {
int ek_init(int, ek_ctx** out) {
    if (out) *out = nullptr;
    return absent("ek_init");
}
void ek_destroy(ek_ctx*) {}
void ek_lanczos_default_opts(ek_lanczos_opts* o) {
    if (!o) return;
    *o = ek_lanczos_opts{0, 1000, 1e-10, 1, 0, 1, 8};
}
int ek_spmv_setup(ek_ctx*, int64_t, int64_t, int64_t, const int32_t*, const int32_t*, const double*) {
    return absent("ek_spmv_setup");
}
int ek_spmv_setup_pins(ek_ctx*, int64_t, int64_t, const int64_t*, const int32_t*, int32_t*) {
    return absent("ek_spmv_setup_pins");
}
int ek_lanczos_fiedler(ek_ctx*, const ek_lanczos_opts*, double*, double*, ek_lanczos_stats*) {
    return absent("ek_lanczos_fiedler");
}
int ek_kl_graph_setup(ek_ctx*, int64_t, const int32_t*, const int32_t*, const float*) { return absent("kl"); }
int ek_kl_nets_setup(ek_ctx*, int64_t, const int64_t*, const int32_t*) { return absent("kl"); }
int ek_kl_set_partition(ek_ctx*, const int32_t*, int64_t, const int32_t*, int64_t) { return absent("kl"); }
int ek_kl_set_partition_fiedler(ek_ctx*, double*, int64_t*, int64_t*) { return absent("kl"); }
int ek_kl_run(ek_ctx*, int32_t, ek_swap*, int64_t, ek_kl_result*) { return absent("kl"); }
}
