// ORACLE — test infrastructure only (see eko_kl.cpp header).
#ifndef EKO_INTERNAL_HPP
#define EKO_INTERNAL_HPP
#include <cstdint>
#include <unordered_map>
#include <vector>

struct eko_graph {
    uint32_t nodes = 0, nets = 0;
    std::vector<int64_t> net_ptr;  // pins of net e: pins[net_ptr[e] .. net_ptr[e+1])
    std::vector<int32_t> pins;     // 0-based
    std::vector<std::unordered_map<uint32_t, float>> adj;  // cKL.cpp:37
    // cKL-order CSR (built lazily)
    std::vector<int32_t> rowptr, col, nfwd;
    std::vector<float> w;
};

#endif
