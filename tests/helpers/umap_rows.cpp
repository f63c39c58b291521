// Test helper (not product code): dumps the iteration order of the LIVE
// libstdc++ std::unordered_map<uint32_t, float> rows that cKL's reader builds
// (pairs of every net, smaller id as the row, accumulated in net order —
// cKL.cpp:107-131), so tests can check the product's emulated row order
// (graph_build.cpp, hashtable_order) against the real container.
//
//   umap_rows rows <file.hgr>     one line per row: the keys in begin()->end() order
//   umap_rows buckets <nkeys>     bucket_count() after each of nkeys distinct inserts
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

int main(int argc, char** argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s rows <file.hgr> | buckets <nkeys>\n", argv[0]);
        return 2;
    }
    if (std::strcmp(argv[1], "buckets") == 0) {
        std::unordered_map<uint32_t, float> m;
        const long n = std::atol(argv[2]);
        for (long i = 0; i < n; ++i) {
            m[uint32_t(i * 7919u + 3u)] += 1.0f;
            std::printf("%zu\n", m.bucket_count());
        }
        return 0;
    }
    std::ifstream in(argv[2]);
    if (!in) return 1;
    std::string line;
    std::getline(in, line);
    uint64_t nets = 0, nodes = 0;
    std::istringstream(line) >> nets >> nodes;
    std::vector<std::unordered_map<uint32_t, float>> adj(nodes);
    std::vector<uint32_t> pins;
    for (uint64_t e = 0; e < nets && std::getline(in, line); ++e) {
        std::istringstream ss(line);
        pins.clear();
        uint32_t p;
        while (ss >> p) pins.push_back(p - 1);
        if (pins.size() < 2) continue;
        const float w = 1.0f / float(pins.size() - 1);
        for (size_t a = 0; a < pins.size(); ++a)
            for (size_t b = a + 1; b < pins.size(); ++b) {
                const uint32_t lo = pins[a] < pins[b] ? pins[a] : pins[b];
                const uint32_t hi = pins[a] < pins[b] ? pins[b] : pins[a];
                adj[lo][hi] += w;
            }
    }
    std::string out;
    char buf[16];
    for (const auto& row : adj) {
        bool first = true;
        for (const auto& kv : row) {
            if (!first) out += ' ';
            first = false;
            std::snprintf(buf, sizeof buf, "%u", kv.first);
            out += buf;
        }
        out += '\n';
    }
    std::fwrite(out.data(), 1, out.size(), stdout);
    return 0;
}
