// .hgr ingest / write / seeded synthetic generator (host side).
//
// Reader semantics follow the reference readers (cKL.cpp:92-116,
// cEIG.cpp:177-182,91-101): the header's first two integers are
// `nets nodes`; then exactly `nets` lines are consumed, one net per line,
// pins are 1-based unsigned integers separated by whitespace (a line ends the
// net; extraction stops at the first non-numeric token, like `ss >> node`).
// Missing lines give empty nets (getline failure).  Unlike the reference,
// pin ids outside [1, nodes] are rejected (they are out-of-bounds writes
// there) and the parse is two-pass and multi-threaded.
#include <atomic>
#include <cerrno>
#include <memory>
#include <cmath>
#include <cstring>
#include <mutex>
#include <random>

#include "ek_internal.hpp"

namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

// Parse unsigned integers on [p, end) (one line); calls emit(value).  Returns
// false on overflow.  Stops at the first non-numeric token.
template <class Emit>
inline bool parse_line(const char* p, const char* end, Emit&& emit) {
    while (p < end) {
        while (p < end && is_space(*p)) ++p;
        if (p >= end) break;
        if (*p == '+') ++p;
        if (p >= end || *p < '0' || *p > '9') break;
        uint64_t v = 0;
        while (p < end && *p >= '0' && *p <= '9') {
            v = v * 10 + uint64_t(*p - '0');
            if (v > 0xffffffffull) return false;
            ++p;
        }
        emit(v);
        if (p < end && !is_space(*p)) break;  // e.g. "12x": stream stops after 12
    }
    return true;
}

// the whole file (not zero-filled first: dvec leaves its elements uninitialised)
void slurp(const char* path, ek::dvec<char>& buf) {
    FILE* f = std::fopen(path, "rb");
    if (!f) ek::fail(EK_EIO, "cannot open %s: %s", path, std::strerror(errno));
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    buf.resize(size_t(sz > 0 ? sz : 0));
    const size_t got = sz > 0 ? std::fread(buf.data(), 1, size_t(sz), f) : 0;
    std::fclose(f);
    buf.resize(got);
}

// The file buffer and the per-thread pin lists of ek_hgr_read, kept across
// calls (a service re-reading circuits of similar size): fresh ones cost a
// page fault per 4 KB on first touch, ~1 ms a read of the ibm18-shape file.
// One caller at a time uses them; a concurrent read gets its own.
// The result arrays (net_ptr, pins) of a freed ek_hgr come back here too
// (ek_hgr_free) and are handed to the next read: in a solve loop the heap
// churn between reads otherwise gave them fresh pages every time.
struct ReadCache {
    std::mutex mu;
    ek::dvec<char> buf;
    std::vector<ek::dvec<int32_t>> part;
    ek::dvec<int64_t> net_ptr;
    ek::dvec<int32_t> pins;
};
ReadCache& read_cache() {
    static ReadCache c;
    return c;
}

// xoshiro256** seeded by splitmix64: the generator's only RNG (seeded, unlike
// circuit_generator.py's module-level `random`).
struct Rng {
    uint64_t s[4];
    explicit Rng(uint64_t seed) {
        for (auto& x : s) {
            seed += 0x9e3779b97f4a7c15ull;
            uint64_t z = seed;
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
            x = z ^ (z >> 31);
        }
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9;
        const uint64_t t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    double uniform01() { return double(next() >> 11) * 0x1.0p-53; }
    uint64_t below(uint64_t n) {  // unbiased (Lemire)
        unsigned __int128 m = (unsigned __int128)next() * n;
        uint64_t l = uint64_t(m);
        if (l < n) {
            const uint64_t t = (0 - n) % n;
            while (l < t) {
                m = (unsigned __int128)next() * n;
                l = uint64_t(m);
            }
        }
        return uint64_t(m >> 64);
    }
};

}  // namespace

extern "C" {

int ek_hgr_read(const char* path, ek_hgr** out) {
    EK_TRY
    if (!path || !out) ek::fail(EK_EINVAL, "ek_hgr_read: null argument");
    ek::PhaseTimer pt("hgr_read");
    std::unique_lock<std::mutex> cache_lk(read_cache().mu, std::try_to_lock);
    ek::dvec<char> own_buf;
    std::vector<ek::dvec<int32_t>> own_part;
    ek::dvec<char>& buf = cache_lk.owns_lock() ? read_cache().buf : own_buf;
    std::vector<ek::dvec<int32_t>>& part = cache_lk.owns_lock() ? read_cache().part : own_part;
    slurp(path, buf);
    pt.mark("slurp");
    const char* b = buf.empty() ? "" : buf.data();  // (memchr must not see a null pointer)
    const char* e = b + buf.size();
    const char* nl = static_cast<const char*>(std::memchr(b, '\n', size_t(e - b)));
    const char* hend = nl ? nl : e;
    uint64_t hv[2] = {0, 0};
    int nh = 0;
    parse_line(b, hend, [&](uint64_t v) {
        if (nh < 2) hv[nh] = v;
        ++nh;
    });
    if (nh < 2) ek::fail(EK_EINVAL, "%s: header must be '<nets> <nodes>'", path);
    auto h = std::make_unique<ek_hgr>();
    if (cache_lk.owns_lock()) {  // a freed result's arrays (capacity kept)
        h->net_ptr.swap(read_cache().net_ptr);
        h->pins.swap(read_cache().pins);
    }
    h->nets = int64_t(hv[0]);
    h->nodes = int64_t(hv[1]);
    if (h->nodes > INT32_MAX || h->nets > INT32_MAX) ek::fail(EK_EINVAL, "%s: sizes exceed int32", path);
    const int64_t nets = h->nets;
    // One parallel pass over whole-line byte chunks: each thread counts its
    // lines (so it knows the net index of its first one), then parses them
    // into its own pin list; the lists are concatenated in net order.  Lines
    // past `nets` are ignored; nets past the last line are empty (getline
    // failure).
    const char* body = nl ? nl + 1 : e;
    const int64_t bytes = int64_t(e - body);
    const int T = int(std::max<int64_t>(1, std::min<int64_t>(ek::host_threads(), bytes / (256 * 1024))));
    std::vector<const char*> cs(size_t(T) + 1, e);
    cs[0] = body;
    for (int t = 1; t < T; ++t) {  // chunk starts at line starts
        const char* q = body + bytes * t / T;
        if (q > cs[size_t(t) - 1]) {
            const char* r = static_cast<const char*>(std::memchr(q - 1, '\n', size_t(e - (q - 1))));
            q = r ? r + 1 : e;
        }
        cs[size_t(t)] = std::max(q, cs[size_t(t) - 1]);
    }
    std::vector<int64_t> lines(size_t(T) + 1, 0);  // lines starting in chunk t
    ek::run_threads(T, [&](int t) {
        int64_t c = 0;
        for (const char* p = cs[size_t(t)]; p < cs[size_t(t) + 1];) {
            const char* r = static_cast<const char*>(std::memchr(p, '\n', size_t(cs[size_t(t) + 1] - p)));
            ++c;
            p = r ? r + 1 : cs[size_t(t) + 1];
        }
        lines[size_t(t) + 1] = c;
    });
    for (int t = 0; t < T; ++t) lines[size_t(t) + 1] += lines[size_t(t)];
    pt.mark("lines");
    h->net_ptr.assign(size_t(nets) + 1, 0);
    if (part.size() < size_t(T)) part.resize(size_t(T));
    for (int t = 0; t < T; ++t) part[size_t(t)].clear();  // (capacity kept)
    std::atomic<bool> bad{false};
    std::atomic<int64_t> bad_pin{-1};
    std::atomic<int64_t> raw_pairs{0};
    ek::run_threads(T, [&](int t) {
        int64_t pairs = 0;  // this thread's nets' k (k - 1), k >= 2
        int64_t net = lines[size_t(t)];
        auto& pv = part[size_t(t)];
        const char* p = cs[size_t(t)];
        const char* const e = cs[size_t(t) + 1];
        // a pin takes at least two bytes (a digit and a separator) but the last
        pv.resize(size_t((e - p) / 2 + 16));
        int32_t* const out = pv.data();
        size_t cnt = 0;
        const int64_t nodes = h->nodes;
        auto emit = [&](uint64_t v) {
            if (v < 1 || int64_t(v) > nodes) bad_pin = int64_t(v);
            out[cnt++] = int32_t(v) - 1;
        };
        // one pass per line over digits, blanks and the newline; any other
        // byte (or a token over 10 digits) re-parses the line with
        // parse_line, the reference-semantics reader
        while (p < e && net < nets) {
            const char* const ls = p;
            const size_t before = cnt;
            uint64_t v = 0;
            int nd = 0;
            bool slow = false;
            for (; p < e; ++p) {
                const unsigned c = static_cast<unsigned char>(*p);
                const unsigned d = c - unsigned('0');
                if (d < 10u) {
                    v = v * 10u + d;
                    if (++nd > 10) {
                        slow = true;
                        break;
                    }
                } else if (c == ' ' || c == '\t' || c == '\r') {
                    if (nd) {
                        if (v > 0xffffffffull) {
                            slow = true;
                            break;
                        }
                        emit(v);
                    }
                    v = 0;
                    nd = 0;
                } else {
                    slow = c != '\n';
                    break;
                }
            }
            if (!slow && nd) {
                if (v > 0xffffffffull) slow = true;
                else emit(v);
            }
            if (slow) {
                cnt = before;
                const char* r = static_cast<const char*>(std::memchr(ls, '\n', size_t(e - ls)));
                const char* le = r ? r : e;
                if (!parse_line(ls, le, emit)) bad = true;
                p = le;
            }
            const int64_t k = int64_t(cnt - before);
            h->net_ptr[size_t(net) + 1] = k;
            pairs += k >= 2 ? k * (k - 1) : 0;
            if (p < e) ++p;  // the newline
            ++net;
        }
        pv.resize(cnt);
        raw_pairs += pairs;
    });
    pt.mark("parse (threads)");
    if (bad) ek::fail(EK_EINVAL, "%s: pin id overflows uint32", path);
    if (bad_pin.load() >= 0)
        ek::fail(EK_EINVAL, "%s: pin id %lld outside [1, %lld]", path, (long long)bad_pin.load(),
                 (long long)h->nodes);
    for (int64_t i = 0; i < nets; ++i) h->net_ptr[size_t(i) + 1] += h->net_ptr[size_t(i)];
    h->raw_pairs = raw_pairs.load();
    pt.mark("net prefix");
    h->pins.resize(size_t(h->net_ptr.back()));
    std::vector<size_t> off(size_t(T) + 1, 0);
    for (int t = 0; t < T; ++t) off[size_t(t) + 1] = off[size_t(t)] + part[size_t(t)].size();
    ek::run_threads(T, [&](int t) {
        if (!part[size_t(t)].empty())
            std::memcpy(h->pins.data() + off[size_t(t)], part[size_t(t)].data(), part[size_t(t)].size() * 4);
    });
    // (a file far smaller than the cached buffers would keep them: shrink
    // what exceeds 4x this read's needs)
    if (buf.capacity() > 4 * buf.size() + (size_t(1) << 20)) ek::dvec<char>().swap(buf);
    pt.mark("pins copy");
    *out = h.release();
    return EK_OK;
    EK_CATCH
}

int ek_hgr_from_pins(int64_t nets, int64_t nodes, const int64_t* net_ptr, const int32_t* pins, ek_hgr** out) {
    EK_TRY
    if (!net_ptr || !out || nets < 0 || nodes < 0 || nodes > INT32_MAX) ek::fail(EK_EINVAL, "ek_hgr_from_pins: bad argument");
    auto h = std::make_unique<ek_hgr>();
    h->nets = nets;
    h->nodes = nodes;
    h->net_ptr.assign(net_ptr, net_ptr + nets + 1);
    if (h->net_ptr[0] != 0) ek::fail(EK_EINVAL, "net_ptr[0] must be 0");
    for (int64_t i = 0; i < nets; ++i)
        if (h->net_ptr[size_t(i) + 1] < h->net_ptr[size_t(i)]) ek::fail(EK_EINVAL, "net_ptr not monotone");
    h->pins.assign(pins, pins + h->net_ptr.back());
    for (int32_t v : h->pins)
        if (v < 0 || v >= nodes) ek::fail(EK_EINVAL, "pin %d outside [0, %lld)", v, (long long)nodes);
    *out = h.release();
    return EK_OK;
    EK_CATCH
}

// circuit_generator.py:41-59 restated with a seeded RNG: net size from the
// cumulative table {2:84,3:2,4:6,5:2,6:4,8:2}/100 (r <= cumulative, as
// _choose_net_size :22-30), then `size` distinct uniform nodes, sorted
// (_select_nodes_for_net :32-39).
int ek_hgr_generate(double multiplier, uint64_t seed, ek_hgr** out) {
    EK_TRY
    if (!out || !(multiplier > 0)) ek::fail(EK_EINVAL, "ek_hgr_generate: bad argument");
    auto h = std::make_unique<ek_hgr>();
    h->nodes = int64_t(std::floor(201920.0 * multiplier));
    h->nets = int64_t(std::floor(210613.0 * multiplier));
    if (h->nodes < 2 || h->nodes > INT32_MAX) ek::fail(EK_EINVAL, "ek_hgr_generate: bad size");
    static const int sizes[6] = {2, 3, 4, 5, 6, 8};
    static const int cum[6] = {84, 86, 92, 94, 98, 100};
    Rng rng(seed);
    h->net_ptr.reserve(size_t(h->nets) + 1);
    h->pins.reserve(size_t(h->nets) * 3);
    h->net_ptr.push_back(0);
    int32_t pick[8];
    for (int64_t e = 0; e < h->nets; ++e) {
        const double r = rng.uniform01() * 100.0;
        int k = 2;
        for (int t = 0; t < 6; ++t)
            if (r <= cum[t]) {
                k = sizes[t];
                break;
            }
        if (k > h->nodes) k = int(h->nodes);
        for (int j = 0; j < k;) {
            const int32_t v = int32_t(rng.below(uint64_t(h->nodes)));
            bool dup = false;
            for (int q = 0; q < j; ++q) dup |= pick[q] == v;
            if (!dup) pick[j++] = v;
        }
        std::sort(pick, pick + k);
        h->pins.insert(h->pins.end(), pick, pick + k);
        h->net_ptr.push_back(int64_t(h->pins.size()));
    }
    *out = h.release();
    return EK_OK;
    EK_CATCH
}

// Largest connected component (union-find over each net's pins), nets kept in
// file order with their pins renumbered by ascending original id.
int ek_hgr_largest_component(const ek_hgr* h, ek_hgr** out, int32_t* node_map) {
    EK_TRY
    if (!h || !out) ek::fail(EK_EINVAL, "ek_hgr_largest_component: null argument");
    const int64_t n = h->nodes;
    std::vector<int32_t> parent(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) parent[size_t(i)] = int32_t(i);
    auto find = [&](int32_t x) {
        while (parent[size_t(x)] != x) {
            parent[size_t(x)] = parent[size_t(parent[size_t(x)])];
            x = parent[size_t(x)];
        }
        return x;
    };
    for (int64_t e = 0; e < h->nets; ++e) {
        const int64_t p0 = h->net_ptr[size_t(e)], p1 = h->net_ptr[size_t(e) + 1];
        if (p1 - p0 < 2) continue;
        int32_t a = find(h->pins[size_t(p0)]);
        for (int64_t p = p0 + 1; p < p1; ++p) {
            const int32_t b = find(h->pins[size_t(p)]);
            if (a == b) continue;
            if (a < b) parent[size_t(b)] = a;  // the root is the component's smallest id
            else {
                parent[size_t(a)] = b;
                a = b;
            }
        }
    }
    std::vector<int64_t> size(static_cast<size_t>(n), 0);
    int32_t best = -1;
    for (int64_t i = 0; i < n; ++i) ++size[size_t(find(int32_t(i)))];
    for (int64_t i = 0; i < n; ++i)  // ties: the root (= smallest id) that comes first
        if (parent[size_t(i)] == i && (best < 0 || size[size_t(i)] > size[size_t(best)])) best = int32_t(i);
    std::vector<int32_t> nid(static_cast<size_t>(n), -1);
    int32_t m = 0;
    for (int64_t i = 0; i < n; ++i)
        if (best >= 0 && find(int32_t(i)) == best) nid[size_t(i)] = m++;
    auto c = std::make_unique<ek_hgr>();
    c->nodes = m;
    c->net_ptr.push_back(0);
    for (int64_t e = 0; e < h->nets; ++e) {
        const int64_t p0 = h->net_ptr[size_t(e)], p1 = h->net_ptr[size_t(e) + 1];
        if (p1 == p0 || nid[size_t(h->pins[size_t(p0)])] < 0) continue;  // every pin of a kept net is kept
        for (int64_t p = p0; p < p1; ++p) c->pins.push_back(nid[size_t(h->pins[size_t(p)])]);
        c->net_ptr.push_back(int64_t(c->pins.size()));
    }
    c->nets = int64_t(c->net_ptr.size()) - 1;
    if (node_map) std::copy(nid.begin(), nid.end(), node_map);
    *out = c.release();
    return EK_OK;
    EK_CATCH
}

int ek_hgr_write(const ek_hgr* h, const char* path) {
    EK_TRY
    if (!h || !path) ek::fail(EK_EINVAL, "ek_hgr_write: null argument");
    FILE* f = std::fopen(path, "w");
    if (!f) ek::fail(EK_EIO, "cannot write %s: %s", path, std::strerror(errno));
    std::string out;
    out.reserve(size_t(h->pins.size()) * 8 + 64);
    out += std::to_string(h->nets) + " " + std::to_string(h->nodes) + "\n";
    char tmp[16];
    for (int64_t e = 0; e < h->nets; ++e) {
        for (int64_t p = h->net_ptr[size_t(e)]; p < h->net_ptr[size_t(e) + 1]; ++p) {
            if (p != h->net_ptr[size_t(e)]) out += ' ';
            const int len = snprintf(tmp, sizeof tmp, "%d", h->pins[size_t(p)] + 1);
            out.append(tmp, size_t(len));
        }
        out += '\n';
    }
    const size_t wr = std::fwrite(out.data(), 1, out.size(), f);
    std::fclose(f);
    if (wr != out.size()) ek::fail(EK_EIO, "short write to %s", path);
    return EK_OK;
    EK_CATCH
}

int ek_hgr_dims(const ek_hgr* h, int64_t* nets, int64_t* nodes, int64_t* pins) {
    if (!h) {
        ek::set_error("ek_hgr_dims: null handle");
        return EK_EINVAL;
    }
    if (nets) *nets = h->nets;
    if (nodes) *nodes = h->nodes;
    if (pins) *pins = int64_t(h->pins.size());
    return EK_OK;
}

int ek_hgr_copy_pins(const ek_hgr* h, int64_t* net_ptr, int32_t* pins) {
    if (!h) {
        ek::set_error("ek_hgr_copy_pins: null handle");
        return EK_EINVAL;
    }
    if (net_ptr) std::copy(h->net_ptr.begin(), h->net_ptr.end(), net_ptr);
    if (pins) std::copy(h->pins.begin(), h->pins.end(), pins);
    return EK_OK;
}

void ek_hgr_free(ek_hgr* h) {
    if (!h) return;
    {
        ReadCache& c = read_cache();
        std::unique_lock<std::mutex> lk(c.mu, std::try_to_lock);
        if (lk.owns_lock()) {  // keep the larger arrays for the next read
            if (h->net_ptr.capacity() > c.net_ptr.capacity()) c.net_ptr.swap(h->net_ptr);
            if (h->pins.capacity() > c.pins.capacity()) c.pins.swap(h->pins);
            c.net_ptr.clear();
            c.pins.clear();
        }
    }
    delete h;
}

}  // extern "C"
