// Median split and the pre_saved_EIG file format (host side).
//   median / split : cEIG.cpp:55-65, 207-209, 218 (bit = median > v[i])
//   writer         : cEIG.cpp:213-220 (ostream setprecision(12) == %.12g)
//   reader         : cKL.cpp:155-174 (skip 2 lines; "node side value" rows;
//                    split[side].push_back(node) in file order)
#include <cerrno>
#include <cmath>
#include <cstring>
#include <string>

#include "ek_internal.hpp"

extern "C" {

int ek_median_split(int64_t n, const double* v, double* median_out, uint8_t* bits_out) {
    EK_TRY
    if (n <= 0 || !v) ek::fail(EK_EINVAL, "ek_median_split: empty vector");
    // The values at ranks hi = n/2 (and hi-1 for even n, whose mean is the
    // median) are the ones nth_element over all of v returns.  Large n: a
    // fixed-stride sample brackets them between two pivots, one pass counts
    // the values below the lower pivot and keeps those inside the bracket,
    // and nth_element runs on that ~2 % only; a bracket that misses (or a NaN
    // in v) falls back to the whole vector.
    const size_t hi = size_t(n / 2), rlo = n % 2 == 0 ? hi - 1 : hi;
    std::vector<double> s;
    size_t below = 0;
    bool bracketed = false;
    if (n >= (int64_t(1) << 16)) {
        constexpr size_t NS = 4096, MARGIN = 96;  // sample size; pivots +-MARGIN samples around the median's
        std::vector<double> smp(NS);
        for (size_t k = 0; k < NS; ++k) smp[k] = v[size_t(k * size_t(n) / NS)];
        std::sort(smp.begin(), smp.end());
        const double plo = smp[NS / 2 - MARGIN], phi = smp[NS / 2 + MARGIN];
        // one pass on the host threads: each counts the values below the
        // bracket and keeps those inside it (in index order, concatenated)
        const int T = int(std::min<int64_t>(ek::host_threads(), std::max<int64_t>(1, n / 32768)));
        std::vector<std::vector<double>> part(static_cast<size_t>(T));
        std::vector<size_t> nb(static_cast<size_t>(T), 0);
        std::vector<char> nan(static_cast<size_t>(T), 0);
        ek::run_threads(T, [&](int t) {
            const int64_t lo = n * t / T, hi2 = n * (t + 1) / T;
            auto& ps = part[size_t(t)];
            ps.reserve(size_t(hi2 - lo) / 16 + 16);
            size_t b = 0;
            bool bad = false;
            for (int64_t i = lo; i < hi2; ++i) {
                const double x = v[i];
                if (x < plo) ++b;
                else if (x <= phi) ps.push_back(x);
                else bad |= x != x;
            }
            nb[size_t(t)] = b;
            nan[size_t(t)] = bad;
        });
        bool any_nan = false;
        for (int t = 0; t < T; ++t) {
            below += nb[size_t(t)];
            any_nan |= nan[size_t(t)] != 0;
            s.insert(s.end(), part[size_t(t)].begin(), part[size_t(t)].end());
        }
        bracketed = !any_nan && below <= rlo && hi < below + s.size();
    }
    if (!bracketed) {
        s.assign(v, v + n);
        below = 0;
    }
    const size_t h = hi - below;
    std::nth_element(s.begin(), s.begin() + std::ptrdiff_t(h), s.end());
    double med = s[h];
    if (n % 2 == 0) {  // mean of the two middle values
        const double lo = *std::max_element(s.begin(), s.begin() + std::ptrdiff_t(h));
        med = (lo + med) / 2.0;
    }
    if (median_out) *median_out = med;
    if (bits_out)
        ek::parallel_for(n, [&](int64_t lo, int64_t hi2) {
            for (int64_t i = lo; i < hi2; ++i) bits_out[i] = uint8_t(med > v[i]);
        });
    return EK_OK;
    EK_CATCH
}

int ek_align_sign(int64_t n, double* v, const double* ref) {
    if (n < 0 || !v || !ref) {
        ek::set_error("ek_align_sign: bad argument");
        return EK_EINVAL;
    }
    double dot = 0.0;
    for (int64_t i = 0; i < n; ++i) dot += v[i] * ref[i];
    if (dot < 0)
        for (int64_t i = 0; i < n; ++i) v[i] = -v[i];
    return EK_OK;
}

int ek_eig_write(const char* path, int64_t n, double lambda, double median, const uint8_t* bits, const double* v) {
    EK_TRY
    if (!path || n < 0 || (n && (!bits || !v))) ek::fail(EK_EINVAL, "ek_eig_write: bad argument");
    FILE* f = std::fopen(path, "w");
    if (!f) ek::fail(EK_EIO, "Error opening output file: %s (%s)", path, std::strerror(errno));
    std::string out;
    out.reserve(size_t(n) * 32 + 64);
    char buf[96];
    int len = snprintf(buf, sizeof buf, "%.12g\n%.12g\n", lambda, median);
    out.append(buf, size_t(len));
    for (int64_t i = 0; i < n; ++i) {
        len = snprintf(buf, sizeof buf, "%lld\t%d\t%.12g\n", (long long)i, int(bits[i] != 0), v[i]);
        out.append(buf, size_t(len));
    }
    const size_t wr = std::fwrite(out.data(), 1, out.size(), f);
    std::fclose(f);
    if (wr != out.size()) ek::fail(EK_EIO, "short write to %s", path);
    return EK_OK;
    EK_CATCH
}

int ek_eig_read(const char* path, int64_t n, double* lambda, double* median, uint8_t* bits, double* v,
                int32_t* order0, int64_t* n0, int32_t* order1, int64_t* n1) {
    EK_TRY
    if (!path || n < 0) ek::fail(EK_EINVAL, "ek_eig_read: bad argument");
    FILE* f = std::fopen(path, "rb");
    if (!f) ek::fail(EK_EIO, "Error: EIG file not found (%s)", path);
    std::string buf;
    {
        char tmp[1 << 16];
        size_t got;
        while ((got = std::fread(tmp, 1, sizeof tmp, f)) > 0) buf.append(tmp, got);
        std::fclose(f);
    }
    const char* p = buf.c_str();
    const char* e = p + buf.size();
    auto next_line = [&](const char*& q) -> const char* {  // returns line start, advances q
        const char* s = q;
        const char* nl = static_cast<const char*>(std::memchr(q, '\n', size_t(e - q)));
        q = nl ? nl + 1 : e;
        return s;
    };
    const char* q = p;
    const double lam = std::strtod(next_line(q), nullptr);
    const double med = std::strtod(next_line(q), nullptr);
    int64_t c0 = 0, c1 = 0;
    while (q < e) {
        const char* s = next_line(q);
        char* endp = nullptr;
        const long long node = std::strtoll(s, &endp, 10);
        if (endp == s) continue;  // blank line
        const char* t = endp;
        const long long side = std::strtoll(t, &endp, 10);
        if (endp == t) ek::fail(EK_EINVAL, "%s: malformed row", path);
        t = endp;
        const double val = std::strtod(t, &endp);
        if (node < 0 || node >= n || (side != 0 && side != 1))
            ek::fail(EK_EINVAL, "%s: row (%lld, %lld) out of range for n=%lld", path, node, side, (long long)n);
        if (bits) bits[node] = uint8_t(side);
        if (v) v[node] = val;
        if (side == 0) {
            if (order0) order0[c0] = int32_t(node);
            ++c0;
        } else {
            if (order1) order1[c1] = int32_t(node);
            ++c1;
        }
        if (c0 + c1 > n) ek::fail(EK_EINVAL, "%s: more than n=%lld rows", path, (long long)n);
    }
    if (lambda) *lambda = lam;
    if (median) *median = med;
    if (n0) *n0 = c0;
    if (n1) *n1 = c1;
    return EK_OK;
    EK_CATCH
}

}  // extern "C"
