// Test helper (CPU): ek::tridiag_qr_shifts, the interleaved restart shifts of
// the Lanczos driver, against ek::tridiag_qr_shift applied shift by shift —
// d, e and every recorded rotation bit for bit — on random symmetric
// tridiagonals with split points (zero, denormal-small and tiny
// off-diagonals), sizes 2..128 and the restart's shift counts.
// Built by tests/test_host_logic.py with host_linalg.cpp's own flags.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "ek_internal.hpp"

int main() {
    std::mt19937_64 g(20261018);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    int bad = 0, runs = 0;
    for (int trial = 0; trial < 600; ++trial) {
        const int m = trial < 450 ? 2 + int(U(g) * 127) : 100;
        const size_t M = static_cast<size_t>(m);
        std::vector<double> d(M), e(M), th(M), zl(M);
        for (int i = 0; i < m; ++i) {
            d[size_t(i)] = 4.0 + 3.0 * std::sin(0.37 * i + trial) + U(g);
            e[size_t(i)] = 0.5 + 2.0 * U(g);
            const double r = U(g);
            if (r < 0.05) e[size_t(i)] = 0.0;
            else if (r < 0.10) e[size_t(i)] = 1e-18;
            else if (r < 0.12) e[size_t(i)] *= 1e-9;
        }
        if (!ek::tridiag_eig(m, d.data(), e.data(), th.data(), zl.data(), nullptr)) continue;
        const int knew = std::max(1, int(U(g) * m * 0.5));
        std::vector<double> d1(d), e1(e), d2(d), e2(e);
        std::vector<ek::QRot> r1, r2;
        for (int i = knew; i < m; ++i) ek::tridiag_qr_shift(m, d1.data(), e1.data(), th[size_t(i)], r1);
        ek::tridiag_qr_shifts(m, d2.data(), e2.data(), th.data() + knew, m - knew, r2);
        bool ok = std::memcmp(d1.data(), d2.data(), size_t(m) * 8) == 0 &&
                  std::memcmp(e1.data(), e2.data(), size_t(m - 1) * 8) == 0 && r1.size() == r2.size();
        for (size_t k = 0; ok && k < r1.size(); ++k)
            ok = r1[k].p == r2[k].p && std::memcmp(&r1[k].c, &r2[k].c, 8) == 0 && std::memcmp(&r1[k].s, &r2[k].s, 8) == 0;
        if (!ok) {
            ++bad;
            std::printf("mismatch: trial %d m %d shifts %d\n", trial, m, m - knew);
        }
        ++runs;
    }
    std::printf("runs %d mismatches %d\n", runs, bad);
    return bad == 0 ? 0 : 1;
}
