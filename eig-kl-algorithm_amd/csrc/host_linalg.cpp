// Small host-side linear algebra for the implicitly restarted Lanczos driver
// (the m x m projected problem, m = ncv <= 128).  The n-length work runs on
// the GPU (kernels_lanczos.hip); these routines restate the two small dense
// steps of Spectra's SymEigsSolver (the solver cEIG.cpp:195-198 calls):
// TridiagEigen of the projected H and the shifted QR sweeps of its restart.
#include <cfloat>
#include <algorithm>
#include <cmath>
#include <numeric>

#include "ek_internal.hpp"

namespace ek {

// sqrt(a^2 + b^2) without hypot's scaling: the entries of the projected
// Laplacian are O(1e-20 .. 1e4), far from over/underflow, and std::hypot was
// a third of the time of these routines
static inline double pyth(double a, double b) { return std::sqrt(a * a + b * b); }

// Implicit QL with Wilkinson-type shifts on a symmetric tridiagonal matrix
// (diagonal d, off-diagonal e[i] = T(i+1, i)).  Eigenvalues ascending in
// evals; zlast[j] = last component of eigenvector j (the Ritz estimates need
// only that row); the full eigenvector matrix (col-major) when Z != nullptr.
bool tridiag_eig(int m, const double* d_in, const double* e_in, double* evals, double* zlast, double* Z) {
    std::vector<double> d(d_in, d_in + m), e(size_t(m), 0.0), zl(size_t(m), 0.0);
    for (int i = 0; i + 1 < m; ++i) e[size_t(i)] = e_in[i];
    zl[size_t(m - 1)] = 1.0;
    if (Z)
        for (int j = 0; j < m; ++j)
            for (int k = 0; k < m; ++k) Z[size_t(j) * m + k] = (j == k) ? 1.0 : 0.0;
    for (int l = 0; l < m; ++l) {
        int iter = 0;
        for (;;) {
            int mm = l;
            for (; mm < m - 1; ++mm) {
                const double dd = std::fabs(d[size_t(mm)]) + std::fabs(d[size_t(mm) + 1]);
                if (std::fabs(e[size_t(mm)]) <= DBL_EPSILON * dd) break;
            }
            if (mm == l) break;
            if (++iter > 64) return false;
            double g = (d[size_t(l) + 1] - d[size_t(l)]) / (2.0 * e[size_t(l)]);
            double r = pyth(g, 1.0);
            g = d[size_t(mm)] - d[size_t(l)] + e[size_t(l)] / (g + std::copysign(r, g));
            double s = 1.0, c = 1.0, p = 0.0;
            bool early = false;
            for (int i = mm - 1; i >= l; --i) {
                const double f = s * e[size_t(i)], b = c * e[size_t(i)];
                r = pyth(f, g);
                e[size_t(i) + 1] = r;
                if (r == 0.0) {  // underflow: split here and restart the sweep
                    d[size_t(i) + 1] -= p;
                    e[size_t(mm)] = 0.0;
                    early = true;
                    break;
                }
                s = f / r;
                c = g / r;
                g = d[size_t(i) + 1] - p;
                r = (d[size_t(i)] - g) * s + 2.0 * c * b;
                p = s * r;
                d[size_t(i) + 1] = g + p;
                g = c * r - b;
                const double t = zl[size_t(i) + 1];
                zl[size_t(i) + 1] = s * zl[size_t(i)] + c * t;
                zl[size_t(i)] = c * zl[size_t(i)] - s * t;
                if (Z) {
                    double* zi = Z + size_t(i) * m;
                    double* zj = Z + size_t(i + 1) * m;
                    for (int k = 0; k < m; ++k) {
                        const double tk = zj[k];
                        zj[k] = s * zi[k] + c * tk;
                        zi[k] = c * zi[k] - s * tk;
                    }
                }
            }
            if (early) continue;
            d[size_t(l)] -= p;
            e[size_t(l)] = g;
            e[size_t(mm)] = 0.0;
        }
    }
    std::vector<int> idx(static_cast<size_t>(m));
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return d[size_t(a)] < d[size_t(b)]; });
    for (int j = 0; j < m; ++j) {
        evals[j] = d[size_t(idx[size_t(j)])];
        if (zlast) zlast[j] = zl[size_t(idx[size_t(j)])];
    }
    if (Z) {
        std::vector<double> tmp(Z, Z + size_t(m) * m);
        for (int j = 0; j < m; ++j)
            std::copy(tmp.begin() + size_t(idx[size_t(j)]) * m, tmp.begin() + size_t(idx[size_t(j)] + 1) * m,
                      Z + size_t(j) * m);
    }
    return true;
}

// Sturm count: the eigenvalues of T below x (LDL^T pivots of T - xI; a zero
// pivot is nudged, the standard guard of dstebz)
static int sturm_below(int m, const double* d, const double* e2, double x, double pivmin) {
    int c = 0;
    double q = d[0] - x;
    if (std::fabs(q) < pivmin) q = -pivmin;
    if (q < 0.0) ++c;
    for (int i = 1; i < m; ++i) {
        q = d[i] - x - e2[i - 1] / q;
        if (std::fabs(q) < pivmin) q = -pivmin;
        if (q < 0.0) ++c;
    }
    return c;
}

bool tridiag_smallest(int m, const double* d, const double* e, int k, double* evals, double* zlast) {
    if (m <= 0 || k <= 0 || k > m) return false;
    if (k > 1) {
        // Inverse iteration for two close eigenvalues, without orthogonalising
        // the vectors against each other (LAPACK dstein does), can converge to
        // the same vector and report the wrong last component.
        // Several values are only asked for with nev = 2 (no deflation): the
        // full QL gives them all, exactly.
        std::vector<double> ev(static_cast<size_t>(m)), zl(static_cast<size_t>(m));
        if (!tridiag_eig(m, d, e, ev.data(), zl.data(), nullptr)) return false;
        for (int j = 0; j < k; ++j) {
            evals[j] = ev[size_t(j)];
            zlast[j] = zl[size_t(j)];
        }
        return true;
    }
    std::vector<double> e2(size_t(std::max(m - 1, 1)), 0.0);
    double lo = d[0], hi = d[0], tnorm = 0.0, emax2 = 0.0;
    for (int i = 0; i < m; ++i) {
        const double r = (i > 0 ? std::fabs(e[i - 1]) : 0.0) + (i + 1 < m ? std::fabs(e[i]) : 0.0);
        lo = std::min(lo, d[i] - r);
        hi = std::max(hi, d[i] + r);
        tnorm = std::max(tnorm, std::fabs(d[i]) + r);
        if (i + 1 < m) {
            e2[size_t(i)] = e[i] * e[i];
            emax2 = std::max(emax2, e2[size_t(i)]);
        }
    }
    const double pivmin = std::max(DBL_MIN, DBL_MIN * emax2);
    std::vector<double> a(static_cast<size_t>(m)), b(static_cast<size_t>(m)), x(static_cast<size_t>(m)),
        y(static_cast<size_t>(m));
    for (int j = 0; j < k; ++j) {
        // the (j+1)-th smallest: count(x) > j  <=>  x above it
        double l = lo, h = hi;
        // (to 1e-12 relative: the convergence test reads lambda through
        // tol * max(eps^(2/3), |lambda|) only, and inverse iteration from it
        // converges at the rate 1e-12 |lambda| / gap)
        for (int it = 0; it < 200 && h - l > 1e-12 * std::max(std::fabs(l), std::fabs(h)) + pivmin; ++it) {
            const double mid = 0.5 * (l + h);
            if (mid <= l || mid >= h) break;
            if (sturm_below(m, d, e2.data(), mid, pivmin) > j) h = mid;
            else l = mid;
        }
        const double lam = 0.5 * (l + h);
        evals[j] = lam;
        // inverse iteration on T - (lam - delta) I, three solves by Gaussian
        // elimination with partial pivoting of the tridiagonal (LAPACK dgtsv's
        // scheme; a zero pivot is replaced by eps ||T||)
        const double shift = lam - 1e-12 * std::fabs(lam) - DBL_EPSILON * tnorm, tiny = DBL_EPSILON * tnorm + DBL_MIN;
        for (int i = 0; i < m; ++i) x[size_t(i)] = 1.0;
        for (int pass = 0; pass < 3; ++pass) {
            for (int i = 0; i < m; ++i) {
                a[size_t(i)] = d[i] - shift;                  // D
                b[size_t(i)] = i + 1 < m ? e[i] : 0.0;       // DL (sub), then DU2 after an interchange
                y[size_t(i)] = i + 1 < m ? e[i] : 0.0;       // DU (super)
            }
            for (int i = 0; i + 1 < m; ++i) {
                if (std::fabs(a[size_t(i)]) >= std::fabs(b[size_t(i)])) {
                    if (a[size_t(i)] == 0.0) a[size_t(i)] = tiny;
                    const double f = b[size_t(i)] / a[size_t(i)];
                    a[size_t(i) + 1] -= f * y[size_t(i)];
                    x[size_t(i) + 1] -= f * x[size_t(i)];
                    b[size_t(i)] = 0.0;
                } else {  // interchange rows i and i+1
                    const double f = a[size_t(i)] / b[size_t(i)];
                    a[size_t(i)] = b[size_t(i)];
                    const double t = a[size_t(i) + 1];
                    a[size_t(i) + 1] = y[size_t(i)] - f * t;
                    if (i + 2 < m) {
                        b[size_t(i)] = y[size_t(i) + 1];
                        y[size_t(i) + 1] = -f * b[size_t(i)];
                    } else {
                        b[size_t(i)] = 0.0;
                    }
                    y[size_t(i)] = t;
                    const double r = x[size_t(i)];
                    x[size_t(i)] = x[size_t(i) + 1];
                    x[size_t(i) + 1] = r - f * x[size_t(i) + 1];
                }
            }
            if (a[size_t(m) - 1] == 0.0) a[size_t(m) - 1] = tiny;
            for (int i = m - 1; i >= 0; --i) {
                double v = x[size_t(i)];
                if (i + 1 < m) v -= y[size_t(i)] * x[size_t(i) + 1];
                if (i + 2 < m) v -= b[size_t(i)] * x[size_t(i) + 2];
                x[size_t(i)] = v / a[size_t(i)];
            }
            double nrm = 0.0;
            for (int i = 0; i < m; ++i) nrm += x[size_t(i)] * x[size_t(i)];
            nrm = std::sqrt(nrm);
            if (!(nrm > 0.0) || !std::isfinite(nrm)) return false;
            for (int i = 0; i < m; ++i) x[size_t(i)] /= nrm;
        }
        zlast[j] = x[size_t(m) - 1];
    }
    return true;
}

// One implicitly shifted symmetric QR step (bulge chase) with shift mu:
// T <- G^T T G, where G = G_0 ... G_{m-2} is the orthogonal factor of the QR
// decomposition of T - mu I (implicit-Q theorem); G's rotations are appended
// to rots in order (Q <- Q G_p each).  Equivalent to Spectra's explicit
// TridiagQR(H - mu I) followed by R Q + mu I.  The implicit-Q theorem needs an
// unreduced matrix, so negligible off-diagonals (|e_i| <= eps (|d_i| +
// |d_i+1|), zeroed as TridiagQR does) split T into blocks and the chase
// restarts at the top of every block — a chase that simply ran through a
// split would stop there and never shift the trailing block, which is the one
// that carries the residual row (Q(m-1, :)).
void tridiag_qr_shift(int m, double* d, double* e, double mu, std::vector<QRot>& rots) {
    if (m < 2) return;
    // band scratch: only |i-j| <= 2 is ever non-zero (the chase's bulge), so
    // row i keeps columns i-2 .. i+2 (5 entries; same operations, same order
    // as a dense matrix, without zero-filling m x m per shift)
    std::vector<double> A(size_t(m) * 5, 0.0);
    std::vector<char> split(size_t(m), 0);  // split[p]: a block starts at p
    auto at = [&](int i, int j) -> double& { return A[size_t(i) * 5 + size_t(j - i + 2)]; };
    for (int i = 0; i < m; ++i) at(i, i) = d[i];
    for (int i = 0; i + 1 < m; ++i) {
        const double ei = std::fabs(e[i]) <= DBL_EPSILON * (std::fabs(d[i]) + std::fabs(d[i + 1])) ? 0.0 : e[i];
        at(i + 1, i) = at(i, i + 1) = ei;
        split[size_t(i) + 1] = ei == 0.0;
    }
    split[0] = 1;
    double x = 0.0, z = 0.0;
    for (int p = 0; p + 1 < m; ++p) {
        const int q = p + 1;
        if (split[size_t(q)]) continue;  // 1x1 block or block end: nothing couples p and q
        if (split[size_t(p)]) {          // top of an unreduced block: first column of T - mu I
            x = at(p, p) - mu;
            z = at(q, p);
        } else {                          // chase the bulge
            x = at(p, p - 1);
            z = at(q, p - 1);
        }
        const double r = pyth(x, z);
        const double c = r == 0.0 ? 1.0 : x / r, s = r == 0.0 ? 0.0 : z / r;
        const int lo = std::max(0, p - 1), hi = std::min(m - 1, p + 2);
        for (int j = lo; j <= hi; ++j) {  // rows p, q  (G^T T)
            const double ap = at(p, j), aq = at(q, j);
            at(p, j) = c * ap + s * aq;
            at(q, j) = -s * ap + c * aq;
        }
        for (int i = lo; i <= hi; ++i) {  // cols p, q  (T G)
            const double ap = at(i, p), aq = at(i, q);
            at(i, p) = c * ap + s * aq;
            at(i, q) = -s * ap + c * aq;
        }
        if (!split[size_t(p)]) at(q, p - 1) = at(p - 1, q) = 0.0;  // bulge annihilated
        rots.push_back(QRot{p, c, s});
    }
    for (int i = 0; i < m; ++i) d[i] = at(i, i);
    for (int i = 0; i + 1 < m; ++i) e[i] = 0.5 * (at(i + 1, i) + at(i, i + 1));
}

// tridiag_qr_shift for mus[0], mus[1], ... in turn: the same d, e and
// rotations bit for bit, with the chases of two consecutive shifts
// interleaved.  Rotation p of a chase reads and writes only the band window
// [p-1, p+2], so once the first chase has done rotation p+3 its rows up to
// p+2 are final, which is all that rotation p of the second reads: the second
// runs three positions behind, its band rows filled from the first's final
// rows just before it needs them (row p+2 before rotation p, with the same
// split rule).  Two independent sqrt/divide chains per step: 137 -> 89 us for
// the headline's 80 shifts at ncv 100 on the GPU hosts' EPYC 9575F (one
// chain per step is latency-bound there; more chains per step, 3-8, measured
// slower, and this container's CPU showed no gain at all).
namespace {
inline double& band(double* A, int i, int j) { return A[size_t(i) * 5 + size_t(j - i + 2)]; }
void band_init(double* A, char* split, int m, const double* d, const double* e) {
    std::fill(A, A + size_t(m) * 5, 0.0);
    for (int i = 0; i < m; ++i) band(A, i, i) = d[i];
    for (int i = 0; i + 1 < m; ++i) {
        const double ei = std::fabs(e[i]) <= DBL_EPSILON * (std::fabs(d[i]) + std::fabs(d[i + 1])) ? 0.0 : e[i];
        band(A, i + 1, i) = band(A, i, i + 1) = ei;
        split[size_t(i) + 1] = ei == 0.0;
    }
    split[0] = 1;
}
// row i of band B from band A's final rows (tridiag_qr_shift's extraction and
// split rule, row by row)
void band_row_from(double* B, char* split, const double* A, int i) {
    double* b = B + size_t(i) * 5;
    const double di = A[size_t(i) * 5 + 2];
    b[2] = di;
    if (i == 0) {
        split[0] = 1;
        return;
    }
    const double dim1 = A[size_t(i - 1) * 5 + 2];
    const double eim1 = 0.5 * (A[size_t(i) * 5 + 1] + A[size_t(i - 1) * 5 + 3]);
    const double ei = std::fabs(eim1) <= DBL_EPSILON * (std::fabs(dim1) + std::fabs(di)) ? 0.0 : eim1;
    b[1] = ei;
    B[size_t(i - 1) * 5 + 3] = ei;
    split[i] = ei == 0.0;
}
// rotation p of the chase with shift mu (tridiag_qr_shift's loop body)
void band_rot(double* A, const char* split, int m, double mu, int p, std::vector<QRot>& rots) {
    const int q = p + 1;
    if (split[q]) return;
    double x, z;
    if (split[p]) {
        x = band(A, p, p) - mu;
        z = band(A, q, p);
    } else {
        x = band(A, p, p - 1);
        z = band(A, q, p - 1);
    }
    const double r = pyth(x, z);
    const double c = r == 0.0 ? 1.0 : x / r, s = r == 0.0 ? 0.0 : z / r;
    const int lo = std::max(0, p - 1), hi = std::min(m - 1, p + 2);
    for (int j = lo; j <= hi; ++j) {
        const double ap = band(A, p, j), aq = band(A, q, j);
        band(A, p, j) = c * ap + s * aq;
        band(A, q, j) = -s * ap + c * aq;
    }
    for (int i = lo; i <= hi; ++i) {
        const double ap = band(A, i, p), aq = band(A, i, q);
        band(A, i, p) = c * ap + s * aq;
        band(A, i, q) = -s * ap + c * aq;
    }
    if (!split[p]) band(A, q, p - 1) = band(A, p - 1, q) = 0.0;
    rots.push_back(QRot{p, c, s});
}
}  // namespace

void tridiag_qr_shifts(int m, double* d, double* e, const double* mus, int ns, std::vector<QRot>& rots) {
    if (m < 3) {  // (no room for the stagger: one chase at a time)
        for (int g = 0; g < ns; ++g) tridiag_qr_shift(m, d, e, mus[g], rots);
        return;
    }
    std::vector<double> A0(size_t(m) * 5), A1(size_t(m) * 5);
    std::vector<char> s0(static_cast<size_t>(m)), s1(static_cast<size_t>(m));
    std::vector<QRot> r1;
    r1.reserve(size_t(m));
    const int P = m - 1;
    int g = 0;
    for (; g + 1 < ns; g += 2) {
        band_init(A0.data(), s0.data(), m, d, e);
        std::fill(A1.begin(), A1.end(), 0.0);
        r1.clear();
        for (int t = 0; t < P + 3; ++t) {
            if (t < P) band_rot(A0.data(), s0.data(), m, mus[g], t, rots);
            const int p = t - 3;
            if (p >= 0) {
                if (p == 0) {
                    band_row_from(A1.data(), s1.data(), A0.data(), 0);
                    band_row_from(A1.data(), s1.data(), A0.data(), 1);
                }
                if (p + 2 < m) band_row_from(A1.data(), s1.data(), A0.data(), p + 2);
                band_rot(A1.data(), s1.data(), m, mus[g + 1], p, r1);
            }
        }
        rots.insert(rots.end(), r1.begin(), r1.end());
        for (int i = 0; i < m; ++i) d[i] = A1[size_t(i) * 5 + 2];
        for (int i = 0; i + 1 < m; ++i) e[i] = 0.5 * (A1[size_t(i + 1) * 5 + 1] + A1[size_t(i) * 5 + 3]);
    }
    for (; g < ns; ++g) tridiag_qr_shift(m, d, e, mus[g], rots);
}

// Columns [0, kk) of Q = G_1 G_2 ... G_R (the recorded rotations, in order)
// into Qcm (column-major m x kk).  The restart needs only those kk columns,
// so Q E (E = I(:, 0:kk)) is formed right to left, G_1 (G_2 (... (G_R E))):
// each rotation then mixes two ROWS of an m x kk matrix X (kk contiguous
// doubles each) instead of two length-m columns of the full m x m Q, and X
// is zero below a row `hi` that a rotation (p, p+1) can raise only to p+1 —
// one row per shift sweep walked backwards — so rotations below it are
// skipped.  At ncv 100 with 20 kept: ~100k row-element updates instead of
// ~600k for the forward accumulation of all of Q.
void accumulate_q(int m, const std::vector<QRot>& rots, int kk, double* Qcm, std::vector<double>& X) {
    X.assign(size_t(m) * size_t(kk), 0.0);
    for (int i = 0; i < kk; ++i) X[size_t(i) * kk + i] = 1.0;
    int hi = kk - 1;  // rows > hi of X are zero
    for (size_t r = rots.size(); r-- > 0;) {
        const QRot g = rots[r];
        const int p = g.p;
        if (p > hi) continue;
        if (p + 1 > hi) hi = p + 1;
        // G_p X on rows p, p+1: G_p(p,p) = c, G_p(p,q) = -s, G_p(q,p) = s, G_p(q,q) = c
        double* xp = X.data() + size_t(p) * kk;
        double* xq = xp + kk;
        for (int j = 0; j < kk; ++j) {
            const double a = xp[j], b = xq[j];
            xp[j] = g.c * a - g.s * b;
            xq[j] = g.s * a + g.c * b;
        }
    }
    for (int j = 0; j < kk; ++j)
        for (int i = 0; i < m; ++i) Qcm[size_t(j) * m + i] = X[size_t(i) * kk + j];
}

}  // namespace ek
