#include "ek_internal.hpp"
#include <cfloat>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <cmath>
static inline double pyth(double a, double b) { return std::sqrt(a * a + b * b); }
struct Chase {  // one shift's bulge chase on its own band (same ops as tridiag_qr_shift)
    double* A; char* split; int m; double mu; int p;  // next rotation position
    std::vector<ek::QRot>* out;
};
static inline double& at(double* A, int i, int j) { return A[size_t(i) * 5 + size_t(j - i + 2)]; }
static inline void init_band(double* A, char* split, int m, const double* d, const double* e) {
    std::memset(A, 0, sizeof(double) * size_t(m) * 5);
    for (int i = 0; i < m; ++i) at(A, i, i) = d[i];
    for (int i = 0; i + 1 < m; ++i) {
        const double ei = std::fabs(e[i]) <= DBL_EPSILON * (std::fabs(d[i]) + std::fabs(d[i + 1])) ? 0.0 : e[i];
        at(A, i + 1, i) = at(A, i, i + 1) = ei;
        split[i + 1] = ei == 0.0;
    }
    split[0] = 1;
}
static inline void rot(double* A, const char* split, int m, double mu, int p, std::vector<ek::QRot>& rots) {
    const int q = p + 1;
    if (split[q]) return;
    double x, z;
    if (split[p]) { x = at(A, p, p) - mu; z = at(A, q, p); }
    else { x = at(A, p, p - 1); z = at(A, q, p - 1); }
    const double r = pyth(x, z);
    const double c = r == 0.0 ? 1.0 : x / r, s = r == 0.0 ? 0.0 : z / r;
    const int lo = std::max(0, p - 1), hi = std::min(m - 1, p + 2);
    for (int j = lo; j <= hi; ++j) { const double ap = at(A, p, j), aq = at(A, q, j); at(A, p, j) = c * ap + s * aq; at(A, q, j) = -s * ap + c * aq; }
    for (int i = lo; i <= hi; ++i) { const double ap = at(A, i, p), aq = at(A, i, q); at(A, i, p) = c * ap + s * aq; at(A, i, q) = -s * ap + c * aq; }
    if (!split[p]) at(A, q, p - 1) = at(A, p - 1, q) = 0.0;
    rots.push_back(ek::QRot{p, c, s});
}
// extract d,e of band A into (d,e)
static inline void extract(const double* A, int m, double* d, double* e) {
    for (int i = 0; i < m; ++i) d[i] = A[size_t(i) * 5 + 2];
    for (int i = 0; i + 1 < m; ++i) e[i] = 0.5 * (A[size_t(i + 1) * 5 + 1] + A[size_t(i) * 5 + 3]);
}
// pairs of shifts: chase g fully materialised band from (d,e); chase g+1 needs rows from g's final band:
// row i of band g+1 depends on d_i, e_{i-1}, d_{i-1} final in g -> after g's rotation i+1 (p+3 rule).
void qr_pair(int m, double* d, double* e, const double* mus, int ns, std::vector<ek::QRot>& rots) {
    std::vector<double> A0(size_t(m) * 5), A1(size_t(m) * 5);
    std::vector<char> s0(m), s1(m);
    std::vector<ek::QRot> r0, r1; r0.reserve(m); r1.reserve(m);
    int g = 0;
    for (; g + 1 < ns; g += 2) {
        init_band(A0.data(), s0.data(), m, d, e);
        std::memset(A1.data(), 0, sizeof(double) * size_t(m) * 5);
        r0.clear(); r1.clear();
        // lazily init rows of A1 from A0's final rows
        auto init1 = [&](int i) {
            double* a = A1.data() + size_t(i) * 5;
            const double* pa = A0.data();
            const double di = pa[size_t(i) * 5 + 2];
            a[2] = di;
            if (i > 0) {
                const double dim1 = pa[size_t(i - 1) * 5 + 2];
                const double eim1 = 0.5 * (pa[size_t(i) * 5 + 1] + pa[size_t(i - 1) * 5 + 3]);
                const double ei = std::fabs(eim1) <= DBL_EPSILON * (std::fabs(dim1) + std::fabs(di)) ? 0.0 : eim1;
                a[1] = ei; A1[size_t(i - 1) * 5 + 3] = ei; s1[i] = ei == 0.0;
            } else s1[0] = 1;
        };
        const int P = m - 1;
        for (int t = 0; t < P + 3; ++t) {
            if (t < P) rot(A0.data(), s0.data(), m, mus[g], t, r0);
            const int p = t - 3;
            if (p >= 0) {
                if (p == 0) { init1(0); init1(1); }
                if (p + 2 < m) init1(p + 2);
                rot(A1.data(), s1.data(), m, mus[g + 1], p, r1);
            }
        }
        // (rows of A1 beyond P+2: all inited by p+2 < m condition at p up to m-3)
        rots.insert(rots.end(), r0.begin(), r0.end());
        rots.insert(rots.end(), r1.begin(), r1.end());
        extract(A1.data(), m, d, e);
    }
    for (; g < ns; ++g) ek::tridiag_qr_shift(m, d, e, mus[g], rots);
}
// groups of K shifts: chase k of the group runs rotation t - 3k at step t; its band rows are
// filled lazily from chase k-1's final rows (row p+2 before rotation p): identical operations.
template <int K>
void qr_group(int m, double* d, double* e, const double* mus, int ns, std::vector<ek::QRot>& rots) {
    std::vector<double> A(static_cast<size_t>(K) * static_cast<size_t>(m) * 5);
    std::vector<char> sp(static_cast<size_t>(K) * static_cast<size_t>(m));
    std::vector<ek::QRot> rr[K];
    for (int k = 0; k < K; ++k) rr[k].reserve(m);
    int g = 0;
    const int P = m - 1;
    for (; g + K <= ns; g += K) {
        double* A0 = A.data();
        init_band(A0, sp.data(), m, d, e);
        for (int k = 1; k < K; ++k) std::memset(A.data() + size_t(k) * m * 5, 0, sizeof(double) * size_t(m) * 5);
        for (int k = 0; k < K; ++k) rr[k].clear();
        auto initk = [&](int k, int i) {
            double* Ak = A.data() + size_t(k) * m * 5;
            const double* pa = A.data() + size_t(k - 1) * m * 5;
            char* sk = sp.data() + size_t(k) * m;
            double* a = Ak + size_t(i) * 5;
            const double di = pa[size_t(i) * 5 + 2];
            a[2] = di;
            if (i > 0) {
                const double dim1 = pa[size_t(i - 1) * 5 + 2];
                const double eim1 = 0.5 * (pa[size_t(i) * 5 + 1] + pa[size_t(i - 1) * 5 + 3]);
                const double ei = std::fabs(eim1) <= DBL_EPSILON * (std::fabs(dim1) + std::fabs(di)) ? 0.0 : eim1;
                a[1] = ei; Ak[size_t(i - 1) * 5 + 3] = ei; sk[i] = ei == 0.0;
            } else sk[0] = 1;
        };
        for (int t = 0; t < P + 3 * (K - 1); ++t) {
            for (int k = 0; k < K; ++k) {
                const int p = t - 3 * k;
                if (p < 0 || p >= P) continue;
                if (k > 0) {
                    if (p == 0) { initk(k, 0); initk(k, 1); }
                    if (p + 2 < m) initk(k, p + 2);
                }
                rot(A.data() + size_t(k) * m * 5, sp.data() + size_t(k) * m, m, mus[g + k], p, rr[k]);
            }
        }
        for (int k = 0; k < K; ++k) rots.insert(rots.end(), rr[k].begin(), rr[k].end());
        extract(A.data() + size_t(K - 1) * m * 5, m, d, e);
    }
    for (; g < ns; ++g) ek::tridiag_qr_shift(m, d, e, mus[g], rots);
}
int main(){
  std::mt19937_64 gen(7); std::uniform_real_distribution<double> U(0,1);
  int bad=0;
  for(int trial=0;trial<400;trial++){
    int m = trial<300 ? 3+int(U(gen)*126) : 100;
    std::vector<double> d(m), e(m), th(m), zl(m);
    for(int i=0;i<m;i++){d[i]=4+3*std::sin(i*0.37+trial)+U(gen); e[i]=0.5+2*U(gen);
      double r=U(gen); if(r<0.05) e[i]=0.0; else if(r<0.1) e[i]=1e-18; else if (r<0.12) e[i]*=1e-9;}
    if(!ek::tridiag_eig(m,d.data(),e.data(),th.data(),zl.data(),nullptr)) continue;
    int knew = std::max(1, int(U(gen)*m*0.5));
    std::vector<double> d1(d),e1(e),d2(d),e2(e);
    std::vector<ek::QRot> r1,r2;
    for(int i=knew;i<m;i++) ek::tridiag_qr_shift(m,d1.data(),e1.data(),th[i],r1);
    if(trial%3==0) qr_pair(m,d2.data(),e2.data(),th.data()+knew,m-knew,r2); else if(trial%3==1) qr_group<3>(m,d2.data(),e2.data(),th.data()+knew,m-knew,r2); else qr_group<4>(m,d2.data(),e2.data(),th.data()+knew,m-knew,r2);
    bool ok = memcmp(d1.data(),d2.data(),8*m)==0 && memcmp(e1.data(),e2.data(),8*(m-1))==0 && r1.size()==r2.size();
    for(size_t k=0;ok && k<r1.size();k++) ok = r1[k].p==r2[k].p && memcmp(&r1[k].c,&r2[k].c,8)==0 && memcmp(&r1[k].s,&r2[k].s,8)==0;
    if(!ok){bad++; if(bad<5) printf("mismatch trial %d m %d knew %d rots %zu %zu\n",trial,m,knew,r1.size(),r2.size());}
  }
  printf("bad %d\n",bad);
  const int m=100; std::vector<double> d(m), e(m), th(m), zl(m);
  for(int i=0;i<m;i++){d[i]=4+3*std::sin(i*0.37)+U(gen); e[i]=0.5+2*U(gen);}
  ek::tridiag_eig(m,d.data(),e.data(),th.data(),zl.data(),nullptr);
  int R=200; std::vector<ek::QRot> rots; rots.reserve(20000);
  double tt[6]={0};
  for(int r=0;r<R;r++){
    for(int v=0;v<5;v++){
      std::vector<double> dd(d),ee(e); rots.clear();
      auto t0=std::chrono::steady_clock::now();
      if(v==0) for(int i=20;i<m;i++) ek::tridiag_qr_shift(m,dd.data(),ee.data(),th[i],rots);
      else if(v==1) qr_group<2>(m,dd.data(),ee.data(),th.data()+20,m-20,rots);
      else if(v==2) qr_group<3>(m,dd.data(),ee.data(),th.data()+20,m-20,rots);
      else if(v==3) qr_group<4>(m,dd.data(),ee.data(),th.data()+20,m-20,rots);
      else qr_group<8>(m,dd.data(),ee.data(),th.data()+20,m-20,rots);
      auto t1=std::chrono::steady_clock::now();
      tt[v]+=std::chrono::duration<double,std::micro>(t1-t0).count();
    }
  }
  printf("serial %.1f  K2 %.1f  K3 %.1f  K4 %.1f  K8 %.1f us\n",tt[0]/R,tt[1]/R,tt[2]/R,tt[3]/R,tt[4]/R);
}
