// dmt_filter.h — the exact discrete backward filter of a linear auxiliary law (the guiding
// term H, F, c of GuidedProposals' recompute_guiding_term!), shared
// by the host entry point dmt_guiding_linear and the device kernel k_backward_filter so that
// both produce the same bits.  Plain IEEE operations in a fixed order (no fma contraction:
// -ffp-contract=off on both sides); the one transcendental, log|det|, uses the build's own
// polynomial log (flt_log == rng_log of dmt_device.h).  Restated in oracle/dmt_oracle.c.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#ifndef DMT_HD
#define DMT_HD __host__ __device__ __forceinline__
#endif

namespace dmt {
namespace flt {

struct Mat {
  int n;
  double a[9];
  DMT_HD double& operator()(int i, int j) { return a[i * n + j]; }
  DMT_HD double operator()(int i, int j) const { return a[i * n + j]; }
};
DMT_HD Mat mzero(int n) { Mat m; m.n = n; for (int i = 0; i < 9; ++i) m.a[i] = 0.0; return m; }
DMT_HD Mat meye(int n) { Mat m = mzero(n); for (int i = 0; i < n; ++i) m(i, i) = 1.0; return m; }
DMT_HD Mat mmul(const Mat& A, const Mat& B) {
  Mat C = mzero(A.n);
  for (int i = 0; i < A.n; ++i)
    for (int j = 0; j < A.n; ++j) {
      double s = 0.0;
      for (int k = 0; k < A.n; ++k) s += A(i, k) * B(k, j);
      C(i, j) = s;
    }
  return C;
}
DMT_HD Mat mT(const Mat& A) {
  Mat C = mzero(A.n);
  for (int i = 0; i < A.n; ++i) for (int j = 0; j < A.n; ++j) C(i, j) = A(j, i);
  return C;
}
DMT_HD Mat madd(const Mat& A, const Mat& B) {
  Mat C = A;
  for (int i = 0; i < A.n * A.n; ++i) C.a[i] += B.a[i];
  return C;
}
DMT_HD void mvec(const Mat& A, const double* x, double* y) {
  for (int i = 0; i < A.n; ++i) {
    double s = 0.0;
    for (int k = 0; k < A.n; ++k) s += A(i, k) * x[k];
    y[i] = s;
  }
}
DMT_HD double mnorm(const Mat& A) {
  double s = 0.0;
  for (int i = 0; i < A.n * A.n; ++i) s = fmax(s, fabs(A.a[i]));
  return s * A.n;
}

// log(u), u > 0 finite: the rng_log polynomial kernel (dmt_device.h), as host/device code
DMT_HD double flt_log(double u) {
  int e;
  double m = frexp(u, &e);
  const int lo = m < 0x1.6a09e667f3bcdp-1;
  m = lo ? m * 2.0 : m;
  e = lo ? e - 1 : e;
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s;
  double p = 0x1.642c8590b2164p-4;
  p = fma(p, z, 0x1.8618618618618p-4); p = fma(p, z, 0x1.af286bca1af28p-4);
  p = fma(p, z, 0x1.e1e1e1e1e1e1ep-4); p = fma(p, z, 0x1.1111111111111p-3);
  p = fma(p, z, 0x1.3b13b13b13b14p-3); p = fma(p, z, 0x1.745d1745d1746p-3);
  p = fma(p, z, 0x1.c71c71c71c71cp-3); p = fma(p, z, 0x1.2492492492492p-2);
  p = fma(p, z, 0x1.999999999999ap-2); p = fma(p, z, 0x1.5555555555555p-1);
  const double lm = fma(s, z * p, 2.0 * s);
  const double de = (double)e;
  return fma(de, 0x1.62e42p-1, fma(de, 0x1.fdf473de6af28p-22, lm));
}

// inverse and log|det| by Gauss–Jordan with partial pivoting; false if singular
DMT_HD bool minv(const Mat& A, Mat& Inv, double& logabsdet) {
  const int n = A.n;
  double w[3][6];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) { w[i][j] = A(i, j); w[i][n + j] = (i == j) ? 1.0 : 0.0; }
  logabsdet = 0.0;
  for (int c = 0; c < n; ++c) {
    int p = c;
    for (int i = c + 1; i < n; ++i) if (fabs(w[i][c]) > fabs(w[p][c])) p = i;
    if (w[p][c] == 0.0) return false;
    if (p != c)
      for (int j = 0; j < 2 * n; ++j) { const double tmp = w[p][j]; w[p][j] = w[c][j]; w[c][j] = tmp; }
    const double piv = w[c][c];
    logabsdet += flt_log(fabs(piv));
    for (int j = 0; j < 2 * n; ++j) w[c][j] /= piv;
    for (int i = 0; i < n; ++i)
      if (i != c) {
        const double f = w[i][c];
        if (f != 0.0) for (int j = 0; j < 2 * n; ++j) w[i][j] -= f * w[c][j];
      }
  }
  Inv = mzero(n);
  for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) Inv(i, j) = w[i][n + j];
  return true;
}

// Exact transition of dX = (BX + beta)dt + sigma dW over a step h:
// X_{t+h} = Phi X_t + mu + N(0, K).  Taylor series with scaling and squaring.
DMT_HD void transition(const Mat& B, const double* beta, const Mat& At, double h, Mat& Phi,
                       double* mu, Mat& K) {
  const int n = B.n;
  int sq = 0;
  double hs = h;
  const double nb = mnorm(B);
  while (nb * hs > 0.25 && sq < 40) { hs *= 0.5; ++sq; }
  Mat A = B;
  for (int i = 0; i < n * n; ++i) A.a[i] *= hs;
  Phi = meye(n);
  Mat term = meye(n);
  Mat S1 = meye(n);  // sum A^k/(k+1)!
  Mat Lk = At;       // L^k(At) hs^k / k!,  L(X) = BX + XB^T
  K = mzero(n);
  for (int i = 0; i < n * n; ++i) K.a[i] = hs * Lk.a[i];
  const Mat BT = mT(B);
  for (int k = 1; k <= 30; ++k) {
    term = mmul(term, A);
    for (int i = 0; i < n * n; ++i) term.a[i] /= k;
    Phi = madd(Phi, term);
    Mat t2 = term;
    for (int i = 0; i < n * n; ++i) t2.a[i] /= (k + 1);
    S1 = madd(S1, t2);
    Mat nl = madd(mmul(B, Lk), mmul(Lk, BT));
    for (int i = 0; i < n * n; ++i) nl.a[i] *= hs / k;
    Lk = nl;
    for (int i = 0; i < n * n; ++i) K.a[i] += hs * Lk.a[i] / (k + 1);
    if (mnorm(term) < 1e-18 && mnorm(Lk) * hs < 1e-18 * (1.0 + mnorm(K))) break;
  }
  double sb[3];
  mvec(S1, beta, sb);
  for (int i = 0; i < n; ++i) mu[i] = hs * sb[i];
  for (int s = 0; s < sq; ++s) {  // compose two half steps
    double m2[3];
    mvec(Phi, mu, m2);
    for (int i = 0; i < n; ++i) mu[i] = m2[i] + mu[i];
    K = madd(mmul(mmul(Phi, K), mT(Phi)), K);
    Phi = mmul(Phi, Phi);
  }
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) { const double v = 0.5 * (K(i, j) + K(j, i)); K(i, j) = v; K(j, i) = v; }
}

// One backward step of the filter: (H, F, c) at t_{i+1} -> at t_i over the step h.
// Returns false if I + HK is singular.
DMT_HD bool filter_step(const Mat& B, const double* beta, const Mat& A, double h, Mat& Hc,
                        double* Fc, double& cc) {
  const int d = B.n;
  Mat Phi, K;
  double mu[3];
  transition(B, beta, A, h, Phi, mu, K);
  // Gaussian integral over X_{t+h} ~ N(Phi x + mu, K) of exp(-c - x'Hx/2 + F'x)
  const Mat IHK = madd(meye(d), mmul(Hc, K));
  Mat S;
  double lad;
  if (!minv(IHK, S, lad)) return false;
  Mat Hh = mmul(S, Hc);
  for (int p = 0; p < d; ++p)
    for (int q = p + 1; q < d; ++q) { const double v = 0.5 * (Hh(p, q) + Hh(q, p)); Hh(p, q) = v; Hh(q, p) = v; }
  double Fh[3], KF[3];
  mvec(S, Fc, Fh);
  mvec(K, Fc, KF);
  double fkf = 0.0;
  for (int p = 0; p < d; ++p) fkf += Fh[p] * KF[p];
  const double ch = cc + 0.5 * lad - 0.5 * fkf;
  double Hmu[3];
  mvec(Hh, mu, Hmu);
  double g[3];
  for (int p = 0; p < d; ++p) g[p] = Fh[p] - Hmu[p];
  const Mat PhT = mT(Phi);
  double Fn[3];
  mvec(PhT, g, Fn);
  Mat Hn = mmul(mmul(PhT, Hh), Phi);
  for (int p = 0; p < d; ++p)
    for (int q = p + 1; q < d; ++q) { const double v = 0.5 * (Hn(p, q) + Hn(q, p)); Hn(p, q) = v; Hn(q, p) = v; }
  double fmu = 0.0, muHmu = 0.0;
  for (int p = 0; p < d; ++p) { fmu += Fh[p] * mu[p]; muHmu += mu[p] * Hmu[p]; }
  cc = ch - fmu + 0.5 * muHmu;
  Hc = Hn;
  for (int p = 0; p < d; ++p) Fc[p] = Fn[p];
  return true;
}

DMT_HD int packed_ix(int d, int a, int b) {
  if (a > b) { const int t = a; a = b; b = t; }
  return a * d - (a * (a - 1)) / 2 + (b - a);
}

}  // namespace flt
}  // namespace dmt
