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

// Dimension N is a compile-time constant (1, 2 or 3): fixed-size arrays, fully unrolled
// loops — registers, never scratch, on the device.
template <int N>
struct Mat {
  static constexpr int n = N;
  double a[N * N];
  DMT_HD double& operator()(int i, int j) { return a[i * N + j]; }
  DMT_HD double operator()(int i, int j) const { return a[i * N + j]; }
};
template <int N>
DMT_HD Mat<N> mzero() {
  Mat<N> m;
#pragma unroll
  for (int i = 0; i < N * N; ++i) m.a[i] = 0.0;
  return m;
}
template <int N>
DMT_HD Mat<N> meye() {
  Mat<N> m = mzero<N>();
#pragma unroll
  for (int i = 0; i < N; ++i) m(i, i) = 1.0;
  return m;
}
template <int N>
DMT_HD Mat<N> mmul(const Mat<N>& A, const Mat<N>& B) {
  Mat<N> C;
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < N; ++k) s += A(i, k) * B(k, j);
      C(i, j) = s;
    }
  return C;
}
template <int N>
DMT_HD Mat<N> mT(const Mat<N>& A) {
  Mat<N> C;
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) C(i, j) = A(j, i);
  return C;
}
template <int N>
DMT_HD Mat<N> madd(const Mat<N>& A, const Mat<N>& B) {
  Mat<N> C = A;
#pragma unroll
  for (int i = 0; i < N * N; ++i) C.a[i] += B.a[i];
  return C;
}
template <int N>
DMT_HD void mvec(const Mat<N>& A, const double* x, double* y) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < N; ++k) s += A(i, k) * x[k];
    y[i] = s;
  }
}
template <int N>
DMT_HD double mnorm(const Mat<N>& A) {
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < N * N; ++i) s = fmax(s, fabs(A.a[i]));
  return s * N;
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

// inverse and log|det| by Gauss–Jordan with partial pivoting; false if singular.  Row swaps
// are done with selects over all rows (no dynamic register indexing).  The pivot row is scaled
// by the correctly rounded reciprocal of the pivot, and log|det| is one log of the product of
// the |pivots| (guiding term).
template <int N>
DMT_HD bool minv(const Mat<N>& A, Mat<N>& Inv, double& logabsdet) {
  double w[N][2 * N];
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) { w[i][j] = A(i, j); w[i][N + j] = (i == j) ? 1.0 : 0.0; }
  double detabs = 1.0;  // |det| as the product of the |pivots| in order; one log at the end
#pragma unroll
  for (int c = 0; c < N; ++c) {
    int p = c;
    double best = fabs(w[c][c]);
#pragma unroll
    for (int i = c + 1; i < N; ++i) {
      const double v = fabs(w[i][c]);
      if (v > best) { best = v; p = i; }
    }
    double prow[2 * N];
#pragma unroll
    for (int j = 0; j < 2 * N; ++j) {
      double v = w[c][j];
#pragma unroll
      for (int i = c + 1; i < N; ++i) v = (p == i) ? w[i][j] : v;
      prow[j] = v;
    }
    if (prow[c] == 0.0) return false;
#pragma unroll
    for (int i = c + 1; i < N; ++i)  // the swapped-out row takes pivot row c's place
#pragma unroll
      for (int j = 0; j < 2 * N; ++j) w[i][j] = (p == i) ? w[c][j] : w[i][j];
#pragma unroll
    for (int j = 0; j < 2 * N; ++j) w[c][j] = prow[j];
    const double piv = w[c][c];
    detabs *= fabs(piv);
    const double rp = 1.0 / piv;  // one correctly rounded division per pivot row
#pragma unroll
    for (int j = 0; j < 2 * N; ++j) w[c][j] *= rp;
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (i != c) {
        const double f = w[i][c];
        if (f != 0.0) {
#pragma unroll
          for (int j = 0; j < 2 * N; ++j) w[i][j] -= f * w[c][j];
        }
      }
  }
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) Inv(i, j) = w[i][N + j];
  logabsdet = flt_log(detabs);
  return true;
}

// Exact transition of dX = (BX + beta)dt + sigma dW over a step h:
// X_{t+h} = Phi X_t + mu + N(0, K).  Taylor series with scaling and squaring; the series
// multiplies by the correctly rounded reciprocals 1/k (no per-element divisions).
template <int N>
DMT_HD void transition(const Mat<N>& B, const double* beta, const Mat<N>& At, double h,
                       Mat<N>& Phi, double* mu, Mat<N>& K) {
  constexpr int n = N;
  int sq = 0;
  double hs = h;
  const double nb = mnorm(B);
  while (nb * hs > 0.25 && sq < 40) { hs *= 0.5; ++sq; }
  Mat<N> A = B;
#pragma unroll
  for (int i = 0; i < n * n; ++i) A.a[i] *= hs;
  Phi = meye<N>();
  Mat<N> term = meye<N>();
  Mat<N> S1 = meye<N>();  // sum A^k/(k+1)!
  Mat<N> Lk = At;         // L^k(At) hs^k / k!,  L(X) = BX + XB^T
  K = mzero<N>();
#pragma unroll
  for (int i = 0; i < n * n; ++i) K.a[i] = hs * Lk.a[i];
  const Mat<N> BT = mT(B);
  double rk = 1.0;  // 1/k, correctly rounded; one division per term
  for (int k = 1; k <= 30; ++k) {
    const double rk1 = 1.0 / (double)(k + 1);
    term = mmul(term, A);
#pragma unroll
    for (int i = 0; i < n * n; ++i) term.a[i] *= rk;
    Phi = madd(Phi, term);
    Mat<N> t2 = term;
#pragma unroll
    for (int i = 0; i < n * n; ++i) t2.a[i] *= rk1;
    S1 = madd(S1, t2);
    Mat<N> nl = madd(mmul(B, Lk), mmul(Lk, BT));
    const double c0 = hs * rk, c1 = hs * rk1;
#pragma unroll
    for (int i = 0; i < n * n; ++i) nl.a[i] *= c0;
    Lk = nl;
#pragma unroll
    for (int i = 0; i < n * n; ++i) K.a[i] += Lk.a[i] * c1;
    if (mnorm(term) < 1e-18 && mnorm(Lk) * hs < 1e-18 * (1.0 + mnorm(K))) break;
    rk = rk1;
  }
  double sb[N];
  mvec(S1, beta, sb);
#pragma unroll
  for (int i = 0; i < n; ++i) mu[i] = hs * sb[i];
  for (int s = 0; s < sq; ++s) {  // compose two half steps
    double m2[N];
    mvec(Phi, mu, m2);
#pragma unroll
    for (int i = 0; i < n; ++i) mu[i] = m2[i] + mu[i];
    K = madd(mmul(mmul(Phi, K), mT(Phi)), K);
    Phi = mmul(Phi, Phi);
  }
#pragma unroll
  for (int i = 0; i < n; ++i)
#pragma unroll
    for (int j = i + 1; j < n; ++j) { const double v = 0.5 * (K(i, j) + K(j, i)); K(i, j) = v; K(j, i) = v; }
}

// Transition (Phi, mu, K) of the auxiliary law over one step or a run of steps.
template <int N>
struct Trans {
  Mat<N> Phi;
  double mu[N];
  Mat<N> K;
};

template <int N>
DMT_HD Trans<N> step_trans(const Mat<N>& B, const double* beta, const Mat<N>& A, double h) {
  Trans<N> r;
  transition(B, beta, A, h, r.Phi, r.mu, r.K);
  return r;
}

// The transition over `f` then `s`: (Phi_s Phi_f, Phi_s mu_f + mu_s, Phi_s K_f Phi_s' + K_s).
template <int N>
DMT_HD Trans<N> compose(const Trans<N>& f, const Trans<N>& s) {
  constexpr int n = N;
  Trans<N> r;
  r.Phi = mmul(s.Phi, f.Phi);
  double m[N];
  mvec(s.Phi, f.mu, m);
#pragma unroll
  for (int i = 0; i < n; ++i) r.mu[i] = m[i] + s.mu[i];
  r.K = madd(mmul(mmul(s.Phi, f.K), mT(s.Phi)), s.K);
#pragma unroll
  for (int i = 0; i < n; ++i)
#pragma unroll
    for (int j = i + 1; j < n; ++j) { const double v = 0.5 * (r.K(i, j) + r.K(j, i)); r.K(i, j) = v; r.K(j, i) = v; }
  return r;
}

// The guiding term (H, F, c) at the start of a transition q from the one at its end:
// the Gaussian integral over X_end ~ N(Phi x + mu, K) of exp(-c - x'Hx/2 + F'x).
// Returns false if I + HK is singular.
template <int N>
DMT_HD bool filter_combine(const Trans<N>& q, Mat<N>& Hc, double* Fc, double& cc) {
  constexpr int d = N;
  const Mat<N>& Phi = q.Phi;
  const Mat<N>& K = q.K;
  const double* mu = q.mu;
  const Mat<N> IHK = madd(meye<N>(), mmul(Hc, K));
  Mat<N> S;
  double lad;
  if (!minv(IHK, S, lad)) return false;
  Mat<N> Hh = mmul(S, Hc);
#pragma unroll
  for (int p = 0; p < d; ++p)
#pragma unroll
    for (int r = p + 1; r < d; ++r) { const double v = 0.5 * (Hh(p, r) + Hh(r, p)); Hh(p, r) = v; Hh(r, p) = v; }
  double Fh[N], KF[N];
  mvec(S, Fc, Fh);
  mvec(K, Fc, KF);
  double fkf = 0.0;
#pragma unroll
  for (int p = 0; p < d; ++p) fkf += Fh[p] * KF[p];
  const double ch = cc + 0.5 * lad - 0.5 * fkf;
  double Hmu[N];
  mvec(Hh, mu, Hmu);
  double g[N];
#pragma unroll
  for (int p = 0; p < d; ++p) g[p] = Fh[p] - Hmu[p];
  const Mat<N> PhT = mT(Phi);
  double Fn[N];
  mvec(PhT, g, Fn);
  Mat<N> Hn = mmul(mmul(PhT, Hh), Phi);
#pragma unroll
  for (int p = 0; p < d; ++p)
#pragma unroll
    for (int r = p + 1; r < d; ++r) { const double v = 0.5 * (Hn(p, r) + Hn(r, p)); Hn(p, r) = v; Hn(r, p) = v; }
  double fmu = 0.0, muHmu = 0.0;
#pragma unroll
  for (int p = 0; p < d; ++p) { fmu += Fh[p] * mu[p]; muHmu += mu[p] * Hmu[p]; }
  cc = ch - fmu + 0.5 * muHmu;
  Hc = Hn;
#pragma unroll
  for (int p = 0; p < d; ++p) Fc[p] = Fn[p];
  return true;
}

// The canonical chunked filter of one segment (guiding term).  The steps are cut into chunks
// of kFiltChunk counted from the segment end; inside a chunk, every step's transition is
// composed with the rest of the chunk by an inclusive Kogge–Stone suffix scan (stage k: step l
// takes compose(Q_l, Q_{l+k}) when l + k < cnt, from the previous stage's values), and every
// point of the chunk gets its (H, F, c) by one filter_combine from the chunk end's guiding
// term; the chunk's first point is the next chunk's end.  The device runs a chunk on one wave
// (k_filter_scan / k_filter_chain); this is the serial host statement of the same arithmetic.
constexpr int kFiltChunk = 64;

// Coef(i, B, beta, A): the auxiliary law of step i — drift B, beta and, where ã is
// time-dependent, A (in: the segment's ã) — constant, or a time-dependent law's trapezoidal
// average over [t_i, t_i+1] (second order).
template <int N, class TimeAt, class Coef, class Store>
inline bool filter_segment(Coef coef, const Mat<N>& A, int npts, TimeAt tat, Mat<N>& Hc,
                           double* Fc, double& cc, Store store) {
  store(npts - 1, Hc, Fc, cc);
  Trans<N> Q[kFiltChunk], Qn[kFiltChunk];
  for (int hi = npts - 1; hi > 0; hi -= kFiltChunk) {
    const int lo = hi > kFiltChunk ? hi - kFiltChunk : 0, cnt = hi - lo;
    for (int l = 0; l < cnt; ++l) {
      Mat<N> B, As = A;
      double beta[N];
      coef(lo + l, B, beta, As);
      Q[l] = step_trans(B, beta, As, tat(lo + l + 1) - tat(lo + l));
    }
    for (int k = 1; k < kFiltChunk; k *= 2) {
      for (int l = 0; l < cnt; ++l) Qn[l] = (l + k < cnt) ? compose(Q[l], Q[l + k]) : Q[l];
      for (int l = 0; l < cnt; ++l) Q[l] = Qn[l];
    }
    const Mat<N> H0 = Hc;
    double F0[N];
    for (int p = 0; p < N; ++p) F0[p] = Fc[p];
    const double c0 = cc;
    for (int l = cnt - 1; l >= 0; --l) {
      Mat<N> H = H0;
      double F[N];
      for (int p = 0; p < N; ++p) F[p] = F0[p];
      double c = c0;
      if (!filter_combine(Q[l], H, F, c)) return false;
      store(lo + l, H, F, c);
      if (l == 0) {
        Hc = H;
        for (int p = 0; p < N; ++p) Fc[p] = F[p];
        cc = c;
      }
    }
  }
  return true;
}

DMT_HD int packed_ix(int d, int a, int b) {
  if (a > b) { const int t = a; a = b; b = t; }
  return a * d - (a * (a - 1)) / 2 + (b - a);
}

}  // namespace flt
}  // namespace dmt
