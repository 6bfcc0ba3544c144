// dmt_device.h — device building blocks of the guided-bridge engine (gfx950).
//
// Every arithmetic routine here follows the CANONICAL ARITHMETIC written in
// DESIGN.md §3 operation by operation (explicit fma, -ffp-contract=off), so a
// path computed on the MI355X is bit-identical to the CPU restatement.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dmt.h"
#include "dmt_internal.h"

namespace dmt {

// packed upper-triangular index of a symmetric d×d matrix (non-recursive so that it folds to
// a constant inside unrolled loops: a runtime index into a register array spills to scratch)
__host__ __device__ constexpr int packed_idx(int d, int a, int b) {
  return (a < b ? a : b) * d - ((a < b ? a : b) * ((a < b ? a : b) - 1)) / 2 + ((a < b ? b : a) - (a < b ? a : b));
}

__device__ __forceinline__ double dfma(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float dfma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// Load through the constant address space: for data a kernel only reads (law records,
// structure arrays, selectors inside the block kernels) with a wave-uniform address this
// becomes a scalar load into SGPRs instead of a vector load into VGPRs.
template <class T>
__device__ __forceinline__ T ldc(const T* p) {
  return *(const __attribute__((address_space(4))) T*)(p);
}

// ---------------------------------------------------------------- models
// Drifts of the DiffusionDefinition models.
template <class T, int D_, int M_>
struct OU {
  static constexpr int D = D_, M = M_, NTH = 12;
  static constexpr bool kLinear = true;  // drift folded into the guiding coefficients
  static constexpr bool kAffineStep = false;
  static constexpr int kNoiseCoord = -1;  // σ invertible (d = m)
  // theta: Theta (d×d row-major) at 0, mu at 9
  __device__ __forceinline__ static void drift(const T* th, const T* x, T* b) {
    T y[D];
#pragma unroll
    for (int q = 0; q < D; ++q) y[q] = x[q] - th[9 + q];
#pragma unroll
    for (int a = 0; a < D; ++a) {
      T acc = (-th[a * D + 0]) * y[0];
#pragma unroll
      for (int q = 1; q < D; ++q) acc = dfma(-th[a * D + q], y[q], acc);
      b[a] = acc;
    }
  }
};

template <class T>
struct FHN {
  static constexpr int D = 2, M = 1, NTH = 4;
  static constexpr bool kLinear = false;
  static constexpr int kNoiseCoord = 1;  // hypoelliptic: the noise enters coordinate 1 only
  // The guided Euler step as a per-step affine map plus the cubic term (round 6):
  // the drift's linear part (ε⁻¹(y − v + s), γy − v + β) and the guiding term's u = c − Mx are
  // folded into x' = A x + e, and only −ε⁻¹·dt·y³ depends on x non-linearly:
  //   ed = ε⁻¹·dt;  A00 = fma(−M00, dt, 1) + ed;  A01 = fma(−M01, dt, −ed);
  //   A10 = fma(−M10, dt, γ·dt);  A11 = fma(−M11, dt, 1 − dt);
  //   e0 = fma(c0, dt, fma(s, ed, σdW0));  e1 = fma(c1, dt, fma(β, dt, σdW1));  r = (−ed)·(y·y)
  //   y' = fma(r, y, fma(A00, y, fma(A01, v, e0)));   v' = fma(A10, y, fma(A11, v, e1))
  // The map {A, e, −ed} does not depend on x (computed lane-parallel ahead of a serial
  // recursion); the recursion's dependent chain per step is y·y → r → y' (three operations,
  // seven fp64 instructions per step in all), against five (sixteen) for the round-5 form.
  static constexpr bool kAffineStep = true;
  static constexpr int NS = 7;  // step-map values: A00, A01, A10, A11, e0, e1, −ed
  __device__ __forceinline__ static void step_map(const T* th, const T* Mg, const T* cg, T dt,
                                                  const T* sdW, T* sm) {
    const T ed = th[0] * dt;
    sm[0] = dfma(-Mg[0], dt, (T)1) + ed;
    sm[1] = dfma(-Mg[1], dt, -ed);
    sm[2] = dfma(-Mg[2], dt, th[2] * dt);
    sm[3] = dfma(-Mg[3], dt, (T)1 - dt);
    sm[4] = dfma(cg[0], dt, dfma(th[1], ed, sdW[0]));
    sm[5] = dfma(cg[1], dt, dfma(th[3], dt, sdW[1]));
    sm[6] = -ed;
  }
  __device__ __forceinline__ static void step_apply(const T* sm, T* x) {
    const T y = x[0], v = x[1];
    const T r = sm[6] * (y * y);
    const T y1 = dfma(r, y, dfma(sm[0], y, dfma(sm[1], v, sm[4])));
    const T v1 = dfma(sm[2], y, dfma(sm[3], v, sm[5]));
    x[0] = y1;
    x[1] = v1;
  }
  // theta: 1/eps, s, gamma, beta.  Canonical (round 5): t0 = fma(−y², y, y) +
  // (s − v), b0 = t0·ε⁻¹ (the drift of the Girsanov term) and the guided drift
  // bg0 = fma(t0, ε⁻¹, u0) (guided(): find_W_for_X!'s increment); the forward Euler step is the
  // step map above
  __device__ __forceinline__ static T t0(const T* th, const T* x) {
    const T y = x[0], v = x[1];
    return dfma(-(y * y), y, y) + (th[1] - v);
  }
  __device__ __forceinline__ static void drift(const T* th, const T* x, T* b) {
    const T y = x[0], v = x[1];
    b[0] = t0(th, x) * th[0];
    b[1] = dfma(th[2], y, th[3] - v);
  }
  // b_p + u_p of the Euler step (b from drift())
  __device__ __forceinline__ static T guided(const T* th, const T* x, const T* b, T u, int p) {
    return p == 0 ? dfma(t0(th, x), th[0], u) : b[p] + u;
  }
};

template <class T>
struct Lorenz {
  static constexpr int D = 3, M = 3, NTH = 3;
  static constexpr bool kLinear = false;
  static constexpr bool kAffineStep = false;
  static constexpr int kNoiseCoord = -1;
  // theta: s, r, beta
  __device__ __forceinline__ static void drift(const T* th, const T* x, T* b) {
    b[0] = th[0] * (x[1] - x[0]);
    b[1] = dfma(x[0], th[1] - x[2], -x[1]);
    b[2] = dfma(x[0], x[1], -(th[2] * x[2]));
  }
  __device__ __forceinline__ static T guided(const T*, const T*, const T* b, T u, int p) {
    return b[p] + u;
  }
};

// ---------------------------------------------------------------- law record in registers
template <class Mdl, class T>
struct Law {
  static constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2;
  T th[Mdl::NTH];
  T sg[D * M];
  T a[HP];
  T Bt[D * D];
  T beta[D];
  T da[HP];
  T thmu[D];  // Theta·mu of a linear (OU) drift, canonical order
  bool trace;
  bool auxtd;  // DMT_LAW_AUXTD: B̃, β̃ per step from the per-point table (dmt_upload_aux)
  bool auxa;   // DMT_LAW_AUXTD = 2: ã = σ̃σ̃ᵀ per step from the table too (dmt_upload_aux_a)
  // non-linear drift with σ exactly the identity (d = m; C5's Lorenz): canonical M = H, c = F,
  // σ·dW = dW, which the lane kernels take as a wave-uniform fast path
  bool unit;
  __device__ __forceinline__ void load(const double* L) {
    static_assert(DMT_LAW_THETA + Mdl::NTH <= DMT_LAW_GSTALE, "theta would overwrite the gstale slot");
#pragma unroll
    for (int i = 0; i < Mdl::NTH; ++i) th[i] = (T)ldc(L + DMT_LAW_THETA + i);
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int k = 0; k < M; ++k) sg[p * M + k] = (T)ldc(L + DMT_LAW_SIGMA + p * M + k);
#pragma unroll
    for (int i = 0; i < HP; ++i) a[i] = (T)ldc(L + DMT_LAW_A + i);
#pragma unroll
    for (int i = 0; i < D * D; ++i) Bt[i] = (T)ldc(L + DMT_LAW_BT + i);
#pragma unroll
    for (int i = 0; i < D; ++i) beta[i] = (T)ldc(L + DMT_LAW_BETA + i);
#pragma unroll
    for (int i = 0; i < HP; ++i) da[i] = (T)ldc(L + DMT_LAW_DA + i);
    trace = ldc(L + DMT_LAW_TRACE) != 0.0;
    auxtd = ldc(L + DMT_LAW_AUXTD) != 0.0;
    auxa = ldc(L + DMT_LAW_AUXTD) == 2.0;
    unit = !Mdl::kLinear && D == M;
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int k = 0; k < M; ++k) unit = unit && sg[p * M + k] == (p == k ? (T)1 : (T)0);
    if (Mdl::kLinear) {
#pragma unroll
      for (int p = 0; p < D; ++p) {
        T tm = th[p * D + 0] * th[9 + 0];
#pragma unroll
        for (int c = 1; c < D; ++c) tm = dfma(th[p * D + c], th[9 + c], tm);
        thmu[p] = tm;
      }
    }
  }
};

// Guiding coefficients of one step (independent of x): M = a·H (+ Theta for a linear
// drift), c = a·F (+ Theta·mu), canonical order.
template <class Mdl, class T>
__device__ __forceinline__ void guide_coeffs(const Law<Mdl, T>& L, const T* H, const T* F, T* Mg,
                                             T* cg) {
  constexpr int D = Mdl::D;
#pragma unroll
  for (int p = 0; p < D; ++p) {
#pragma unroll
    for (int q = 0; q < D; ++q) {
      T v = L.a[packed_idx(D, p, 0)] * H[packed_idx(D, 0, q)];
#pragma unroll
      for (int c = 1; c < D; ++c) v = dfma(L.a[packed_idx(D, p, c)], H[packed_idx(D, c, q)], v);
      Mg[p * D + q] = Mdl::kLinear ? (L.th[p * D + q] + v) : v;
    }
    T f = L.a[packed_idx(D, p, 0)] * F[0];
#pragma unroll
    for (int c = 1; c < D; ++c) f = dfma(L.a[packed_idx(D, p, c)], F[c], f);
    cg[p] = Mdl::kLinear ? (L.thmu[p] + f) : f;
  }
  if constexpr (!Mdl::kLinear) {  // σ = I: M = H, c = F exactly (canonical, per law)
#pragma unroll
    for (int p = 0; p < D; ++p) {
#pragma unroll
      for (int q = 0; q < D; ++q) Mg[p * D + q] = L.unit ? H[packed_idx(D, p, q)] : Mg[p * D + q];
      cg[p] = L.unit ? F[p] : cg[p];
    }
  }
}
// guide_coeffs of a law with L.unit (the caller knows it for the whole wave): no arithmetic
template <class Mdl, class T>
__device__ __forceinline__ void guide_coeffs_unit(const T* H, const T* F, T* Mg, T* cg) {
  constexpr int D = Mdl::D;
#pragma unroll
  for (int p = 0; p < D; ++p) {
#pragma unroll
    for (int q = 0; q < D; ++q) Mg[p * D + q] = H[packed_idx(D, p, q)];
    cg[p] = F[p];
  }
}

// G(t_i, x_i) of the Girsanov weight with the auxiliary drift B̃x + β̃ and the trace weights
// a − ã given (a time-dependent auxiliary law: step i's B̃(t_i), β̃(t_i), a − ã(t_i)); trace: the
// −½ tr((a − ã)(H − rrᵀ)) term is taken; returns G, writes r = F - Hx and the drift b.
template <class Mdl, class T>
__device__ __forceinline__ T g_at_aux(const Law<Mdl, T>& L, const T* H, const T* F, const T* x,
                                      T* r, T* b, const T* Bt, const T* beta, const T* da,
                                      bool trace) {
  constexpr int D = Mdl::D;
#pragma unroll
  for (int p = 0; p < D; ++p) {
    T acc = F[p];
#pragma unroll
    for (int q = 0; q < D; ++q) acc = dfma(-H[packed_idx(D, p, q)], x[q], acc);
    r[p] = acc;
  }
  Mdl::drift(L.th, x, b);
  T db[D];
#pragma unroll
  for (int p = 0; p < D; ++p) {
    T bt = beta[p];
#pragma unroll
    for (int q = 0; q < D; ++q) bt = dfma(Bt[p * D + q], x[q], bt);
    db[p] = b[p] - bt;
  }
  T G = db[0] * r[0];
#pragma unroll
  for (int p = 1; p < D; ++p) G = dfma(db[p], r[p], G);
  if (trace) {
    T tr = (T)0;
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int q = 0; q < D; ++q) {
        T tmp = dfma(-r[p], r[q], H[packed_idx(D, p, q)]);
        T w = da[packed_idx(D, p, q)];
        tr = (p == 0 && q == 0) ? (w * tmp) : dfma(w, tmp, tr);
      }
    G = dfma((T)-0.5, tr, G);
  }
  return G;
}
// G with the law's own (time-homogeneous) auxiliary drift
template <class Mdl, class T>
__device__ __forceinline__ T g_at(const Law<Mdl, T>& L, const T* H, const T* F, const T* x, T* r,
                                  T* b) {
  return g_at_aux<Mdl, T>(L, H, F, x, r, b, L.Bt, L.beta, L.da, L.trace);
}
// Columns of a per-point auxiliary-law table (dmt_upload_aux): B̃ (d·d), β̃ (d), ã packed (hp)
template <int D>
constexpr int kAuxCols = D * D + D + D * (D + 1) / 2;
// The auxiliary law of one step: the law's B̃, β̃, a − ã, or — where the lane's law is
// time-dependent (DMT_LAW_AUXTD) — the step's row of the per-point table, component c at
// row[c * cstride]: B̃, β̃, and with DMT_LAW_AUXTD = 2 also a − ã(t_i) = a − row's ã (in T);
// trace: whether G takes the trace term (the law's flag, or a table ã)
template <class Mdl, class T, class Ld>
__device__ __forceinline__ void aux_step(const Law<Mdl, T>& L, const T* row, int64_t cstride,
                                         T* Bt, T* beta, T* da, bool& trace, Ld ld) {
  constexpr int D = Mdl::D, HP = D * (D + 1) / 2;
#pragma unroll
  for (int c = 0; c < D * D; ++c) {
    const T v = ld(&row[c * cstride]);
    Bt[c] = L.auxtd ? v : L.Bt[c];
  }
#pragma unroll
  for (int p = 0; p < D; ++p) {
    const T v = ld(&row[(D * D + p) * cstride]);
    beta[p] = L.auxtd ? v : L.beta[p];
  }
  // the ã columns only where some lane's law takes ã(t) from the table (DMT_LAW_AUXTD = 2)
  if (__ballot(L.auxa) != 0) {
#pragma unroll
    for (int e = 0; e < HP; ++e) {
      const T v = ld(&row[(D * D + D + e) * cstride]);
      da[e] = L.auxa ? L.a[e] - v : L.da[e];
    }
  } else {
#pragma unroll
    for (int e = 0; e < HP; ++e) da[e] = L.da[e];
  }
  trace = L.trace || L.auxa;
}

// sigma·dW of one step (canonical: sdW_a = s_a0 dW_0, then fma over k)
template <class Mdl, class T>
__device__ __forceinline__ void sigma_dw(const Law<Mdl, T>& L, const T* dW, T* sdW) {
  constexpr int D = Mdl::D, M = Mdl::M;
#pragma unroll
  for (int p = 0; p < D; ++p) {
    T v = L.sg[p * M + 0] * dW[0];
#pragma unroll
    for (int k = 1; k < M; ++k) v = dfma(L.sg[p * M + k], dW[k], v);
    if constexpr (!Mdl::kLinear && D == M) v = L.unit ? dW[p] : v;  // σ = I: σ·dW = dW exactly
    sdW[p] = v;
  }
}

// One guided Euler–Maruyama step (left point), canonical order:
//   u_a = c_a - Σ_b M_ab x_b ;  bg = u (linear drift) or b(x) + u ;  x'_a = fma(bg_a, dt, x_a + sdW_a)
// b is the model drift at x (ignored for a linear drift, which M, c already contain).
template <class Mdl, class T>
__device__ __forceinline__ void euler_step(const T* th, const T* Mg, const T* cg, const T* b,
                                           T dt, const T* sdW, T* x) {
  constexpr int D = Mdl::D;
  if constexpr (Mdl::kAffineStep) {  // FHN: the step map, then the recursion's step (b unused)
    T sm[Mdl::NS];
    Mdl::step_map(th, Mg, cg, dt, sdW, sm);
    Mdl::step_apply(sm, x);
    return;
  }
  T xn[D];
#pragma unroll
  for (int p = 0; p < D; ++p) {
    T u = cg[p];
#pragma unroll
    for (int q = 0; q < D; ++q) u = dfma(-Mg[p * D + q], x[q], u);
    T bg;
    if constexpr (Mdl::kLinear) bg = u;
    else bg = Mdl::guided(th, x, b, u, p);
    xn[p] = dfma(bg, dt, x[p] + sdW[p]);
  }
#pragma unroll
  for (int p = 0; p < D; ++p) x[p] = xn[p];
}

// ---------------------------------------------------------------- affine form (linear drift)
// With a linear drift the guided Euler step is affine in x:
//   x' = A x + e,   A_ab = fma(-M_ab, dt, δ_ab),   e_a = fma(c_a, dt, sdW_a).
template <int D, class T>
__device__ __forceinline__ void affine_step(const T* Mg, const T* cg, T dt, const T* sdW, T* A,
                                            T* e) {
#pragma unroll
  for (int p = 0; p < D; ++p) {
#pragma unroll
    for (int q = 0; q < D; ++q) A[p * D + q] = dfma(-Mg[p * D + q], dt, p == q ? (T)1 : (T)0);
    e[p] = dfma(cg[p], dt, sdW[p]);
  }
}

// (A2, e2) ∘ (A1, e1): apply map 1, then map 2.  A = A2·A1, e = A2·e1 + e2, canonical order:
//   A_ab = A2_a0·A1_0b ; fma(A2_ac, A1_cb, ·) for c = 1..D-1 ;  e_a = e2_a ; fma(A2_ac, e1_c, ·)
template <int D, class T>
__device__ __forceinline__ void affine_compose(const T* A2, const T* e2, const T* A1, const T* e1,
                                               T* A, T* e) {
#pragma unroll
  for (int p = 0; p < D; ++p) {
#pragma unroll
    for (int q = 0; q < D; ++q) {
      T v = A2[p * D + 0] * A1[0 * D + q];
#pragma unroll
      for (int c = 1; c < D; ++c) v = dfma(A2[p * D + c], A1[c * D + q], v);
      A[p * D + q] = v;
    }
    T u = e2[p];
#pragma unroll
    for (int c = 0; c < D; ++c) u = dfma(A2[p * D + c], e1[c], u);
    e[p] = u;
  }
}

// y = A x + e:  y_a = e_a ; fma(A_ac, x_c, ·) for c = 0..D-1
template <int D, class T>
__device__ __forceinline__ void affine_apply(const T* A, const T* e, const T* x, T* y) {
#pragma unroll
  for (int p = 0; p < D; ++p) {
    T u = e[p];
#pragma unroll
    for (int c = 0; c < D; ++c) u = dfma(A[p * D + c], x[c], u);
    y[p] = u;
  }
}

// One step of DD.invsolve! (find_W_for_X!): the increment that maps x to xn under the guided
// Euler step, canonical order:
//   r_a  = fma(−bg_a, dt, xn_a − x_a)      (bg = c − Mx [+ b(x)], as in euler_step)
//   ΔW_k = σinv_k0·r_0 ; fma(σinv_ka, r_a, ·)     (d = m)
//   ΔW_0 = r_j / σ_j0                             (one noise on coordinate j = kNoiseCoord)
template <class Mdl, class T>
__device__ __forceinline__ void inv_step(const Law<Mdl, T>& L, const T* siginv, const T* Hi,
                                         const T* Fi, T dt, const T* x, const T* xn, T* dW) {
  constexpr int D = Mdl::D, M = Mdl::M;
  T Mg[D * D], cg[D], b[D];
  guide_coeffs<Mdl, T>(L, Hi, Fi, Mg, cg);
  if (!Mdl::kLinear) Mdl::drift(L.th, x, b);
  T r[D];
#pragma unroll
  for (int p = 0; p < D; ++p) {
    T u = cg[p];
#pragma unroll
    for (int q = 0; q < D; ++q) u = dfma(-Mg[p * D + q], x[q], u);
    T bg;
    if constexpr (Mdl::kLinear) bg = u;
    else bg = Mdl::guided(L.th, x, b, u, p);
    r[p] = dfma(-bg, dt, xn[p] - x[p]);
  }
  if constexpr (Mdl::kNoiseCoord >= 0) {
    dW[0] = r[Mdl::kNoiseCoord] / L.sg[Mdl::kNoiseCoord * M + 0];
  } else {
#pragma unroll
    for (int k = 0; k < M; ++k) {
      T v = siginv[k * D + 0] * r[0];
#pragma unroll
      for (int a = 1; a < D; ++a) v = dfma(siginv[k * D + a], r[a], v);
      dW[k] = v;
    }
  }
}

// loglikhd_obs = -c0 - 1/2 x'H x + F'x
template <int D, class T>
__device__ __forceinline__ T obs_term(const T* H0, const T* F0, const T* x, T c0) {
  T Hx[D];
#pragma unroll
  for (int p = 0; p < D; ++p) {
    T acc = H0[packed_idx(D, p, 0)] * x[0];
#pragma unroll
    for (int q = 1; q < D; ++q) acc = dfma(H0[packed_idx(D, p, q)], x[q], acc);
    Hx[p] = acc;
  }
  T quad = x[0] * Hx[0];
#pragma unroll
  for (int p = 1; p < D; ++p) quad = dfma(x[p], Hx[p], quad);
  T lin = F0[0] * x[0];
#pragma unroll
  for (int p = 1; p < D; ++p) lin = dfma(F0[p], x[p], lin);
  T tmp = dfma((T)-0.5, quad, lin);
  return tmp - c0;
}

// ---------------------------------------------------------------- chunked pairwise sum
// Streaming form of the adjacent-pair tree over chunks of 64 steps.
template <class T>
struct PSum {
  // s[j] holds the sum of the last complete aligned group of 2^j leaves while bit j of n is
  // set.  Updates are branch-free selects on the (wave-uniform) counter: no dynamic register
  // indexing (which would go through scratch memory).
  T s[7];
  int n;
  T acc;
  __device__ __forceinline__ void init() {
    n = 0;
    acc = (T)0;
#pragma unroll
    for (int j = 0; j < 7; ++j) s[j] = (T)0;
  }
  template <int LOG0>
  __device__ __forceinline__ void insert(T v) {  // a group of 2^LOG0 leaves, n % 2^LOG0 == 0
    bool go = true;
#pragma unroll
    for (int j = LOG0; j < 6; ++j) {
      const bool bit = (n >> j) & 1;
      const T merged = s[j] + v;
      s[j] = (go && !bit) ? v : s[j];
      v = (go && bit) ? merged : v;
      go = go && bit;
    }
    s[6] = go ? v : s[6];
    n += 1 << LOG0;
    if (n == 64) { acc = acc + (s[6] + (T)0); n = 0; }
  }
  __device__ __forceinline__ void add(T v) { insert<0>(v); }
  // Insert the sum of K consecutive leaves (an aligned subtree, K a power of two dividing 64,
  // n a multiple of K): identical to K single add()s.
  template <int LOGK>
  __device__ __forceinline__ void add_subtree(T v) { insert<LOGK>(v); }
  __device__ __forceinline__ T finish() {
    if (n > 0) {
      bool have = false;
      T r = (T)0;
#pragma unroll
      for (int lvl = 0; lvl < 6; ++lvl) {
        const bool bit = (n >> lvl) & 1;
        const T m = have ? (s[lvl] + r) : s[lvl];
        r = bit ? m : r;
        have = have || bit;
      }
      acc = acc + (r + (T)0);
      n = 0;
    }
    return acc;
  }
};

// ---------------------------------------------------------------- Philox4x32-10 + normals
struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
  k0 = __builtin_amdgcn_readfirstlane(k0);  // the key is the ensemble's seed: wave-uniform
  k1 = __builtin_amdgcn_readfirstlane(k1);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // full 64-bit products: one v_mad_u64_u32 each instead of a mul_lo + mul_hi pair
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    U4 n = {(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1,
            (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// ---------------------------------------------------------------- canonical transcendentals
// The normal and exponential draws use these explicit polynomial kernels (not the device
// libm), restated operation for operation in oracle/dmt_oracle.c, so that device-RNG draws
// are bit-identical to the CPU restatement.
#define RNG_SQRT_HALF 0x1.6a09e667f3bcdp-1
#define RNG_LN2_HI 0x1.62e42p-1
#define RNG_LN2_LO 0x1.fdf473de6af28p-22
#define RNG_P1 0x1.5555555555555p-1
#define RNG_P2 0x1.999999999999ap-2
#define RNG_P3 0x1.2492492492492p-2
#define RNG_P4 0x1.c71c71c71c71cp-3
#define RNG_P5 0x1.745d1745d1746p-3
#define RNG_P6 0x1.3b13b13b13b14p-3
#define RNG_P7 0x1.1111111111111p-3
#define RNG_P8 0x1.e1e1e1e1e1e1ep-4
#define RNG_P9 0x1.af286bca1af28p-4
#define RNG_P10 0x1.8618618618618p-4
#define RNG_P11 0x1.642c8590b2164p-4
#define RNGF_SQRT_HALF 0x1.6a09e6p-1f
#define RNGF_LN2_HI 0x1.62ep-1f
#define RNGF_LN2_LO 0x1.0bfbe8p-15f
#define RNGF_P1 0x1.555556p-1f
#define RNGF_P2 0x1.99999ap-2f
#define RNGF_P3 0x1.24924ap-2f
#define RNGF_P4 0x1.c71c72p-3f
#define RNGF_P5 0x1.745d18p-3f
#define RNGF_S0 0x1.921fb6p+1f
#define RNGF_S1 -0x1.4abbcep+2f
#define RNGF_S2 0x1.466bc6p+1f
#define RNGF_S3 -0x1.32d2ccp-1f
#define RNGF_S4 0x1.507834p-4f
#define RNGF_C1 -0x1.3bd3ccp+2f
#define RNGF_C2 0x1.03c1f0p+2f
#define RNGF_C3 -0x1.55d3c8p+0f
#define RNGF_C4 0x1.e1f506p-3f
#define RNGF_C5 -0x1.a6d1f2p-6f
/* log(u) for finite u > 0: u = m·2^e with m in [√½, √2); s = (m-1)/(m+1);
 * log(m) = 2s + s·z·P(z), z = s², P(z) = Σ_k 2/(2k+1) z^(k-1) (k = 1..11, Horner with fma);
 * log(u) = e·ln2_hi + (e·ln2_lo + log(m)). */
__device__ __forceinline__ double rng_log(double u) {
    int e;
    double m = __builtin_frexp(u, &e);
    const int lo = m < RNG_SQRT_HALF;
    m = lo ? m * 2.0 : m;
    e = lo ? e - 1 : e;
    const double f = m - 1.0;
    const double s = f / (2.0 + f);
    const double z = s * s;
    double p = RNG_P11;
    p = __builtin_fma(p, z, RNG_P10); p = __builtin_fma(p, z, RNG_P9); p = __builtin_fma(p, z, RNG_P8);
    p = __builtin_fma(p, z, RNG_P7); p = __builtin_fma(p, z, RNG_P6); p = __builtin_fma(p, z, RNG_P5);
    p = __builtin_fma(p, z, RNG_P4); p = __builtin_fma(p, z, RNG_P3); p = __builtin_fma(p, z, RNG_P2);
    p = __builtin_fma(p, z, RNG_P1);
    const double lm = __builtin_fma(s, z * p, 2.0 * s);
    const double de = (double)e;
    return __builtin_fma(de, RNG_LN2_HI, __builtin_fma(de, RNG_LN2_LO, lm));
}
__device__ __forceinline__ float rng_logf(float u) {
    int e;
    float m = __builtin_frexpf(u, &e);
    const int lo = m < RNGF_SQRT_HALF;
    m = lo ? m * 2.0f : m;
    e = lo ? e - 1 : e;
    const float f = m - 1.0f;
    const float s = f / (2.0f + f);
    const float z = s * s;
    float p = RNGF_P5;
    p = __builtin_fmaf(p, z, RNGF_P4); p = __builtin_fmaf(p, z, RNGF_P3); p = __builtin_fmaf(p, z, RNGF_P2);
    p = __builtin_fmaf(p, z, RNGF_P1);
    const float lm = __builtin_fmaf(s, z * p, 2.0f * s);
    const float de = (float)e;
    return __builtin_fmaf(de, RNGF_LN2_HI, __builtin_fmaf(de, RNGF_LN2_LO, lm));
}
// (round 5: a table-driven, division-free binary32 log in bm_log's form measured 17 % slower in
// the C5 packet kernel — 1 682–1 710 vs 1 437–1 442 µs per draw, profiles/r05e: the per-lane
// table reads are memory operations in a kernel that waits on its loads — and was not kept)
__device__ __forceinline__ void rng_sincospif(float x, float* sn, float* cs) {
    const float n = __builtin_rintf(2.0f * x);
    const float r = __builtin_fmaf(-0.5f, n, x);
    const float z = r * r;
    float sp = RNGF_S4;
    sp = __builtin_fmaf(sp, z, RNGF_S3); sp = __builtin_fmaf(sp, z, RNGF_S2); sp = __builtin_fmaf(sp, z, RNGF_S1);
    sp = __builtin_fmaf(sp, z, RNGF_S0);
    float cp = RNGF_C5;
    cp = __builtin_fmaf(cp, z, RNGF_C4); cp = __builtin_fmaf(cp, z, RNGF_C3); cp = __builtin_fmaf(cp, z, RNGF_C2);
    cp = __builtin_fmaf(cp, z, RNGF_C1);
    const float s0 = r * sp, c0 = __builtin_fmaf(cp, z, 1.0f);
    const int q = (int)n & 3;
    // quadrant q: (sin, cos) = (s0, c0), (c0, −s0), (−s0, −c0), (−c0, s0) — a swap on odd q and
    // sign flips (exact) on the sign bit, branch-free (the chained selects became divergent
    // branches)
    const bool sw = (q & 1) != 0;
    const uint32_t sa = __builtin_bit_cast(uint32_t, sw ? c0 : s0);
    const uint32_t ca = __builtin_bit_cast(uint32_t, sw ? s0 : c0);
    *sn = __builtin_bit_cast(float, sa ^ ((uint32_t)(q & 2) << 30));
    *cs = __builtin_bit_cast(float, ca ^ ((uint32_t)((q + 1) & 2) << 30));
}

// ---- fp64 Box–Muller kernels: table-driven (scripts/gen_bm_tables.py), no division, short
// dependency chains.  The fp64 normals are the dominant VALU cost of the OU MCMC kernels (C2:
// Box–Muller ≈ 45 % of k_mcmc_resident_pc's producer wave); the atanh-series rng_log with its
// division and the degree-17/18 sincospi took ≈ 1.6× the instructions.
#include "dmt_bm_tables.inc"
__constant__ double kBmLog[128][2] = DMT_BM_LOG_TABLE;
__constant__ double kBmSc[65][2] = DMT_BM_SC_TABLE;

/* log(u), u in [2^-53, 1]: u = m·2^e, m in [1, 2), j = top 7 mantissa bits; j < 64:
 * r = fma(m, c_j, -1), log u = e·ln2 + (L_j + log1p(r)); j >= 64: the same with e + 1 (c_j, L_j
 * relative to the interval's right end over 2); log1p(r) = fma(r², Q(r), r), Q Horner. */
__device__ __forceinline__ double bm_log(double u) {
  const uint64_t b = __builtin_bit_cast(uint64_t, u);
  const uint32_t hi = (uint32_t)(b >> 32);
  const int j = (int)((hi >> 13) & 0x7fu);
  const int e = (int)((hi >> 20) & 0x7ffu) - 1023 + (j >> 6);
  const double m = __builtin_bit_cast(double, (b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
  const double cj = kBmLog[j][0], Lj = kBmLog[j][1];
  const double r = __builtin_fma(m, cj, -1.0);
  const double r2 = r * r;
  double q = DMT_BM_Q6;
  q = __builtin_fma(q, r, DMT_BM_Q5); q = __builtin_fma(q, r, DMT_BM_Q4);
  q = __builtin_fma(q, r, DMT_BM_Q3); q = __builtin_fma(q, r, DMT_BM_Q2);
  q = __builtin_fma(q, r, DMT_BM_Q1); q = __builtin_fma(q, r, DMT_BM_Q0);
  const double lm = Lj + __builtin_fma(r2, q, r);
  const double de = (double)e;
  return __builtin_fma(de, RNG_LN2_HI, __builtin_fma(de, RNG_LN2_LO, lm));
}
/* sin(πx), cos(πx), x in [0, 2]: n = rint(32x), r = x - n/32 (exact), angle addition with
 * (S_n, C_n) = (sin, cos)(πn/32) from the table, sin(πr) = r·SP(r²), cos(πr) = fma(r², CP(r²), 1). */
__device__ __forceinline__ void bm_sincospi(double x, double* sn, double* cs) {
  const double n = __builtin_rint(32.0 * x);
  const double r = __builtin_fma(-0x1p-5, n, x);
  const double z = r * r;
  double sp = DMT_BM_S4;
  sp = __builtin_fma(sp, z, DMT_BM_S3); sp = __builtin_fma(sp, z, DMT_BM_S2);
  sp = __builtin_fma(sp, z, DMT_BM_S1); sp = __builtin_fma(sp, z, DMT_BM_S0);
  double cp = DMT_BM_C3;
  cp = __builtin_fma(cp, z, DMT_BM_C2); cp = __builtin_fma(cp, z, DMT_BM_C1);
  cp = __builtin_fma(cp, z, DMT_BM_C0);
  const double sr = r * sp, cr = __builtin_fma(cp, z, 1.0);
  const int k = (int)n;
  const double Sn = kBmSc[k][0], Cn = kBmSc[k][1];
  *sn = __builtin_fma(Sn, cr, Cn * sr);
  *cs = __builtin_fma(Cn, cr, -(Sn * sr));
}

__device__ __forceinline__ void normal_pair(U4 o, double& z0, double& z1) {
  uint64_t k1 = ((uint64_t)(o.x >> 5) << 26) | (o.y >> 6);
  uint64_t k2 = ((uint64_t)(o.z >> 5) << 26) | (o.w >> 6);
  double u1 = (double)(k1 + 1) * 0x1p-53;
  double u2 = (double)k2 * 0x1p-53;
  double rad = sqrt(-2.0 * bm_log(u1));
  double s, c;
  bm_sincospi(2.0 * u2, &s, &c);
  z0 = rad * c;
  z1 = rad * s;
}
__device__ __forceinline__ void normal_pair(U4 o, float& z0, float& z1) {
  float u1 = (float)((o.x >> 8) + 1u) * 0x1p-24f;
  float u2 = (float)(o.z >> 8) * 0x1p-24f;
  float rad = sqrtf(-2.0f * rng_logf(u1));
  float s, c;
  rng_sincospif(2.0f * u2, &s, &c);
  z0 = rad * c;
  z1 = rad * s;
}

__device__ __forceinline__ double exp1_draw(uint64_t seed, uint32_t blk, uint32_t iter,
                                            uint32_t salt) {
  U4 o = philox4x32_10(U4{blk, 0xFFFFFFFFu, iter, (salt << 1) | 1u}, (uint32_t)seed,
                       (uint32_t)(seed >> 32));
  uint64_t k1 = ((uint64_t)(o.x >> 5) << 26) | (o.y >> 6);
  double u = (double)(k1 + 1) * 0x1p-53;
  return -rng_log(u);
}

// Normals per Philox block of the perf-mode stream: fp64 Box–Muller takes 53-bit uniforms,
// built of the whole 128-bit block, for one pair; fp32 takes 24-bit uniforms, so a block gives
// two pairs — (z0, z1) of words (x, z), (z2, z3) of words (y, w) (orc_normal_block).
template <class T>
struct NormPerBlock {
  static constexpr int v = 2;
};
template <>
struct NormPerBlock<float> {
  static constexpr int v = 4;
};
__device__ __forceinline__ void normal_block(U4 o, double* z) { normal_pair(o, z[0], z[1]); }
__device__ __forceinline__ void normal_block(U4 o, float* z) {
  normal_pair(o, z[0], z[1]);
  normal_pair(U4{o.y, o.x, o.w, o.z}, z[2], z[3]);
}
// entry q of a block's normals without dynamic register indexing
template <class T, int NPB>
__device__ __forceinline__ T pick_normal(const T (&zb)[NPB], uint32_t q) {
  T r = zb[0];
#pragma unroll
  for (int e = 1; e < NPB; ++e) r = q == (uint32_t)e ? zb[e] : r;
  return r;
}

// Normal stream of one segment: normal n = step*M + k is entry n % NPB of the Philox block
// with counter (n / NPB, segment, iter, salt<<1).  get() is called with increasing n.
template <class T>
struct NormalStream {
  static constexpr int NPB = NormPerBlock<T>::v;
  uint32_t k0, k1, seg, iter, c3, have;
  T zb[NPB];
  __device__ __forceinline__ void init(uint64_t seed, uint32_t g, uint32_t it, uint32_t salt) {
    k0 = (uint32_t)seed; k1 = (uint32_t)(seed >> 32); seg = g; iter = it; c3 = salt << 1;
    have = 0xFFFFFFFFu;
  }
  __device__ __forceinline__ T get(uint32_t n) {
    if (n / NPB != have) {
      have = n / NPB;
      normal_block(philox4x32_10(U4{have, seg, iter, c3}, k0, k1), zb);
    }
    return pick_normal<T, NPB>(zb, n % NPB);
  }
};

}  // namespace dmt
