/*
 * dmt_oracle.c — CPU restatement of the guided-bridge imputation hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libdmt, the Python host
 * mirror, the Julia shim) links, loads or calls this file.  It is imported only
 * by tests/, __graft_entry__.smoke() and the cpu_baseline leg of bench.py, as
 * the checker and as the timed CPU baseline ("kind": "port").
 *
 * Parity status: the reference (DiffusionMCMCTools.jl) is pure Julia and its
 * arithmetic lives in GuidedProposals.jl v0.1.0 (git-tree 65cd150e…) and
 * DiffusionDefinition.jl v0.1.0 (git-tree 0ed61dbd…), pinned at
 * /root/reference/Manifest.toml:131-135,200-206 and NOT vendored; no julia
 * binary exists and the reference's own tests are empty
 * (/root/reference/test/runtests.jl:4-6).  This restatement is therefore
 * "parity unpinned" against reference outputs; it is pinned instead by the
 * analytic known-answer tests in tests/test_oracle_kat.py and by an
 * independent numpy restatement (oracle/np_oracle.py).
 *
 * What it restates (reference file:line → here):
 *   GP.rand!(PP, X°, W°, W, ρ, Val(:ll), y1)   src/biblock.jl:94-106       orc_pcn_segment + orc_solve_segment
 *   GP.solve_and_ll!(X, W, P, y1)              src/block.jl:165-167,180    orc_solve_segment
 *   GP.loglikhd(P, X)                          src/block.jl:138-144        orc_path_ll_segment
 *   GP.loglikhd_obs(P, y1)                     src/block.jl:178            orc_obs_term
 *   rand(Exponential(1.0))                     src/biblock.jl:122          orc_exp1 (perf-mode stream)
 *   randn inside rand!                         (upstream)                  orc_normal_pair (perf-mode stream)
 *
 * CANONICAL ARITHMETIC (the build's definition of one Euler step; the HIP
 * kernels follow it operation for operation, so that paths and log-weights
 * agree bit for bit under -ffp-contract=off with explicit fma):
 *
 *   Wiener paths are held as INCREMENTS: row 0 of a segment's W holds W(t_0), row i+1
 *   holds dW_i = W(t_{i+1}) - W(t_i).  Cumulative paths are converted at the boundary
 *   (dW_i = W[i+1] - W[i] on upload, W[i+1] = W[i] + dW_i on download).
 *
 *   dt      = t[i+1] - t[i]
 *   r_a     = F_a ; r_a = fma(-H_ab, x_b, r_a)        for b = 0..d-1
 *   b       = model drift (see orc_drift)
 *   guiding coefficients of the step (no dependence on x):
 *     aH_ab = a_a0*H_0b ; aH_ab = fma(a_ac, H_cb, aH_ab)  for c = 1..d-1
 *     aF_a  = a_a0*F_0  ; aF_a  = fma(a_ac, F_c, aF_a)
 *     linear drift (OU, b = -Theta(x - mu)):  M_ab = Theta_ab + aH_ab ; c_a = (Theta mu)_a + aF_a
 *       with (Theta mu)_a = Theta_a0*mu_0 ; fma(Theta_ac, mu_c, .)
 *     otherwise:                              M_ab = aH_ab ; c_a = aF_a
 *   u_a     = c_a ; u_a = fma(-M_ab, x_b, u_a)       for b = 0..d-1
 *   bg_a    = u_a (linear drift)  or  b_a + u_a      (= b + a(F - Hx) in exact arithmetic);
 *             FHN's bg_0 = fma(t0, 1/eps, u_0) with b_0 = t0·(1/eps) (orc_guided)
 *   bt_a    = Bt_a-row · x + beta_a  (bt_a = beta_a ; fma(Bt_ab, x_b, bt_a))
 *   db_a    = b_a - bt_a
 *   G       = db_0*r_0 ; G = fma(db_a, r_a, G)
 *   [trace] tr = Σ_a Σ_b da_ab*(H_ab - r_a r_b)  (tmp = fma(-r_a, r_b, H_ab);
 *            first term tr = da_00*tmp, then tr = fma(da_ab, tmp, tr)); G = fma(-0.5, tr, G)
 *   g       = G*dt           -> fed to the chunked pairwise sum
 *   sdW_a   = sigma_a0*dW_0 ; sdW_a = fma(sigma_ak, dW_k, sdW_a)  for k = 1..m-1
 *   x'_a    = fma(bg_a, dt, x_a + sdW_a)
 *
 *   LINEAR DRIFT (OU): the step is affine, x' = A x + e with A_ab = fma(-M_ab, dt, δ_ab),
 *   e_a = fma(c_a, dt, sdW_a), and the segment is evaluated as chunked Kogge–Stone prefix
 *   scans of these maps (solve_segment_scan below) — this REPLACES the last line above
 *   for OU models.  Lorenz uses the step-by-step form.
 *   FHN (round 6): the step is the affine map of the drift's linear part and u plus the cubic
 *   term (fhn_step) — this REPLACES the bg/x' lines above for FHN's forward step; bg_0 (with
 *   the fused scaling) remains the find_W_for_X! increment's (orc_invsolve_segment).
 *
 *   Log-weight summation: within a segment the g's are summed in chunks of 64
 *   consecutive steps by the adjacent-pair binary tree ((g0+g1)+(g2+g3))+…
 *   (a partial last chunk is padded with zeros), each chunk sum is
 *   canonicalised with "+ 0.0" and chunk sums are added left to right
 *   starting from 0.  Block ll = obs term, then += each segment's sum.
 *
 *   pCN (increment form, A.4 of SURVEY.md):  W°(t_0) = rho*W(t_0);
 *   dW°_i = fma(rho, dW_i, srho*(sqrt(t[i+1]-t[i])*Z_i))
 *   with srho = sqrt(1 - rho*rho) computed in double by the host (rho = 0, srho = 1 is a
 *   fresh draw; rho = 1, srho = 0 reproduces dW exactly).
 *
 * Compiled twice: REAL=double (suffix _f64) and REAL=float (suffix _f32).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#ifndef REAL
#define REAL double
#define SFX(n) n##_f64
#define FMA fma
#define SQRT sqrt
#define IS_F64 1
#endif

#define LAW_STRIDE 64
#define L_THETA 0
#define L_SIGMA 16
#define L_A 25
#define L_BT 31
#define L_BETA 40
#define L_DA 43
#define L_C0 49
#define L_TRACE 50
#define L_AUXTD 15

enum { ORC_OU = 0, ORC_FHN = 1, ORC_LORENZ = 2 };

/* packed upper-triangular index of a symmetric d×d matrix */
static inline int pidx(int d, int a, int b) {
    if (a > b) { int t = a; a = b; b = t; }
    return a * d - (a * (a - 1)) / 2 + (b - a);
}

/* FHN's t0 = fma(-y², y, y) + (s - v) (libdmt dmt_device.h FHN::t0). */
static inline REAL fhn_t0(const REAL* th, const REAL* x) {
    const REAL y = x[0], v = x[1];
    return FMA(-(y * y), y, y) + (th[1] - v);
}
/* FHN's guided Euler step as a per-step affine map plus the cubic term (round 6; libdmt
 * dmt_device.h FHN::step_map / step_apply):
 *   ed = (1/eps)·dt; A00 = fma(-M00, dt, 1) + ed; A01 = fma(-M01, dt, -ed);
 *   A10 = fma(-M10, dt, gamma·dt); A11 = fma(-M11, dt, 1 - dt);
 *   e0 = fma(c0, dt, fma(s, ed, sdW0)); e1 = fma(c1, dt, fma(beta, dt, sdW1)); r = (-ed)·(y·y)
 *   y' = fma(r, y, fma(A00, y, fma(A01, v, e0)));  v' = fma(A10, y, fma(A11, v, e1)) */
static inline void fhn_step(const REAL* th, const REAL* Mg, const REAL* cg, REAL dt,
                            const REAL* sdw, REAL* x) {
    const REAL ed = th[0] * dt;
    const REAL A00 = FMA(-Mg[0], dt, (REAL)1) + ed;
    const REAL A01 = FMA(-Mg[1], dt, -ed);
    const REAL A10 = FMA(-Mg[2], dt, th[2] * dt);
    const REAL A11 = FMA(-Mg[3], dt, (REAL)1 - dt);
    const REAL e0 = FMA(cg[0], dt, FMA(th[1], ed, sdw[0]));
    const REAL e1 = FMA(cg[1], dt, FMA(th[3], dt, sdw[1]));
    const REAL ned = -ed;
    const REAL y = x[0], v = x[1];
    const REAL r = ned * (y * y);
    x[0] = FMA(r, y, FMA(A00, y, FMA(A01, v, e0)));
    x[1] = FMA(A10, y, FMA(A11, v, e1));
}
/* b_p + u_p of the Euler step (libdmt FHN/Lorenz::guided): FHN's first coordinate fuses its
 * 1/eps scaling, bg0 = fma(t0, 1/eps, u0); every other coordinate b_p + u_p; OU: u_p. */
static inline REAL orc_guided(int model, const REAL* th, const REAL* x, const REAL* b, REAL u,
                              int p) {
    if (model == ORC_OU) return u;
    if (model == ORC_FHN && p == 0) return FMA(fhn_t0(th, x), th[0], u);
    return b[p] + u;
}

/* Model drifts (DiffusionDefinition models). */
static void orc_drift(int model, int d, const REAL* th, const REAL* x, REAL* b) {
    if (model == ORC_OU) {
        /* theta: Theta (d×d row-major, 0..8), mu (9..11); b = -Theta (x - mu) */
        REAL y[3];
        for (int q = 0; q < d; ++q) y[q] = x[q] - th[9 + q];
        for (int a = 0; a < d; ++a) {
            REAL acc = (-th[a * d + 0]) * y[0];
            for (int q = 1; q < d; ++q) acc = FMA(-th[a * d + q], y[q], acc);
            b[a] = acc;
        }
    } else if (model == ORC_FHN) {
        /* theta: 1/eps, s, gamma, beta.  dY = (Y - Y^3 - X + s)/eps, dX = (gamma Y - X + beta);
         * canonical (round 5): t0 = fma(-y², y, y) + (s - v), b0 = t0·(1/eps) */
        REAL y = x[0], v = x[1];
        b[0] = fhn_t0(th, x) * th[0];
        b[1] = FMA(th[2], y, th[3] - v);
    } else { /* Lorenz-63: theta: s, r, beta */
        b[0] = th[0] * (x[1] - x[0]);
        b[1] = FMA(x[0], th[1] - x[2], -x[1]);
        b[2] = FMA(x[0], x[1], -(th[2] * x[2]));
    }
}

typedef struct { REAL s[7]; int n; REAL acc; } psum_t;

static inline void ps_init(psum_t* p) { p->n = 0; p->acc = (REAL)0; }
static inline void ps_add(psum_t* p, REAL v) {
    int k = p->n, lvl = 0;
    while (k & 1) { v = p->s[lvl] + v; k >>= 1; ++lvl; }
    p->s[lvl] = v;
    if (++p->n == 64) { p->acc = p->acc + (p->s[6] + (REAL)0); p->n = 0; }
}
static inline REAL ps_finish(psum_t* p) {
    if (p->n > 0) {
        int have = 0; REAL r = (REAL)0;
        for (int lvl = 0; lvl < 6; ++lvl)
            if ((p->n >> lvl) & 1) { r = have ? (p->s[lvl] + r) : p->s[lvl]; have = 1; }
        p->acc = p->acc + (r + (REAL)0);
        p->n = 0;
    }
    return p->acc;
}

static void load_law(const double* law, int d, int m, REAL* th, REAL* sg, REAL* a,
                     REAL* Bt, REAL* beta, REAL* da, int* trace) {
    for (int i = 0; i < 16; ++i) th[i] = (REAL)law[L_THETA + i];
    for (int i = 0; i < 9; ++i) sg[i] = (REAL)law[L_SIGMA + i];
    for (int i = 0; i < 6; ++i) a[i] = (REAL)law[L_A + i];
    for (int i = 0; i < 9; ++i) Bt[i] = (REAL)law[L_BT + i];
    for (int i = 0; i < 3; ++i) beta[i] = (REAL)law[L_BETA + i];
    for (int i = 0; i < 6; ++i) da[i] = (REAL)law[L_DA + i];
    *trace = law[L_TRACE] != 0.0;
    (void)d; (void)m;
}

/* G(t_i, x) at a point (canonical), writes r and b for the caller. */
static inline REAL g_at(int model, int d, const REAL* th, const REAL* a, const REAL* Bt,
                        const REAL* beta, const REAL* da, int trace,
                        const REAL* H, const REAL* F, const REAL* x, REAL* r, REAL* b) {
    for (int p = 0; p < d; ++p) {
        REAL acc = F[p];
        for (int q = 0; q < d; ++q) acc = FMA(-H[pidx(d, p, q)], x[q], acc);
        r[p] = acc;
    }
    orc_drift(model, d, th, x, b);
    REAL db[3] = {0, 0, 0};
    for (int p = 0; p < d; ++p) {
        REAL bt = beta[p];
        for (int q = 0; q < d; ++q) bt = FMA(Bt[p * d + q], x[q], bt);
        db[p] = b[p] - bt;
    }
    REAL G = db[0] * r[0];
    for (int p = 1; p < d; ++p) G = FMA(db[p], r[p], G);
    if (trace) {
        REAL tr = (REAL)0; int first = 1;
        for (int p = 0; p < d; ++p)
            for (int q = 0; q < d; ++q) {
                REAL tmp = FMA(-r[p], r[q], H[pidx(d, p, q)]);
                REAL w = da[pidx(d, p, q)];
                tr = first ? (w * tmp) : FMA(w, tmp, tr);
                first = 0;
            }
        G = FMA((REAL)-0.5, tr, G);
    }
    (void)a;
    return G;
}

/* A non-linear drift whose σ is exactly the identity (d = m): the canonical rule M = H, c = F,
 * σ·dW = dW (libdmt dmt_device.h Law::unit). */
static inline int law_unit(int model, int d, int m, const REAL* sg) {
    if (model == ORC_OU || d != m) return 0;
    for (int p = 0; p < d; ++p)
        for (int k = 0; k < m; ++k)
            if (sg[p * m + k] != (p == k ? (REAL)1 : (REAL)0)) return 0;
    return 1;
}

/* Per-step guiding coefficients M (d×d row-major) and c (d) of the Euler update. */
static inline void guide_coeffs(int model, int d, const REAL* th, const REAL* a, const REAL* H,
                                const REAL* F, REAL* Mg, REAL* cg, int unit) {
    for (int p = 0; p < d; ++p) {
        for (int q = 0; q < d; ++q) {
            REAL v = a[pidx(d, p, 0)] * H[pidx(d, 0, q)];
            for (int c = 1; c < d; ++c) v = FMA(a[pidx(d, p, c)], H[pidx(d, c, q)], v);
            Mg[p * d + q] = v;
        }
        REAL f = a[pidx(d, p, 0)] * F[0];
        for (int c = 1; c < d; ++c) f = FMA(a[pidx(d, p, c)], F[c], f);
        cg[p] = f;
    }
    if (model == ORC_OU) { /* linear drift b = -Theta(x - mu) folded in */
        for (int p = 0; p < d; ++p) {
            REAL tm = th[p * d + 0] * th[9 + 0];
            for (int c = 1; c < d; ++c) tm = FMA(th[p * d + c], th[9 + c], tm);
            for (int q = 0; q < d; ++q) Mg[p * d + q] = th[p * d + q] + Mg[p * d + q];
            cg[p] = tm + cg[p];
        }
    }
    if (unit) { /* σ = I: M = H, c = F exactly */
        for (int p = 0; p < d; ++p) {
            for (int q = 0; q < d; ++q) Mg[p * d + q] = H[pidx(d, p, q)];
            cg[p] = F[p];
        }
    }
}

/* Affine form of a linear-drift step and its composition (CANONICAL ARITHMETIC, scan form):
 *   A_ab = fma(-M_ab, dt, δ_ab), e_a = fma(c_a, dt, sdW_a)            x' = A x + e
 *   (A2,e2)∘(A1,e1): A_ab = A2_a0*A1_0b ; fma(A2_ac, A1_cb, .) c=1..d-1
 *                    e_a  = e2_a ; fma(A2_ac, e1_c, .) c=0..d-1
 *   apply:           y_a  = e_a ; fma(A_ac, x_c, .) c=0..d-1 */
static void aff_compose(int d, const REAL* A2, const REAL* e2, const REAL* A1, const REAL* e1,
                        REAL* A, REAL* e) {
    for (int p = 0; p < d; ++p) {
        for (int q = 0; q < d; ++q) {
            REAL v = A2[p * d + 0] * A1[0 * d + q];
            for (int c = 1; c < d; ++c) v = FMA(A2[p * d + c], A1[c * d + q], v);
            A[p * d + q] = v;
        }
        REAL u = e2[p];
        for (int c = 0; c < d; ++c) u = FMA(A2[p * d + c], e1[c], u);
        e[p] = u;
    }
}
static void aff_apply(int d, const REAL* A, const REAL* e, const REAL* x, REAL* y) {
    for (int p = 0; p < d; ++p) {
        REAL u = e[p];
        for (int c = 0; c < d; ++c) u = FMA(A[p * d + c], x[c], u);
        y[p] = u;
    }
}

/* Linear drift (OU): the guided Euler recursion is affine, x_{i+1} = A_i x_i + e_i.  The
 * canonical evaluation (the HIP kernels' scan_block) cuts the segment into
 * chunks of 512 steps and every chunk into 64 runs of 8 consecutive steps:
 *   run map     R_j = step_{last valid} ∘ … ∘ step_first (sequential compose; identity when
 *               the run has no valid step);
 *   prefix      inclusive Kogge–Stone over the 64 run maps (level o = 1,2,4,…,32: element
 *               j ← element j ∘ element j-o for j ≥ o, all reading the previous level);
 *   run start   s_0 = x_{c0}, s_j = apply(P_{j-1}, x_{c0});
 *   points      within a run, x_{i+1} = apply(step_i, x_i) one step at a time from s_j;
 *   next chunk  starts at the end point of the chunk's last valid step.
 * The Girsanov sum keeps the common order: adjacent-pair trees over 64-step chunks from the
 * segment start, chunk sums added left to right (psum). */
#define ORC_RUN 8
#define ORC_SCHUNK 512
extern int orc_ll_skip;
/* The kernels' inclusive scan of the 64 lanes' run maps (libdmt wave_affine_scan, DPP):
 * Kogge–Stone within each row of 16 lanes (lane j composes after lane j − o when j mod 16 >= o,
 * o = 1, 2, 4, 8), then rows 1 and 3 after lane 15 / 47 (row_bcast:15), then rows 2 and 3 after
 * lane 31 (row_bcast:31); every level reads the previous level's maps. */
#ifndef ORC_SCAN_DPP  /* the tree libdmt is built with (DMT_SCAN_DPP) */
#define ORC_SCAN_DPP 0
#endif
#if ORC_SCAN_DPP
static int dpp_src(int level, int j) {
    if (level < 4) { int o = 1 << level; return (j & 15) >= o ? j - o : -1; }
    if (level == 4) return (j & 16) ? (j & ~15) - 1 : -1;
    return j >= 32 ? 31 : -1;
}
static void wave_scan_dpp(int d, REAL RA[64][9], REAL Re[64][3], REAL An[64][9], REAL en[64][3]) {
    for (int level = 0; level < 6; ++level) {
        for (int j = 0; j < 64; ++j) {
            int src = dpp_src(level, j);
            if (src >= 0) aff_compose(d, RA[j], Re[j], RA[src], Re[src], An[j], en[j]);
        }
        for (int j = 0; j < 64; ++j) {
            if (dpp_src(level, j) < 0) continue;
            memcpy(RA[j], An[j], sizeof(REAL) * d * d);
            memcpy(Re[j], en[j], sizeof(REAL) * d);
        }
    }
}
#endif
static inline const REAL* aux_coeffs(const double* law, int model, int d, int i, const REAL* Bt,
                                     const REAL* beta, REAL* Bq, REAL* bq, const REAL** bo,
                                     const REAL* a, const REAL* da, int trace, REAL* dq,
                                     const REAL** dao, int* tro);
static int solve_segment_scan(const double* law, int d, int m, const REAL* th, const REAL* sg,
                              const REAL* a, const REAL* Bt, const REAL* beta, const REAL* da,
                              int trace,
                              int npts, const REAL* t, const REAL* H, const REAL* F,
                              const REAL* W, const REAL* y1, REAL* X, REAL* ll_out) {
    int h = d * (d + 1) / 2;
    int n = npts - 1;
    REAL xs[3];
    for (int p = 0; p < d; ++p) { xs[p] = y1[p]; X[p] = xs[p]; }
    psum_t ps; ps_init(&ps);
    static __thread REAL A[ORC_SCHUNK][9], e[ORC_SCHUNK][3];
    static __thread REAL RA[64][9], Re[64][3], An[64][9], en[64][3];
    for (int c0 = 0; c0 < n; c0 += ORC_SCHUNK) {
        int cnt = n - c0 < ORC_SCHUNK ? n - c0 : ORC_SCHUNK;
        for (int j = 0; j < ORC_SCHUNK; ++j) {
            if (j < cnt) {
                int i = c0 + j;
                REAL dt = t[i + 1] - t[i];
                const REAL* dW = W + (size_t)(i + 1) * m;
                REAL Mg[9], cg[3], sdw[3];
                guide_coeffs(ORC_OU, d, th, a, H + (size_t)i * h, F + (size_t)i * d, Mg, cg, 0);
                for (int p = 0; p < d; ++p) {
                    REAL v = sg[p * m + 0] * dW[0];
                    for (int k = 1; k < m; ++k) v = FMA(sg[p * m + k], dW[k], v);
                    sdw[p] = v;
                }
                for (int p = 0; p < d; ++p) {
                    for (int q = 0; q < d; ++q)
                        A[j][p * d + q] = FMA(-Mg[p * d + q], dt, p == q ? (REAL)1 : (REAL)0);
                    e[j][p] = FMA(cg[p], dt, sdw[p]);
                }
            } else {
                for (int p = 0; p < d; ++p) {
                    for (int q = 0; q < d; ++q) A[j][p * d + q] = p == q ? (REAL)1 : (REAL)0;
                    e[j][p] = (REAL)0;
                }
            }
        }
        /* run maps */
        for (int j = 0; j < 64; ++j) {
            int s0 = ORC_RUN * j;
            int nv = cnt - s0; nv = nv < 0 ? 0 : nv > ORC_RUN ? ORC_RUN : nv;
            memcpy(RA[j], A[s0], sizeof(REAL) * d * d);
            memcpy(Re[j], e[s0], sizeof(REAL) * d);
            for (int r = 1; r < nv; ++r) {
                REAL tA[9], te[3];
                aff_compose(d, A[s0 + r], e[s0 + r], RA[j], Re[j], tA, te);
                memcpy(RA[j], tA, sizeof(REAL) * d * d);
                memcpy(Re[j], te, sizeof(REAL) * d);
            }
        }
#if ORC_SCAN_DPP
        wave_scan_dpp(d, RA, Re, An, en);
#else
        for (int o = 1; o < 64; o <<= 1) {
            for (int j = o; j < 64; ++j) aff_compose(d, RA[j], Re[j], RA[j - o], Re[j - o], An[j], en[j]);
            for (int j = o; j < 64; ++j) {
                memcpy(RA[j], An[j], sizeof(REAL) * d * d);
                memcpy(Re[j], en[j], sizeof(REAL) * d);
            }
        }
#endif
        REAL xend[3];
        for (int j = 0; j < 64 && ORC_RUN * j < cnt; ++j) {
            REAL x[3];
            if (j == 0) { for (int p = 0; p < d; ++p) x[p] = xs[p]; }
            else aff_apply(d, RA[j - 1], Re[j - 1], xs, x);
            int s0 = ORC_RUN * j;
            int nv = cnt - s0 > ORC_RUN ? ORC_RUN : cnt - s0;
            for (int r = 0; r < nv; ++r) {
                int i = c0 + s0 + r;
                REAL dt = t[i + 1] - t[i];
                REAL rr[3] = {0, 0, 0}, b[3] = {0, 0, 0};
                if (i > 0) for (int p = 0; p < d; ++p) X[(size_t)i * d + p] = x[p];
                REAL Bq[9], bq[3], dq[6];
                const REAL *bu, *du;
                int tu;
                const REAL* Bu = aux_coeffs(law, ORC_OU, d, i, Bt, beta, Bq, bq, &bu, a, da, trace,
                                            dq, &du, &tu);
                REAL G = g_at(ORC_OU, d, th, a, Bu, bu, du, tu, H + (size_t)i * h,
                              F + (size_t)i * d, x, rr, b);
                ps_add(&ps, i < n - orc_ll_skip ? G * dt : (REAL)0);
                REAL xp[3];
                aff_apply(d, A[s0 + r], e[s0 + r], x, xp);
                for (int p = 0; p < d; ++p) x[p] = xp[p];
            }
            for (int p = 0; p < d; ++p) xend[p] = x[p];
        }
        for (int p = 0; p < d; ++p) xs[p] = xend[p];
    }
    for (int p = 0; p < d; ++p) X[(size_t)n * d + p] = xs[p];
    REAL ll = ps_finish(&ps);
    *ll_out = ll;
    int ok = isfinite(ll) ? 1 : 0;
    for (int p = 0; p < d; ++p) ok &= isfinite(xs[p]) ? 1 : 0;
    return ok;
}

/* recompute_path!(…; skip) (src/block.jl:159-187 → GP.solve_and_ll!(…; skip), GuidedProposals
 * v0.1.0, not vendored): the last orc_ll_skip Euler steps of a segment add no Girsanov term —
 * the term is replaced by 0 in the same position of the psum tree; the path is solved to the
 * end.  Set by oracle.py around recompute_path (0 everywhere else). */
#if IS_F64
int orc_ll_skip = 0;
void orc_set_ll_skip(int k) { orc_ll_skip = k; }
#else
extern int orc_ll_skip;
#endif

/* Time-dependent auxiliary law of the segment being solved (libdmt dmt_upload_aux(_a); set by
 * oracle.py around a segment call, NULL otherwise): rows [npts][d*d + d + d(d+1)/2] =
 * B~(t_i), beta~(t_i), a~(t_i) packed (zeros where not given), used at step i (left point) in
 * place of the record's Bt, beta when the record's auxtd (offset 15) is set, and — auxtd = 2 —
 * a − a~(t_i) (in the working precision) in place of the record's a − a~ in G's trace term,
 * which is then taken whatever the record's trace flag (libdmt aux_step).  A linear drift's
 * scan (solve_segment_scan) takes it in G only: the recursion is the target law's. */
#if IS_F64
const double* orc_aux = 0;
void orc_set_aux(const double* p) { orc_aux = p; }
#else
extern const double* orc_aux;
#endif
static inline const REAL* aux_coeffs(const double* law, int model, int d, int i, const REAL* Bt,
                                     const REAL* beta, REAL* Bq, REAL* bq, const REAL** bo,
                                     const REAL* a, const REAL* da, int trace, REAL* dq,
                                     const REAL** dao, int* tro) {
    *dao = da;
    *tro = trace;
    if (!orc_aux || law[L_AUXTD] == 0.0) { *bo = beta; return Bt; }
    const int hp = d * (d + 1) / 2;
    const double* row = orc_aux + (size_t)i * (d * d + d + hp);
    for (int k = 0; k < d * d; ++k) Bq[k] = (REAL)row[k];
    for (int p = 0; p < d; ++p) bq[p] = (REAL)row[d * d + p];
    if (law[L_AUXTD] == 2.0) {
        for (int e = 0; e < hp; ++e) dq[e] = a[e] - (REAL)row[d * d + d + e];
        *dao = dq;
        *tro = 1;
    }
    *bo = bq;
    return Bq;
}

/* CPU-baseline switch (bench.py's cpu_baseline only): 1 = evaluate linear-drift segments
 * with the plain step-by-step Euler loop — the natural CPU algorithm, as the reference runs
 * it — instead of the canonical chunked scan (equal up to rounding; not used for parity). */
#if IS_F64
int orc_sequential_ou = 0;
void orc_set_sequential_ou(int on) { orc_sequential_ou = on; }
#else
extern int orc_sequential_ou;
#endif

/* GP.solve_and_ll!(X, W, P, y1): Euler–Maruyama guided solve with given W and
 * the Girsanov sum.  Returns 1 on success (finite end point and ll). */
int SFX(orc_solve_segment)(int model, int d, int m, const double* law, int npts,
                           const REAL* t, const REAL* H, const REAL* F, const REAL* W,
                           const REAL* y1, REAL* X, REAL* ll_out) {
    int h = d * (d + 1) / 2;
    REAL th[16], sg[9], a[6], Bt[9], beta[3], da[6]; int trace;
    load_law(law, d, m, th, sg, a, Bt, beta, da, &trace);
    const int unit = law_unit(model, d, m, sg);
    if (model == ORC_OU && !orc_sequential_ou)
        return solve_segment_scan(law, d, m, th, sg, a, Bt, beta, da, trace, npts, t, H, F, W, y1,
                                  X, ll_out);
    REAL x[3];
    for (int p = 0; p < d; ++p) { x[p] = y1[p]; X[p] = x[p]; }
    psum_t ps; ps_init(&ps);
    for (int i = 0; i < npts - 1; ++i) {
        REAL dt = t[i + 1] - t[i];
        const REAL* dW = W + (size_t)(i + 1) * m;  /* increments */
        const REAL* Hi = H + (size_t)i * h;
        const REAL* Fi = F + (size_t)i * d;
        REAL r[3] = {0, 0, 0}, b[3] = {0, 0, 0};
        REAL Bq[9], bq[3], dq[6];
        const REAL *bu, *du;
        int tu;
        const REAL* Bu = aux_coeffs(law, model, d, i, Bt, beta, Bq, bq, &bu, a, da, trace, dq, &du, &tu);
        REAL G = g_at(model, d, th, a, Bu, bu, du, tu, Hi, Fi, x, r, b);
        ps_add(&ps, i < npts - 1 - orc_ll_skip ? G * dt : (REAL)0);
        REAL Mg[9], cg[3];
        guide_coeffs(model, d, th, a, Hi, Fi, Mg, cg, unit);
        REAL xn[3];
        if (model == ORC_FHN) {  /* the step map (fhn_step) */
            REAL sdw[2];
            for (int p = 0; p < 2; ++p) sdw[p] = sg[p * m + 0] * dW[0];
            xn[0] = x[0]; xn[1] = x[1];
            fhn_step(th, Mg, cg, dt, sdw, xn);
        } else for (int p = 0; p < d; ++p) {
            REAL u = cg[p];
            for (int q = 0; q < d; ++q) u = FMA(-Mg[p * d + q], x[q], u);
            REAL bg = orc_guided(model, th, x, b, u, p);
            REAL sdw = sg[p * m + 0] * dW[0];
            for (int k = 1; k < m; ++k) sdw = FMA(sg[p * m + k], dW[k], sdw);
            if (unit) sdw = dW[p];
            xn[p] = FMA(bg, dt, x[p] + sdw);
        }
        for (int p = 0; p < d; ++p) { x[p] = xn[p]; X[(size_t)(i + 1) * d + p] = xn[p]; }
    }
    REAL ll = ps_finish(&ps);
    *ll_out = ll;
    int ok = isfinite(ll) ? 1 : 0;
    for (int p = 0; p < d; ++p) ok &= isfinite(x[p]) ? 1 : 0;
    return ok;
}


/* DD.invsolve!(X, W, P) (find_W_for_X!, src/block.jl:118-131): increments reproducing X
 * under the guided Euler step of law P (canonical order):
 *   r_a = fma(-bg_a, dt, x_{i+1,a} - x_{i,a});  dW = siginv·r (d = m), or r_1 / sigma_10 (FHN).
 * W is written as increments with W(t0) = 0. */
void SFX(orc_invsolve_segment)(int model, int d, int m, const double* law, int npts,
                               const REAL* t, const REAL* H, const REAL* F, const REAL* X,
                               REAL* W) {
    int h = d * (d + 1) / 2;
    REAL th[16], sg[9], a[6], Bt[9], beta[3], da[6]; int trace;
    load_law(law, d, m, th, sg, a, Bt, beta, da, &trace);
    const int unit = law_unit(model, d, m, sg);
    REAL siginv[9];
    for (int i = 0; i < 9; ++i) siginv[i] = (REAL)law[51 + i];
    for (int k = 0; k < m; ++k) W[k] = (REAL)0;
    for (int i = 0; i < npts - 1; ++i) {
        REAL dt = t[i + 1] - t[i];
        const REAL* x = X + (size_t)i * d;
        const REAL* xn = X + (size_t)(i + 1) * d;
        REAL Mg[9], cg[3], b[3] = {0, 0, 0}, r[3];
        guide_coeffs(model, d, th, a, H + (size_t)i * h, F + (size_t)i * d, Mg, cg, unit);
        if (model != ORC_OU) orc_drift(model, d, th, x, b);
        for (int p = 0; p < d; ++p) {
            REAL u = cg[p];
            for (int q = 0; q < d; ++q) u = FMA(-Mg[p * d + q], x[q], u);
            REAL bg = orc_guided(model, th, x, b, u, p);
            r[p] = FMA(-bg, dt, xn[p] - x[p]);
        }
        REAL* dW = W + (size_t)(i + 1) * m;
        if (model == ORC_FHN) {
            dW[0] = r[1] / sg[1 * m + 0];
        } else {
            for (int k = 0; k < m; ++k) {
                REAL v = siginv[k * d + 0] * r[0];
                for (int q = 1; q < d; ++q) v = FMA(siginv[k * d + q], r[q], v);
                dW[k] = v;
            }
        }
    }
}

/* GP.loglikhd(P, X): Girsanov sum on a stored path (no state update). */
REAL SFX(orc_path_ll_segment)(int model, int d, int m, const double* law, int npts,
                              const REAL* t, const REAL* H, const REAL* F, const REAL* X) {
    int h = d * (d + 1) / 2;
    REAL th[16], sg[9], a[6], Bt[9], beta[3], da[6]; int trace;
    load_law(law, d, m, th, sg, a, Bt, beta, da, &trace);
    psum_t ps; ps_init(&ps);
    for (int i = 0; i < npts - 1; ++i) {
        REAL dt = t[i + 1] - t[i];
        REAL r[3] = {0, 0, 0}, b[3] = {0, 0, 0};
        REAL Bq[9], bq[3], dq[6];
        const REAL *bu, *du;
        int tu;
        const REAL* Bu = aux_coeffs(law, model, d, i, Bt, beta, Bq, bq, &bu, a, da, trace, dq, &du, &tu);
        REAL G = g_at(model, d, th, a, Bu, bu, du, tu, H + (size_t)i * h,
                      F + (size_t)i * d, X + (size_t)i * d, r, b);
        ps_add(&ps, G * dt);
    }
    return ps_finish(&ps);
}

/* GP.loglikhd_obs(P, y1) = log rho~(t0, y1) = -c0 - 1/2 y'H y + F'y */
REAL SFX(orc_obs_term)(int d, const double* law, const REAL* H0, const REAL* F0, const REAL* x) {
    REAL Hx[3] = {0, 0, 0};
    for (int p = 0; p < d; ++p) {
        REAL acc = H0[pidx(d, p, 0)] * x[0];
        for (int q = 1; q < d; ++q) acc = FMA(H0[pidx(d, p, q)], x[q], acc);
        Hx[p] = acc;
    }
    REAL quad = x[0] * Hx[0];
    for (int p = 1; p < d; ++p) quad = FMA(x[p], Hx[p], quad);
    REAL lin = F0[0] * x[0];
    for (int p = 1; p < d; ++p) lin = FMA(F0[p], x[p], lin);
    REAL tmp = FMA((REAL)-0.5, quad, lin);
    return tmp - (REAL)law[L_C0];
}

/* pCN mix of one segment (increment form). */
void SFX(orc_pcn_segment)(int m, int npts, const REAL* t, const REAL* W, const REAL* Z,
                          REAL rho, REAL srho, REAL* Wo) {
    for (int k = 0; k < m; ++k) Wo[k] = rho * W[k];
    for (int q = 0; q < npts - 1; ++q) {
        REAL sdt = SQRT(t[q + 1] - t[q]);
        for (int k = 0; k < m; ++k) {
            REAL zi = sdt * Z[(size_t)q * m + k];
            Wo[(size_t)(q + 1) * m + k] = FMA(rho, W[(size_t)(q + 1) * m + k], srho * zi);
        }
    }
}

/* cumulative <-> increment conversion of one segment's Wiener path (m components) */
void SFX(orc_w_to_increments)(int m, int npts, const REAL* W, REAL* dW) {
    for (int k = 0; k < m; ++k) dW[k] = W[k];
    for (int q = 0; q < npts - 1; ++q)
        for (int k = 0; k < m; ++k)
            dW[(size_t)(q + 1) * m + k] = W[(size_t)(q + 1) * m + k] - W[(size_t)q * m + k];
}
void SFX(orc_w_from_increments)(int m, int npts, const REAL* dW, REAL* W) {
    for (int k = 0; k < m; ++k) W[k] = dW[k];
    for (int q = 0; q < npts - 1; ++q)
        for (int k = 0; k < m; ++k)
            W[(size_t)(q + 1) * m + k] = W[(size_t)q * m + k] + dW[(size_t)(q + 1) * m + k];
}

/*
 * Whole-ensemble draw for single-segment terminal blocks (the synthetic
 * configs C2-C5), OpenMP over blocks.  Reference layout: block b owns points
 * [b*npts, (b+1)*npts).  Used as the timed CPU baseline and for big parity
 * tests.  Z: [B][npts-1][m] (NULL -> perf-mode Philox stream with seed/iter).
 * Each block may have its own tables (H_stride/F_stride = 0 means shared).
 */
/* normals per Philox block of the perf-mode stream (orc_normal_block) */
#if IS_F64
#define ORC_NPB 2
#else
#define ORC_NPB 4
#endif
void SFX(orc_normal_block)(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                           REAL* z);

int SFX(orc_draw_terminal_blocks)(int model, int d, int m, int64_t B, int npts,
                                  const double* laws, int64_t law_stride,
                                  const REAL* t, int64_t t_stride,
                                  const REAL* H, int64_t H_stride,
                                  const REAL* F, int64_t F_stride,
                                  const REAL* Xacc, const REAL* Wacc, const REAL* Z,
                                  uint64_t seed, int64_t iter, uint32_t salt,
                                  const double* rho, REAL* Xo, REAL* Wo, double* ll_out,
                                  int nthreads) {
    int64_t nfail = 0;
    (void)nthreads;
#pragma omp parallel for schedule(static) reduction(+ : nfail) num_threads(nthreads)
    for (int64_t blk = 0; blk < B; ++blk) {
        const double* law = laws + blk * law_stride;
        const REAL* tb = t + blk * t_stride;
        const REAL* Hb = H + blk * H_stride;
        const REAL* Fb = F + blk * F_stride;
        const REAL* Xa = Xacc + (size_t)blk * npts * d;
        const REAL* Wa = Wacc + (size_t)blk * npts * m;
        REAL* Xp = Xo + (size_t)blk * npts * d;
        REAL* Wp = Wo + (size_t)blk * npts * m;
        double r = rho[blk];
        REAL rr = (REAL)r, sr = (REAL)sqrt(1.0 - r * r);
        /* pCN (increment form; W arrays hold increments) */
        for (int k = 0; k < m; ++k) Wp[k] = rr * Wa[k];
        REAL zb[ORC_NPB] = {0};
        for (int q = 0; q < npts - 1; ++q) {
            REAL sdt = SQRT(tb[q + 1] - tb[q]);
            for (int k = 0; k < m; ++k) {
                REAL z;
                if (Z) z = Z[((size_t)blk * (npts - 1) + q) * m + k];
                else {
                    uint32_t n = (uint32_t)(q * m + k);
                    if (n % ORC_NPB == 0)
                        SFX(orc_normal_block)(seed, n / ORC_NPB, (uint32_t)blk, (uint32_t)iter,
                                              salt << 1, zb);
                    z = zb[n % ORC_NPB];
                }
                REAL zi = sdt * z;
                Wp[(size_t)(q + 1) * m + k] = FMA(rr, Wa[(size_t)(q + 1) * m + k], sr * zi);
            }
        }
        /* solve + ll (obs term + segment) */
        REAL ll;
        int ok = SFX(orc_solve_segment)(model, d, m, law, npts, tb, Hb, Fb, Wp, Xa, Xp, &ll);
        REAL obs = SFX(orc_obs_term)(d, law, Hb, Fb, Xa);
        REAL tot = obs + ll;
        ll_out[blk] = ok ? (double)tot : -INFINITY;
        nfail += ok ? 0 : 1;
    }
    return (int)nfail;
}

#if IS_F64
/* ---- Philox4x32-10 (Salmon et al. 2011), shared by both precisions ---- */
void orc_philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}
#else
void orc_philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1);
#endif

/* ---- canonical transcendental kernels of the draws (identical to dmt_device.h) ---- */
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
static inline double rng_log(double u) {
    int e;
    double m = frexp(u, &e);
    const int lo = m < RNG_SQRT_HALF;
    m = lo ? m * 2.0 : m;
    e = lo ? e - 1 : e;
    const double f = m - 1.0;
    const double s = f / (2.0 + f);
    const double z = s * s;
    double p = RNG_P11;
    p = fma(p, z, RNG_P10); p = fma(p, z, RNG_P9); p = fma(p, z, RNG_P8);
    p = fma(p, z, RNG_P7); p = fma(p, z, RNG_P6); p = fma(p, z, RNG_P5);
    p = fma(p, z, RNG_P4); p = fma(p, z, RNG_P3); p = fma(p, z, RNG_P2);
    p = fma(p, z, RNG_P1);
    const double lm = fma(s, z * p, 2.0 * s);
    const double de = (double)e;
    return fma(de, RNG_LN2_HI, fma(de, RNG_LN2_LO, lm));
}
static inline float rng_logf(float u) {
    int e;
    float m = frexpf(u, &e);
    const int lo = m < RNGF_SQRT_HALF;
    m = lo ? m * 2.0f : m;
    e = lo ? e - 1 : e;
    const float f = m - 1.0f;
    const float s = f / (2.0f + f);
    const float z = s * s;
    float p = RNGF_P5;
    p = fmaf(p, z, RNGF_P4); p = fmaf(p, z, RNGF_P3); p = fmaf(p, z, RNGF_P2);
    p = fmaf(p, z, RNGF_P1);
    const float lm = fmaf(s, z * p, 2.0f * s);
    const float de = (float)e;
    return fmaf(de, RNGF_LN2_HI, fmaf(de, RNGF_LN2_LO, lm));
}
static inline void rng_sincospif(float x, float* sn, float* cs) {
    const float n = rintf(2.0f * x);
    const float r = fmaf(-0.5f, n, x);
    const float z = r * r;
    float sp = RNGF_S4;
    sp = fmaf(sp, z, RNGF_S3); sp = fmaf(sp, z, RNGF_S2); sp = fmaf(sp, z, RNGF_S1);
    sp = fmaf(sp, z, RNGF_S0);
    float cp = RNGF_C5;
    cp = fmaf(cp, z, RNGF_C4); cp = fmaf(cp, z, RNGF_C3); cp = fmaf(cp, z, RNGF_C2);
    cp = fmaf(cp, z, RNGF_C1);
    const float s0 = r * sp, c0 = fmaf(cp, z, 1.0f);
    const int q = (int)n & 3;
    *sn = q == 0 ? s0 : q == 1 ? c0 : q == 2 ? -s0 : -c0;
    *cs = q == 0 ? c0 : q == 1 ? -s0 : q == 2 ? -c0 : s0;
}

#include "bm_tables.inc"
#if IS_F64
/* fp64 Box–Muller kernels (libdmt dmt_device.h bm_log / bm_sincospi, DESIGN.md §3 RNG): the
 * tables and coefficients of scripts/gen_bm_tables.py, the same operations in the same order. */
static const double bm_log_tab[128][2] = DMT_BM_LOG_TABLE;
static const double bm_sc_tab[65][2] = DMT_BM_SC_TABLE;

static inline double bm_log(double u) {
    uint64_t b;
    memcpy(&b, &u, 8);
    const uint32_t hi = (uint32_t)(b >> 32);
    const int j = (int)((hi >> 13) & 0x7fu);
    const int e = (int)((hi >> 20) & 0x7ffu) - 1023 + (j >> 6);
    const uint64_t mb = (b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;
    double m;
    memcpy(&m, &mb, 8);
    const double r = fma(m, bm_log_tab[j][0], -1.0);
    const double r2 = r * r;
    double q = DMT_BM_Q6;
    q = fma(q, r, DMT_BM_Q5); q = fma(q, r, DMT_BM_Q4); q = fma(q, r, DMT_BM_Q3);
    q = fma(q, r, DMT_BM_Q2); q = fma(q, r, DMT_BM_Q1); q = fma(q, r, DMT_BM_Q0);
    const double lm = bm_log_tab[j][1] + fma(r2, q, r);
    const double de = (double)e;
    return fma(de, RNG_LN2_HI, fma(de, RNG_LN2_LO, lm));
}
static inline void bm_sincospi(double x, double* sn, double* cs) {
    const double n = rint(32.0 * x);
    const double r = fma(-0x1p-5, n, x);
    const double z = r * r;
    double sp = DMT_BM_S4;
    sp = fma(sp, z, DMT_BM_S3); sp = fma(sp, z, DMT_BM_S2); sp = fma(sp, z, DMT_BM_S1);
    sp = fma(sp, z, DMT_BM_S0);
    double cp = DMT_BM_C3;
    cp = fma(cp, z, DMT_BM_C2); cp = fma(cp, z, DMT_BM_C1); cp = fma(cp, z, DMT_BM_C0);
    const double sr = r * sp, cr = fma(cp, z, 1.0);
    const int k = (int)n;
    *sn = fma(bm_sc_tab[k][0], cr, bm_sc_tab[k][1] * sr);
    *cs = fma(bm_sc_tab[k][1], cr, -(bm_sc_tab[k][0] * sr));
}
#endif

/* Box–Muller normals from one Philox block (perf-mode stream), counter = (c0, c1, c2, c3),
 * key = seed.  fp64: one pair (z[0], z[1]) from 53-bit uniforms built of the whole block.
 * fp32: two pairs from 24-bit uniforms — (z[0], z[1]) of words (x, z), (z[2], z[3]) of words
 * (y, w) — so a block yields ORC_NPB = 4 normals. */
#if !IS_F64
static void orc_bm_f32(uint32_t a, uint32_t b, float* z0, float* z1) {
    float u1 = (float)((a >> 8) + 1u) * 0x1p-24f;
    float u2 = (float)(b >> 8) * 0x1p-24f;
    float rad = sqrtf(-2.0f * rng_logf(u1));
    float sn, cs;
    rng_sincospif(2.0f * u2, &sn, &cs);
    *z0 = rad * cs;
    *z1 = rad * sn;
}
#endif
void SFX(orc_normal_block)(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                           REAL* z) {
    uint32_t c[4] = {c0, c1, c2, c3};
    orc_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
#if IS_F64
    uint64_t k1 = ((uint64_t)(c[0] >> 5) << 26) | (c[1] >> 6);
    uint64_t k2 = ((uint64_t)(c[2] >> 5) << 26) | (c[3] >> 6);
    double u1 = (double)(k1 + 1) * 0x1p-53;
    double u2 = (double)k2 * 0x1p-53;
    double rad = sqrt(-2.0 * bm_log(u1));
    double sn, cs;
    bm_sincospi(2.0 * u2, &sn, &cs);
    z[0] = rad * cs;
    z[1] = rad * sn;
#else
    orc_bm_f32(c[0], c[2], &z[0], &z[1]);
    orc_bm_f32(c[1], c[3], &z[2], &z[3]);
#endif
}

/* The first pair of a block (fp64: the whole block) — the Random123-style known-answer
 * interface of tests/test_gpu_parity.py (dmt_debug_normals). */
void SFX(orc_normal_pair)(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                          REAL* z0, REAL* z1) {
    uint32_t c[4] = {c0, c1, c2, c3};
    orc_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
#if IS_F64
    uint64_t k1 = ((uint64_t)(c[0] >> 5) << 26) | (c[1] >> 6);
    uint64_t k2 = ((uint64_t)(c[2] >> 5) << 26) | (c[3] >> 6);
    double u1 = (double)(k1 + 1) * 0x1p-53;
    double u2 = (double)k2 * 0x1p-53;
    double rad = sqrt(-2.0 * bm_log(u1));
    double sn, cs;
    bm_sincospi(2.0 * u2, &sn, &cs);
    *z0 = rad * cs;
    *z1 = rad * sn;
#else
    float u1 = (float)((c[0] >> 8) + 1u) * 0x1p-24f;
    float u2 = (float)(c[2] >> 8) * 0x1p-24f;
    float rad = sqrtf(-2.0f * rng_logf(u1));
    float sn, cs;
    rng_sincospif(2.0f * u2, &sn, &cs);
    *z0 = rad * cs;
    *z1 = rad * sn;
#endif
}

#if IS_F64
/* Exp(1) draw for the MH test of a block (perf-mode stream); `blk` = global id of the
 * block's first segment. */
double orc_exp1(uint64_t seed, uint32_t blk, uint32_t iter, uint32_t salt) {
    uint32_t c[4] = {blk, 0xFFFFFFFFu, iter, (salt << 1) | 1u};
    orc_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    uint64_t k1 = ((uint64_t)(c[0] >> 5) << 26) | (c[1] >> 6);
    double u = (double)(k1 + 1) * 0x1p-53;
    return -rng_log(u);
}

/* orc_exp1 of blocks whose first segments are g0, g0 + 1, …, g0 + n - 1 (single-segment
 * blocks: the timed CPU baseline's MH decisions), out[n] */
void orc_exp1_range(uint64_t seed, uint32_t g0, int64_t n, uint32_t iter, uint32_t salt,
                    double* out) {
    for (int64_t i = 0; i < n; ++i) out[i] = orc_exp1(seed, g0 + (uint32_t)i, iter, salt);
}

/* raw Philox block, for bit-exact checks of the device generator */
void orc_philox_raw(uint64_t seed, const uint32_t* ctr, uint32_t* out) {
    uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
    orc_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    memcpy(out, c, sizeof c);
}
#endif

/* All perf-mode normals of one segment: Z[i*m + k] for steps i < nsteps (normal n is
 * entry n % ORC_NPB of block n / ORC_NPB, counter (n / ORC_NPB, g, iter, salt<<1)). */
void SFX(orc_normals_segment)(uint64_t seed, uint32_t g, uint32_t iter, uint32_t salt,
                              int nsteps, int m, REAL* Z) {
    int n = nsteps * m;
    for (int i = 0; i < n; i += ORC_NPB) {
        REAL zb[ORC_NPB];
        SFX(orc_normal_block)(seed, (uint32_t)(i / ORC_NPB), g, iter, salt << 1, zb);
        for (int e = 0; e < ORC_NPB && i + e < n; ++e) Z[i + e] = zb[e];
    }
}

#if IS_F64
/* ---- exact discrete backward filter of a linear auxiliary law (recompute_guiding_term!,
 * SURVEY.md A.5), restating the build's algorithm: Taylor series with scaling and squaring
 * for each step's transition (Phi, mu, K), transitions composed within 64-step chunks,
 * Gaussian update with Gauss-Jordan inverse; plain IEEE
 * operations in the same order, log|det| through rng_log.  Double only. */
typedef struct { int n; double a[9]; } fm_t;
static fm_t fm_zero(int n) { fm_t m; m.n = n; for (int i = 0; i < 9; ++i) m.a[i] = 0.0; return m; }
static fm_t fm_eye(int n) { fm_t m = fm_zero(n); for (int i = 0; i < n; ++i) m.a[i * n + i] = 1.0; return m; }
static fm_t fm_mul(const fm_t* A, const fm_t* B) {
    int n = A->n; fm_t C = fm_zero(n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int k = 0; k < n; ++k) s += A->a[i * n + k] * B->a[k * n + j];
            C.a[i * n + j] = s;
        }
    return C;
}
static fm_t fm_T(const fm_t* A) {
    int n = A->n; fm_t C = fm_zero(n);
    for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) C.a[i * n + j] = A->a[j * n + i];
    return C;
}
static fm_t fm_add(const fm_t* A, const fm_t* B) {
    fm_t C = *A; for (int i = 0; i < A->n * A->n; ++i) C.a[i] += B->a[i]; return C;
}
static void fm_vec(const fm_t* A, const double* x, double* y) {
    int n = A->n;
    for (int i = 0; i < n; ++i) { double s = 0.0; for (int k = 0; k < n; ++k) s += A->a[i * n + k] * x[k]; y[i] = s; }
}
static double fm_norm(const fm_t* A) {
    double s = 0.0; for (int i = 0; i < A->n * A->n; ++i) s = fmax(s, fabs(A->a[i])); return s * A->n;
}
static int fm_inv(const fm_t* A, fm_t* Inv, double* lad) {
    int n = A->n; double w[3][6];
    for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) { w[i][j] = A->a[i * n + j]; w[i][n + j] = (i == j) ? 1.0 : 0.0; }
    double detabs = 1.0;
    for (int c = 0; c < n; ++c) {
        int p = c;
        for (int i = c + 1; i < n; ++i) if (fabs(w[i][c]) > fabs(w[p][c])) p = i;
        if (w[p][c] == 0.0) return 0;
        if (p != c) for (int j = 0; j < 2 * n; ++j) { double t = w[p][j]; w[p][j] = w[c][j]; w[c][j] = t; }
        double piv = w[c][c];
        detabs *= fabs(piv);
        double rp = 1.0 / piv;
        for (int j = 0; j < 2 * n; ++j) w[c][j] *= rp;
        for (int i = 0; i < n; ++i) if (i != c) {
            double f = w[i][c];
            if (f != 0.0) for (int j = 0; j < 2 * n; ++j) w[i][j] -= f * w[c][j];
        }
    }
    *Inv = fm_zero(n);
    for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) Inv->a[i * n + j] = w[i][n + j];
    *lad = rng_log(detabs);
    return 1;
}
static void fm_transition(const fm_t* B, const double* beta, const fm_t* At, double h,
                          fm_t* Phi, double* mu, fm_t* K) {
    int n = B->n, sq = 0;
    double hs = h;
    double nb = fm_norm(B);
    while (nb * hs > 0.25 && sq < 40) { hs *= 0.5; ++sq; }
    fm_t A = *B;
    for (int i = 0; i < n * n; ++i) A.a[i] *= hs;
    *Phi = fm_eye(n);
    fm_t term = fm_eye(n), S1 = fm_eye(n), Lk = *At;
    *K = fm_zero(n);
    for (int i = 0; i < n * n; ++i) K->a[i] = hs * Lk.a[i];
    fm_t BT = fm_T(B);
    double rk = 1.0;
    for (int k = 1; k <= 30; ++k) {
        double rk1 = 1.0 / (double)(k + 1);
        term = fm_mul(&term, &A);
        for (int i = 0; i < n * n; ++i) term.a[i] *= rk;
        *Phi = fm_add(Phi, &term);
        fm_t t2 = term;
        for (int i = 0; i < n * n; ++i) t2.a[i] *= rk1;
        S1 = fm_add(&S1, &t2);
        fm_t l1 = fm_mul(B, &Lk), l2 = fm_mul(&Lk, &BT);
        fm_t nl = fm_add(&l1, &l2);
        double c0 = hs * rk, c1 = hs * rk1;
        for (int i = 0; i < n * n; ++i) nl.a[i] *= c0;
        Lk = nl;
        for (int i = 0; i < n * n; ++i) K->a[i] += Lk.a[i] * c1;
        if (fm_norm(&term) < 1e-18 && fm_norm(&Lk) * hs < 1e-18 * (1.0 + fm_norm(K))) break;
        rk = rk1;
    }
    double sb[3];
    fm_vec(&S1, beta, sb);
    for (int i = 0; i < n; ++i) mu[i] = hs * sb[i];
    for (int s = 0; s < sq; ++s) {
        double m2[3];
        fm_vec(Phi, mu, m2);
        for (int i = 0; i < n; ++i) mu[i] = m2[i] + mu[i];
        fm_t PK = fm_mul(Phi, K), PT = fm_T(Phi), PKP = fm_mul(&PK, &PT);
        *K = fm_add(&PKP, K);
        *Phi = fm_mul(Phi, Phi);
    }
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) { double v = 0.5 * (K->a[i * n + j] + K->a[j * n + i]); K->a[i * n + j] = v; K->a[j * n + i] = v; }
}
typedef struct { fm_t Phi; double mu[3]; fm_t K; } ftr_t;

/* transition over f then s: (Phi_s Phi_f, Phi_s mu_f + mu_s, sym(Phi_s K_f Phi_s' + K_s)) */
static ftr_t ftr_compose(const ftr_t* f, const ftr_t* s) {
    int n = f->Phi.n;
    ftr_t r;
    r.Phi = fm_mul(&s->Phi, &f->Phi);
    double m[3];
    fm_vec(&s->Phi, f->mu, m);
    for (int i = 0; i < n; ++i) r.mu[i] = m[i] + s->mu[i];
    fm_t PK = fm_mul(&s->Phi, &f->K), PT = fm_T(&s->Phi), PKP = fm_mul(&PK, &PT);
    r.K = fm_add(&PKP, &s->K);
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) { double v = 0.5 * (r.K.a[i * n + j] + r.K.a[j * n + i]); r.K.a[i * n + j] = v; r.K.a[j * n + i] = v; }
    return r;
}

/* (H, F, c) at the start of transition q from the values at its end (Gaussian integral) */
static int fm_combine(const ftr_t* q, fm_t* Hc, double* Fc, double* cc) {
    int d = q->Phi.n;
    const fm_t* Phi = &q->Phi;
    const fm_t* K = &q->K;
    const double* mu = q->mu;
    fm_t HK = fm_mul(Hc, K), I = fm_eye(d);
    fm_t IHK = fm_add(&I, &HK);
    fm_t S; double lad;
    if (!fm_inv(&IHK, &S, &lad)) return 0;
    fm_t Hh = fm_mul(&S, Hc);
    for (int p = 0; p < d; ++p)
        for (int r = p + 1; r < d; ++r) { double v = 0.5 * (Hh.a[p * d + r] + Hh.a[r * d + p]); Hh.a[p * d + r] = v; Hh.a[r * d + p] = v; }
    double Fh[3], KF[3];
    fm_vec(&S, Fc, Fh);
    fm_vec(K, Fc, KF);
    double fkf = 0.0;
    for (int p = 0; p < d; ++p) fkf += Fh[p] * KF[p];
    double ch = *cc + 0.5 * lad - 0.5 * fkf;
    double Hmu[3], g[3], Fn[3];
    fm_vec(&Hh, mu, Hmu);
    for (int p = 0; p < d; ++p) g[p] = Fh[p] - Hmu[p];
    fm_t PhT = fm_T(Phi);
    fm_vec(&PhT, g, Fn);
    fm_t t1 = fm_mul(&PhT, &Hh);
    fm_t Hn = fm_mul(&t1, Phi);
    for (int p = 0; p < d; ++p)
        for (int r = p + 1; r < d; ++r) { double v = 0.5 * (Hn.a[p * d + r] + Hn.a[r * d + p]); Hn.a[p * d + r] = v; Hn.a[r * d + p] = v; }
    double fmu = 0.0, muHmu = 0.0;
    for (int p = 0; p < d; ++p) { fmu += Fh[p] * mu[p]; muHmu += mu[p] * Hmu[p]; }
    *cc = ch - fmu + 0.5 * muHmu;
    *Hc = Hn;
    for (int p = 0; p < d; ++p) Fc[p] = Fn[p];
    return 1;
}

/* Backward filter over one segment's grid t[npts] from the terminal information (HT packed,
 * FT, cT): H[npts][hp] packed, F[npts][d], c[npts] (double).  Returns 0 if singular.
 * Canonical chunked form (guiding term): chunks of FILT_CHUNK steps counted from the
 * segment end; per chunk an inclusive Kogge-Stone suffix scan of the step transitions
 * (stage k: Q_l <- compose(Q_l, Q_{l+k}) if l + k < cnt, previous-stage values), then every
 * point of the chunk by one combine from the chunk end's (H, F, c). */
#define FILT_CHUNK 64
/* aux: NULL (B~ = Bt, beta~ = beta on every step) or [npts][ncols] per-point coefficients of
 * a time-dependent auxiliary law — B~, beta~ (ncols = d*d + d; a~ = at) or B~, beta~, a~
 * packed (ncols = d*d + d + hp; at unused); step i's exact transition takes the trapezoidal
 * averages (row i + row i+1) * 0.5 — a second-order scheme for the filter ODEs (libdmt
 * filt_aux_step, dmt_guiding_linear_td(a)). */
static int backward_filter(int d, const double* Bt, const double* beta, const double* aux,
                           int ncols, const double* at, int npts, const double* t,
                           const double* HT, const double* FT, double cT, double* H, double* F,
                           double* c) {
    int hp = d * (d + 1) / 2;
    const int tda = aux && ncols == d * d + d + hp;
    fm_t B = fm_zero(d), A = fm_zero(d), Hc = fm_zero(d);
    if (!aux) for (int i = 0; i < d * d; ++i) B.a[i] = Bt[i];
    for (int i = 0; i < d; ++i)
        for (int j = 0; j < d; ++j) {
            A.a[i * d + j] = tda ? 0.0 : at[pidx(d, i, j)];
            Hc.a[i * d + j] = HT[pidx(d, i, j)];
        }
    double Fc[3] = {0, 0, 0}, cc = cT;
    for (int i = 0; i < d; ++i) Fc[i] = FT[i];
#define FILT_STORE(i, Hm, Fv, cv)                                                              \
    do {                                                                                       \
        for (int p = 0; p < d; ++p)                                                            \
            for (int q = p; q < d; ++q) H[(size_t)(i) * hp + pidx(d, p, q)] = (Hm).a[p * d + q]; \
        for (int p = 0; p < d; ++p) F[(size_t)(i) * d + p] = (Fv)[p];                          \
        c[i] = (cv);                                                                           \
    } while (0)
    FILT_STORE(npts - 1, Hc, Fc, cc);
    ftr_t Q[FILT_CHUNK], Qn[FILT_CHUNK];
    for (int hi = npts - 1; hi > 0; hi -= FILT_CHUNK) {
        int lo = hi > FILT_CHUNK ? hi - FILT_CHUNK : 0, cnt = hi - lo;
        for (int l = 0; l < cnt; ++l) {
            const double* bl = beta;
            double bavg[3];
            if (aux) {  /* step lo + l: trapezoidal average of rows lo + l and lo + l + 1 */
                const double* r0 = aux + (size_t)(lo + l) * ncols;
                const double* r1 = r0 + ncols;
                for (int i = 0; i < d * d; ++i) B.a[i] = (r0[i] + r1[i]) * 0.5;
                for (int i = 0; i < d; ++i) bavg[i] = (r0[d * d + i] + r1[d * d + i]) * 0.5;
                bl = bavg;
                if (tda)
                    for (int i = 0; i < d; ++i)
                        for (int j = 0; j < d; ++j) {
                            const int e = d * d + d + pidx(d, i, j);
                            A.a[i * d + j] = (r0[e] + r1[e]) * 0.5;
                        }
            }
            fm_transition(&B, bl, &A, t[lo + l + 1] - t[lo + l], &Q[l].Phi, Q[l].mu, &Q[l].K);
        }
        for (int k = 1; k < FILT_CHUNK; k *= 2) {
            for (int l = 0; l < cnt; ++l) Qn[l] = (l + k < cnt) ? ftr_compose(&Q[l], &Q[l + k]) : Q[l];
            for (int l = 0; l < cnt; ++l) Q[l] = Qn[l];
        }
        fm_t H0 = Hc;
        double F0[3] = {Fc[0], Fc[1], Fc[2]}, c0 = cc;
        for (int l = cnt - 1; l >= 0; --l) {
            fm_t Hl = H0;
            double Fl[3] = {F0[0], F0[1], F0[2]}, cl = c0;
            if (!fm_combine(&Q[l], &Hl, Fl, &cl)) return 0;
            FILT_STORE(lo + l, Hl, Fl, cl);
            if (l == 0) { Hc = Hl; Fc[0] = Fl[0]; Fc[1] = Fl[1]; Fc[2] = Fl[2]; cc = cl; }
        }
    }
#undef FILT_STORE
    return 1;
}
int orc_backward_filter_segment(int d, const double* Bt, const double* beta, const double* at,
                                int npts, const double* t, const double* HT, const double* FT,
                                double cT, double* H, double* F, double* c) {
    return backward_filter(d, Bt, beta, 0, 0, at, npts, t, HT, FT, cT, H, F, c);
}
int orc_backward_filter_segment_td(int d, const double* aux, const double* at, int npts,
                                   const double* t, const double* HT, const double* FT,
                                   double cT, double* H, double* F, double* c) {
    return backward_filter(d, 0, 0, aux, d * d + d, at, npts, t, HT, FT, cT, H, F, c);
}

int orc_backward_filter_segment_tda(int d, const double* aux, int npts, const double* t,
                                    const double* HT, const double* FT, double cT, double* H,
                                    double* F, double* c) {
    return backward_filter(d, 0, 0, aux, d * d + d + d * (d + 1) / 2, 0, npts, t, HT, FT, cT,
                           H, F, c);
}
/* the canonical log kernel, exposed for the Python container restatement */
double orc_rng_log(double u) { return rng_log(u); }
double orc_bm_log(double u) { return bm_log(u); }
#endif
