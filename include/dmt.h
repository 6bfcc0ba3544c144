/*
 * dmt.h — C-ABI of libdmt, the MI355X-native guided-bridge imputation engine.
 *
 * This is the drop-in boundary for the hot path of DiffusionMCMCTools.jl
 * (the reference).  The reference's API is Julia multiple dispatch on
 * SamplingUnit / SamplingPair / BiBlock / BlockCollection / BlockEnsemble
 * (exports at /root/reference/src/DiffusionMCMCTools.jl:28-60).  A Julia shim
 * (diffusionmcmctools.jl_amd/julia/DiffusionMCMCToolsAMD.jl, see
 * INTEGRATION.md) keeps those method names and `ccall`s the entry points below
 * ONCE PER ENSEMBLE OPERATION: a BiBlock is a 1-block range of a layout, a
 * BlockCollection the blocks of one recording, a BlockEnsemble all blocks.
 *
 * Conventions (mirroring the reference):
 *  - every call returns dmt_status (0 = OK); numerical failure is NOT an
 *    error: it is reported per block as success=0 and ll = -Inf, exactly as
 *    upstream GP.rand!/solve_and_ll! return (false, -Inf)
 *    (src/biblock.jl:81-86, src/block.jl:162-169,180-181);
 *  - host pointers are borrowed for the duration of the call only;
 *  - host array layout = the reference's in-memory layout: a segment's path
 *    is Julia Vector{SVector{d,Float64}} == C double[npts][d]; segments are
 *    concatenated recording-major (recording 0 seg 0, seg 1, …, recording 1 …);
 *    Julia Bool == uint8_t, Int == int64_t;
 *  - "mcmciter" is the reference's 1-based MCMC iteration index;
 *  - a handle is not re-entrant; calls are ordered on the handle's HIP
 *    stream; only fetch/download/sync calls block the host;
 *  - dmt_last_error() returns a thread-local message for the last failure.
 *
 * fp32 ensembles (DMT_F32) still take double host buffers; values are
 * rounded to float on upload.
 */
#ifndef DMT_H
#define DMT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t dmt_status;
typedef struct dmt_ens dmt_ens;

enum {
    DMT_OK = 0,
    DMT_ERR_INVALID = 1, /* bad argument / shape */
    DMT_ERR_HIP = 2,     /* HIP runtime failure (no device, launch failure) */
    DMT_ERR_OOM = 3,
    DMT_ERR_STATE = 4,   /* call not valid in the current state (e.g. law not uploaded) */
    DMT_ERR_COMM = 5     /* RCCL failure */
};

/* models (DiffusionDefinition.jl models used by the reference's tutorials and configs) */
enum { DMT_MODEL_OU = 0, DMT_MODEL_FHN = 1, DMT_MODEL_LORENZ = 2 };
enum { DMT_F64 = 0, DMT_F32 = 1 };
/* thread mapping of the recursion kernels of non-linear models (FHN, Lorenz): AUTO picks
 * WAVE (a 2-wave workgroup per block, for small ensembles, latency-bound) or LANE (one lane
 * per block, for large ensembles, bandwidth-bound); both give bit-identical results.
 * Linear-drift models (OU) ignore it: their recursion is a parallel affine scan, one
 * workgroup per block. */
enum { DMT_MAP_AUTO = 0, DMT_MAP_LANE = 1, DMT_MAP_WAVE = 2 };
/* units of a SamplingPair: u (accepted) and u° (proposal), src/sampling_pair.jl:36-55 */
enum { DMT_U = 0, DMT_UPROP = 1 };
/* law kinds of a SamplingUnit: PP (regular) and PPb (blocking), src/sampling_unit.jl:48-53 */
enum { DMT_LAW_PP = 0, DMT_LAW_PPB = 1 };
/* swap masks, src/biblock.jl:148-209 */
enum { DMT_SWAP_XX = 1, DMT_SWAP_WW = 2, DMT_SWAP_PP = 4, DMT_SWAP_LL = 8 };
/* per-block state arrays, src/block.jl:57-58, src/biblock.jl:233-234 */
enum {
    DMT_BLK_LL = 0,        /* b.ll            double[nblocks] */
    DMT_BLK_LLPROP = 1,    /* b°.ll           double[nblocks] */
    DMT_BLK_LL_HIST = 2,   /* b.ll_history    double[hist_len][nblocks] (iteration-major) */
    DMT_BLK_LLPROP_HIST = 3,
    DMT_BLK_ACC_HIST = 4   /* accpt_history   uint8[hist_len][nblocks] */
};
/* kernels whose device time can be queried (dmt_get_timing) */
enum { DMT_K_DRAW = 0, DMT_K_ACCEPT = 1, DMT_K_PATHLL = 2, DMT_K_RECOMPUTE = 3,
       DMT_K_REDUCE = 4, DMT_K_COUNT = 5 };

/*
 * Law record: one per segment per (unit, kind), DMT_LAW_STRIDE doubles.
 * It carries the target-law parameters θ and the auxiliary (linear) law used
 * by the Girsanov weight.  Offsets:
 *   [0,14)  theta  model parameters (at most 14: slot 14 is gstale; Law::load asserts it)
 *             OU:     Theta (d×d row-major) at 0, mu at 9
 *             FHN:    1/eps, s, gamma, beta, then the raw eps, σ at 4, 5
 *                     (σ also goes in sigma)
 *             Lorenz: s, r, beta
 *   14      gstale 1.0: u°'s guiding term no longer matches the record's auxiliary law
 *                  (set_proposal_law with critical_change = false; see DMT_LAW_GSTALE)
 *   15      auxtd  1.0: the auxiliary drift varies within the segment — step i uses
 *                  B̃(t_i), β̃(t_i) of the per-point table of dmt_upload_aux (Bt/beta unused)
 *   [16,25) sigma  d×m row-major (constant diffusion coefficient)
 *   [25,31) a      packed upper-triangular σσᵀ (row-major upper: 00,01,(02),11,(12),22)
 *   [31,40) Bt     auxiliary drift matrix B̃ (d×d row-major)
 *   [40,43) beta   auxiliary drift offset β̃
 *   [43,49) da     packed a − ã (used only when trace != 0)
 *   49      c0     c(t0) of the segment's guiding term (for loglikhd_obs)
 *   50      trace  1.0 if a ≠ ã (adds −½ tr[(a−ã)(H−rrᵀ)] to G)
 *   [51,60) siginv σ⁻¹ (d×d row-major) when d = m (find_W_for_X!; unused for FHN, whose
 *                  single noise enters coordinate 1)
 *   [60,63) anchor the point the auxiliary law is linearised at (FHN: the observed y_T at 60;
 *                  Lorenz: the observed state)
 *   63      auxlin 1.0 if B̃, β̃ are the model's linearisation at `anchor` (re-derived by
 *                  dmt_set_proposal_law when θ changes); 0.0 if the auxiliary law is fixed
 */
#define DMT_LAW_STRIDE 64
#define DMT_LAW_THETA 0
#define DMT_LAW_SIGMA 16
#define DMT_LAW_A 25
#define DMT_LAW_BT 31
#define DMT_LAW_BETA 40
#define DMT_LAW_DA 43
#define DMT_LAW_C0 49
#define DMT_LAW_TRACE 50
#define DMT_LAW_SIGINV 51
#define DMT_LAW_ANCHOR 60
#define DMT_LAW_AUXLIN 63
#define DMT_LAW_AUXTD 15
/* 1.0: u°'s guiding term of this record is stale — set_proposal_law!(…, false) left it although
 * the record's auxiliary law changed; the default (critical_change omitted) treats the record as
 * critical until the guiding term is recomputed.  Kept by libdmt; uploads write 0. */
#define DMT_LAW_GSTALE 14

/* Parameter names of dmt_set_proposal_law (DiffusionDefinition's parameter order):
 *   FHN    (eps, s, gamma, beta, sigma), docs/src/tutorials/preamble.md:77
 *   Lorenz (s, r, beta)
 *   OU     Theta[i][j] = i*d + j, mu[i] = d*d + i  (the auxiliary law stays fixed) */
enum { DMT_PAR_FHN_EPS = 0, DMT_PAR_FHN_S = 1, DMT_PAR_FHN_GAMMA = 2, DMT_PAR_FHN_BETA = 3,
       DMT_PAR_FHN_SIGMA = 4 };
enum { DMT_PAR_LORENZ_S = 0, DMT_PAR_LORENZ_R = 1, DMT_PAR_LORENZ_BETA = 2 };

typedef struct {
    int32_t model;      /* DMT_MODEL_* */
    int32_t precision;  /* DMT_F64 / DMT_F32 */
    int32_t d;          /* state dimension (OU: 1..3, FHN: 2, Lorenz: 3) */
    int32_t m;          /* noise dimension (OU: 1..3, FHN: 1, Lorenz: 3) */
} dmt_model;

typedef struct {
    int64_t n_recordings;        /* R */
    const int32_t* n_segments;   /* [R] segments per recording (= number of observations) */
    const int32_t* n_points;     /* [G] grid points per segment (N_g + 1), recording-major */
} dmt_structure;

typedef struct {
    uint64_t seed;               /* key of the device Philox4x32-10 streams (perf mode) */
    int32_t device;              /* HIP device ordinal */
    int32_t grid_shared;         /* 1: every recording has the same segment structure and time grid;
                                    dmt_upload_grid then takes ONE recording's grid */
    int32_t mapping;             /* DMT_MAP_*: thread mapping of the Euler recursion */
} dmt_config;

/* ---------------- device random streams (perf mode) ----------------
 * Draw calls take a stream key (iter, salt).  An explicit key (salt < DMT_SALT_LIMIT) selects
 * a reproducible stream: normals are keyed by (seed, iter, salt, global segment, step), Exp(1)
 * variables by (seed, mcmciter, salt, global id of the block's first segment).
 * salt = DMT_RNG_AUTO draws from the handle's own stream counter instead, which is how the
 * reference consumes randomness: rand! and rand(Exponential(1.0)) read the global RNG and take
 * no key (src/biblock.jl:94-99,122, src/sampling_unit.jl:119).  Under DMT_RNG_AUTO
 *   - dmt_draw_proposal, dmt_draw_unit and dmt_mcmc_step take the next counter value k
 *     (their `iter` argument is ignored);
 *   - dmt_accept_reject takes the k of the auto draw it follows, once; otherwise the next k
 *     (`mcmciter` still indexes the histories);
 *   - dmt_mcmc_run takes n_iter consecutive values, one per iteration, for its draw and its
 *     decision (so a run equals the loop of auto draw + auto accept calls);
 * so successive calls never reuse normals or Exp(1) variables, and two blockings drawn in one
 * iteration get independent streams.  Counter value k maps to the key
 * (iter = k mod 2^32, salt = DMT_SALT_LIMIT + k div 2^32): auto streams never meet explicit
 * ones.  The counter starts at 0 on dmt_create; dmt_rng_counter / dmt_set_rng_counter read and
 * restore it (checkpoint / resume). */
#define DMT_RNG_AUTO 0xFFFFFFFFu
#define DMT_SALT_LIMIT 0x40000000u

/* ---------------- lifetime (SamplingEnsemble / SamplingPair containers) ---------------- */

/* Allocates the device containers of a SamplingEnsemble (src/sampling_ensemble.jl:17-41):
 * paths XX/WW of u and u° (src/sampling_unit.jl:48-53, src/sampling_pair.jl:51). */
dmt_status dmt_create(dmt_ens** h, const dmt_model* model, const dmt_structure* st,
                      const dmt_config* cfg);
dmt_status dmt_destroy(dmt_ens* h);

/* Time grids tts (ObservationSchemes setup_time_grids, src/sampling_unit.jl:55): t[P] or,
 * with grid_shared, t[points of recording 0]. */
dmt_status dmt_upload_grid(dmt_ens* h, const double* t);

/* Guiding-term tables of the laws u.PP/u°.PP (kind PP) or u.PPb/u°.PPb (kind PPB),
 * built upstream by build_guid_prop / guid_prop_for_blocking (src/sampling_unit.jl:60-66)
 * and recompute_guiding_term! (src/block.jl:102-110).
 *   H[P][d(d+1)/2] packed (or, with H_shared, H[points of recording 0][…] shared by all),
 *   F[P][d], laws[G][DMT_LAW_STRIDE].  Any of H/F/laws may be NULL to keep the previous one. */
dmt_status dmt_upload_law(dmt_ens* h, int32_t unit, int32_t kind, const double* H,
                          int32_t H_shared, const double* F, const double* laws);

/* Time-dependent linear auxiliary laws within a segment: the reference takes any linear
 * auxiliary law of GuidedProposals (aux_laws, src/sampling_unit.jl:55-66), whose B̃(t), β̃(t)
 * may vary in t.  aux[P][d·d + d] holds B̃(t_i) (row-major) then β̃(t_i) at every grid point
 * of every segment (layout of dmt_upload_law's F) for the laws of kind PP or PPB, u and u° alike
 * (the auxiliary law does not depend on θ).  A segment whose law record has DMT_LAW_AUXTD = 1.0
 * takes step i's auxiliary drift B̃(t_i)x + β̃(t_i) (left point) in the Girsanov term G and the
 * trapezoidal average of B̃, β̃ over [t_i, t_{i+1}] in the backward filter's step transition
 * (dmt_recompute_guiding_term); ã stays the record's (σ̃ constant per segment).  aux = NULL
 * removes the table.  Every model: a linear drift (OU) takes the table in G and the filter only
 * (its recursion is the target law's), on the scan kernels (the register-resident kernels are not
 * used while a table is present). */
dmt_status dmt_upload_aux(dmt_ens* h, int32_t kind, const double* aux);
/* The same with a time-dependent ã(t) = σ̃σ̃ᵀ(t) too: aux[P][ncols], ncols = d·d + d (as
 * dmt_upload_aux) or d·d + d + d(d+1)/2 — B̃, β̃ and ã packed (upper triangle, row-major) per
 * point.  A segment whose law record has DMT_LAW_AUXTD = 2 takes step i's a − ã(t_i) in G's trace
 * term (a − ã computed in the working precision; the term is taken whatever the record's trace
 * flag) and the trapezoidal average of ã over [t_i, t_i+1] in the filter's step transition
 * (DESIGN.md §7); DMT_LAW_AUXTD = 1 keeps the record's ã. */
dmt_status dmt_upload_aux_a(dmt_ens* h, int32_t kind, const double* aux, int32_t ncols);

/* Paths of unit u / u°: X[P][d], W[P][m]; NULL keeps the current one.  Used by
 * init_paths! (src/sampling_unit.jl:83-87) and find_W_for_X! (src/block.jl:118-131). */
dmt_status dmt_set_paths(dmt_ens* h, int32_t unit, const double* X, const double* W);

/* Download the guiding tables and law records of u.PP/u°.PP (kind PP) or PPb, resolving
 * swap_PP!: H[P][hp] (or H[points of recording 0][hp] when shared), F[P][d], laws[G][64];
 * any pointer may be NULL. */
dmt_status dmt_download_law(dmt_ens* h, int32_t unit, int32_t kind, double* H, double* F,
                            double* laws);

/* Download XX (what=0) / WW (what=1, the cumulative Wiener path) of a unit, resolving all
 * swaps, reference layout; what=2 (DMT_PATH_DW): the Wiener increments exactly as the device
 * holds them (row 0 = W(t0), row i+1 = ΔW_i; cumulating in the working precision and
 * differencing back is not exact in fp32). */
#define DMT_PATH_DW 2
dmt_status dmt_download_paths(dmt_ens* h, int32_t unit, int32_t what, double* out);

/* draw_proposal_path!(u::SamplingUnit) (src/sampling_unit.jl:118-120): rand! with no pCN
 * (ρ = 0) under u.PP, in place, for recordings [r0, r1).  Z: [steps][m] for all segments
 * in reference order (NULL → device Philox stream keyed by (seed, iter, salt)).
 * ll_out (nullable, double[r1-r0]) / success_out (nullable). */
dmt_status dmt_draw_unit(dmt_ens* h, int32_t unit, int64_t r0, int64_t r1, const double* Z,
                         int64_t iter, uint32_t salt, double* ll_out, uint8_t* success_out);

/* ---------------- block layouts (BiBlock / BlockCollection / BlockEnsemble views) ---------------- */

/* Registers one layout of blocks over the ensemble (src/block_ensemble.jl:20-33,
 * src/block_collection.jl:20-30, src/biblock.jl:49-62).  Blocks are listed
 * recording-major; block i covers segments [seg_first[i], seg_last[i]] (0-based, local to
 * its recording) with terminal flag last[i] (the L type parameter), pCN memory rho[i].
 * hist_len = ll_hist_len (0 = no histories).  Non-terminal blocks need ≥ 2 segments
 * (the reference indexes PP[1] of the block, src/block.jl:66,178). */
dmt_status dmt_create_layout(dmt_ens* h, const int32_t* n_blocks /*[R]*/,
                             const int32_t* seg_first, const int32_t* seg_last,
                             const uint8_t* last, const double* rho, int64_t hist_len,
                             int32_t* layout_id);
dmt_status dmt_layout_size(dmt_ens* h, int32_t layout, int64_t* n_blocks);

/* draw_proposal_path! for blocks [b0, b1) of a layout (src/biblock.jl:78-106,
 * src/block_collection.jl:46, src/block_ensemble.jl:50).  pCN under the accepted law
 * b.PP (+ b.P_last), proposal written to u°; ll° stored in the layout.
 * Z: [steps][m] for all segments (parity mode) or NULL (device Philox, keyed by
 * (seed, iter, salt, segment, step)).  success_out: uint8[b1-b0], nullable. */
dmt_status dmt_draw_proposal(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                             const double* Z, int64_t iter, uint32_t salt,
                             uint8_t* success_out);

/* Success flags of the last draw over blocks [b0, b1) (the value draw_proposal_path! returns,
 * src/biblock.jl:78-92): a caller that passes success_out = NULL to dmt_draw_proposal reads them
 * here, when (and only if) it needs them.
 *
 * Deferred draws.  dmt_draw_proposal with Z = NULL and success_out = NULL over a layout of
 * single-segment linear-drift blocks (the register-resident kernel's range, e.g. C2) only
 * records the draw and its stream key.  The dmt_accept_reject that follows on the same range,
 * E = NULL, acc_out = NULL and the same stream key (the auto key of the draw, or an explicit key
 * equal to the draw's), runs draw, decision, histories and the fetch_ll tree as ONE kernel
 * launch; the next dmt_fetch_ll / dmt_fetch_ll_local of that range (mcmciter 0 or the same)
 * returns the tree's values without a launch.  Any other call first launches the deferred draw,
 * so every result is exactly that of launching each call at once (DMT_DEFER=0).
 *
 * Resident service (DMT_SERVICE, default on; one process, no communicator, the launch's
 * workgroups co-resident).  Consecutive fused iterations of one range — stream keys and
 * mcmciters advancing by one — run in ONE launch of the register-resident kernel that stays on
 * the device between the caller's calls: it computes each iteration ahead, publishes it when
 * dmt_accept_reject posts it (a word in pinned memory), and sends the iteration's fetch_ll sums
 * to pinned memory, which dmt_fetch_ll folds in the canonical order.  Results are bit-identical
 * to the one-launch-per-iteration path (DMT_SERVICE=0).  Any other libdmt call on the handle
 * stops the launch first (and waits for it); a launch with no post for DMT_SVC_IDLE_MS (2 ms)
 * leaves by itself and is launched again when the next iteration is posted.  While it waits,
 * the launch occupies the device: call dmt_sync (or any libdmt call) before a device-wide
 * synchronisation from outside libdmt, or that synchronisation waits up to DMT_SVC_IDLE_MS. */
dmt_status dmt_draw_success(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                            uint8_t* success_out);

/* The resident service's switch and idle window, per handle (the environment's DMT_SERVICE /
 * DMT_SVC_IDLE_MS give the defaults).  enable = 0, or idle_ms = 0, turns it off: every fused
 * iteration is its own launch and no launch waits on the device between calls (for callers
 * that share the device with other work or synchronise it from outside libdmt).  A running
 * service is stopped first.  The service also turns itself off for the handle when launches
 * keep leaving idle before their iteration is posted — more than one relaunch per four posts
 * after 16 posts, e.g. because other work holds CUs the grid needs (co-residency is checked
 * on an empty device only); dmt_service_stats reports it. */
dmt_status dmt_set_service(dmt_ens* h, int32_t enable, double idle_ms);
/* stats[5]: launches started, relaunches, iterations posted, host waits, 1 if the service
 * turned itself off (see above). */
dmt_status dmt_service_stats(dmt_ens* h, uint64_t* stats);

/* accept_reject_proposal_path!(·, mcmciter) (src/biblock.jl:121-127): E > -(ll° - ll),
 * swap XX/WW, set_accepted!, save_ll! (both), swap ll.  E: double[b1-b0] (parity) or NULL
 * (device Exp(1) stream keyed by (seed, mcmciter, salt, global id of the block's first
 * segment)).  acc_out nullable. */
dmt_status dmt_accept_reject(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                             const double* E, int64_t mcmciter, uint32_t salt,
                             uint8_t* acc_out);

/* loglikhd!(b) / loglikhd°!(b) (src/block.jl:138-152, src/biblock.jl:240,248). */
dmt_status dmt_loglikhd(dmt_ens* h, int32_t layout, int32_t unit, int64_t b0, int64_t b1);

/* recompute_path!(b°, b.WW; skip) (src/block.jl:159-187) as called by set_proposal_law!
 * (src/biblock.jl:343): re-solve u° under u°.PP with the accepted Wiener paths. */
dmt_status dmt_recompute_path(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                              int32_t skip, uint8_t* success_out);

/* find_W_for_X!(b) (src/block.jl:118-131, BiBlock src/biblock.jl:300, broadcasts
 * src/block_collection.jl:229, src/block_ensemble.jl:212): the Wiener increments that
 * reproduce the accepted path u.XX under the accepted laws u.PP (+ P_last), written to
 * u.WW in place — DD.invsolve! restated:
 *   ΔW_i = σ⁻¹ (x_{i+1} − x_i − b°(t_i, x_i)·dt_i)   (FHN: on coordinate 1, / σ_1),
 * W(t0) = 0.  Parallel in time. */
dmt_status dmt_find_W_for_X(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1);

/* ---- guiding terms on the device ----
 * Information of the (real) observation at the end of every segment, packed like H:
 * Hobs[G][d(d+1)/2] = LᵀΣ⁻¹L, Fobs[G][d] = LᵀΣ⁻¹v, cobs[G] = ½vᵀΣ⁻¹v + (k/2)log2π + ½log|Σ|
 * (SURVEY.md A.5), and the variance of the artificial exact end observation of blocking laws
 * (artificial_noise, src/sampling_unit.jl:57, default 1e-11). */
dmt_status dmt_upload_obs(dmt_ens* h, const double* Hobs, const double* Fobs, const double* cobs,
                          double artificial_noise);
/* GP.set_obs!(bb) (src/biblock.jl:273-280, broadcasts src/block_collection.jl:199,
 * src/block_ensemble.jl:186): freeze the end point of each non-terminal block's accepted
 * path as the artificial observation of its P_last law (both units; terminal blocks: no-op). */
dmt_status dmt_set_obs(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1);
/* GP.recompute_guiding_term!(b) for the blocks' laws of `unit` (u: bb.b, u°: bb.b°)
 * (src/block.jl:102-110, src/biblock.jl:288-291, src/block_collection.jl:208-221): exact
 * discrete backward filter of the linear auxiliary law (law record B̃, β̃, ã) over each segment,
 * backward from the block end — P_last: observation + artificial observation; other segments:
 * observation + the guiding term at the start of the next segment.  Writes H, F at every point
 * and c(t0) into the law record.  Needs per-segment (not shared) H tables. */
dmt_status dmt_recompute_guiding_term(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                                      int32_t unit);

/* set_proposal_law!(bb, θ°, pnames; skip) (src/biblock.jl:334-345, broadcasts
 * src/block_collection.jl, src/block_ensemble.jl) on the device.
 * For every segment of blocks [b0, b1) and both law kinds:
 *   1. u°'s law record ← u's (GP.equalize_law_params!, src/biblock.jl:390-431; c(t0) of u°
 *      is kept),
 *   2. the n named parameters idx[k] ← val[k] (DD.set_parameters!, :360-364; names
 *      DMT_PAR_*), and the fields derived from θ: sigma, a, and — when auxlin — B̃, β̃ of the
 *      auxiliary law linearised at its anchor (ã = a),
 * then GP.recompute_guiding_term!(bb.b°) (:342) for the blocks whose auxiliary law changed
 * (the "critical change"; needs dmt_upload_obs), and recompute_path!(bb.b°, bb.b.WW; skip)
 * (:343).  success_out, critical_out: uint8[b1-b0], nullable.  Only u° changes: the
 * proposal is taken by swap_PP! (dmt_swap DMT_SWAP_PP) on acceptance. */
dmt_status dmt_set_proposal_law(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int32_t n,
                                const int32_t* idx, const double* val, int32_t skip,
                                uint8_t* success_out, uint8_t* critical_out);
/* set_proposal_law!(bb, θ°, pnames, critical_change; skip) with the reference's explicit
 * critical_change (src/biblock.jl:334-344): 1 (true) recomputes u°'s guiding term for every
 * block; 0 (false) only for the blocks where equalizing u°'s law with u's changed the auxiliary
 * law (GP.equalize_law_params!, :361-362), keeping u°'s guiding term elsewhere even if θ°
 * touched it, as the reference does for a caller that passes false; -1 (the default,
 * GP.is_critical_update's role; dmt_set_proposal_law) for the blocks whose auxiliary law
 * changed — the same bits as 1 whenever u°'s guiding term matches its law, since an unchanged
 * law reproduces its guiding term.  critical_out reports the blocks recomputed. */
dmt_status dmt_set_proposal_law_cc(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int32_t n,
                                   const int32_t* idx, const double* val, int32_t skip,
                                   int32_t critical_change, uint8_t* success_out,
                                   uint8_t* critical_out);

/* swap_XX!/swap_WW!/swap_PP!/swap_ll! (src/biblock.jl:148-209), what = DMT_SWAP_* mask. */
dmt_status dmt_swap(dmt_ens* h, int32_t layout, int32_t what, int64_t b0, int64_t b1);

/* save_ll!(·, i) (src/biblock.jl:256-259) and set_accepted!(·, i, v) (src/biblock.jl:135). */
dmt_status dmt_save_ll(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int64_t mcmciter);
/* set_ll!(b, i, v) (src/block.jl:82-86): ll_history[i] = v of bb.b (unit DMT_U) or bb.b°
 * (DMT_UPROP), v: double[b1-b0]. */
dmt_status dmt_set_ll(dmt_ens* h, int32_t layout, int32_t unit, int64_t b0, int64_t b1,
                      int64_t mcmciter, const double* v);
dmt_status dmt_set_accepted(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                            int64_t mcmciter, const uint8_t* v);

/* Read / write per-block state (DMT_BLK_*), out/in sized for blocks [b0, b1)
 * (histories: [hist_len][b1-b0]). */
dmt_status dmt_get_block_state(dmt_ens* h, int32_t layout, int32_t what, int64_t b0,
                               int64_t b1, void* out);
dmt_status dmt_set_block_state(dmt_ens* h, int32_t layout, int32_t what, int64_t b0,
                               int64_t b1, const void* in);

/* fetch_ll / fetch_ll° (src/block_collection.jl:144,156, src/block_ensemble.jl:140,152)
 * over blocks [b0, b1), with the accepted count of iteration mcmciter (0 = skip).
 * Deterministic: a fixed binary tree over the blocks.  With a communicator
 * (dmt_comm_init) the three partials are combined over ranks with RCCL
 * (all-gather + fixed rank-order tree, so the sum does not depend on the rank count
 * when every rank holds a power-of-two number of blocks). */
dmt_status dmt_fetch_ll(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                        int64_t mcmciter, double* ll, double* ll_prop, int64_t* n_acc);

/* One MCMC path-imputation iteration over blocks [b0, b1), device RNG: exactly
 *   dmt_draw_proposal(Z = NULL, iter = mcmciter) ; dmt_accept_reject(E = NULL, mcmciter) ;
 *   dmt_fetch_ll(mcmciter)
 * (draw_proposal_path!(be); accept_reject_proposal_path!(be, i); fetch_ll(be), fetch_ll°(be)
 * and the accepted count — src/block_ensemble.jl:50,63-67,140,152) issued as one call with
 * the decision and the first reduction level fused in one kernel.  Results are identical to
 * the three separate calls. */
dmt_status dmt_mcmc_step(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int64_t mcmciter,
                         uint32_t salt, double* ll, double* ll_prop, int64_t* n_acc);

/* fetch_ll over [b0, b1) of THIS rank only (BiBlock / BlockCollection level,
 * src/biblock.jl:222, src/block_collection.jl:144,156): no collective even when a
 * communicator is set.  dmt_fetch_ll with a communicator is the BlockEnsemble-level reduction
 * (src/block_ensemble.jl:140,152) and must be entered by every rank. */
dmt_status dmt_fetch_ll_local(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                              int64_t mcmciter, double* ll, double* ll_prop, int64_t* n_acc);

/* dmt_mcmc_step over [b0, b1) of THIS rank only: the fused iteration of a BiBlock or a
 * BlockCollection (src/biblock.jl:78-127, src/block_collection.jl:46,60-64,144,156), whose
 * fetch_ll is rank-local; no collective even when a communicator is set, so one rank may call
 * it alone.  dmt_mcmc_step with a communicator is the BlockEnsemble-level call (every rank). */
dmt_status dmt_mcmc_step_local(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                               int64_t mcmciter, uint32_t salt, double* ll, double* ll_prop,
                               int64_t* n_acc);

/* n_iter consecutive dmt_mcmc_step iterations (mcmciter = iter0 … iter0+n_iter-1) queued
 * back to back on the device with no host synchronisation in between: the body of the
 * reference's sampling loop (docs/src/tutorials/biblock/smoothing.md:40-44, which pushes
 * fetch_ll(be) every iteration).  out (nullable): double[n_iter][3] = (fetch_ll, fetch_ll°,
 * accepted count) of every iteration, identical to what the single-step calls return. */
dmt_status dmt_mcmc_run(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int64_t iter0,
                        int64_t n_iter, uint32_t salt, double* out);
/* dmt_mcmc_run with rank-local sums (BiBlock / BlockCollection level, as dmt_mcmc_step_local):
 * no collective. */
dmt_status dmt_mcmc_run_local(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int64_t iter0,
                              int64_t n_iter, uint32_t salt, double* out);

/* ---------------- guiding term (host set-up, GP.build_guid_prop) ---------------- */

/* Exact discrete backward filter for a linear auxiliary law dX = (B̃X + β̃)dt + σ̃dW on
 * one segment's grid t[npts] with terminal information (H_T, F_T, c_T):
 * writes H[npts][d(d+1)/2], F[npts][d], c[npts].  at = packed σ̃σ̃ᵀ.
 * Host-only (no device needed). */
dmt_status dmt_guiding_linear(int32_t d, const double* Bt, const double* beta,
                              const double* at, int32_t npts, const double* t,
                              const double* HT, const double* FT, double cT,
                              double* H, double* F, double* c);
/* The same filter for a time-dependent auxiliary drift: aux[npts][d·d + d] = B̃(t_i), β̃(t_i);
 * step i's exact transition takes the coefficients of its left point t_i (dmt_upload_aux). */
dmt_status dmt_guiding_linear_td(int32_t d, const double* aux, const double* at, int32_t npts,
                                 const double* t, const double* HT, const double* FT, double cT,
                                 double* H, double* F, double* c);
/* ... and with a time-dependent ã too: aux[npts][d·d + d + d(d+1)/2] = B̃, β̃, ã packed; step
 * i's transition takes the trapezoidal averages of rows i and i + 1 (dmt_upload_aux_a). */
dmt_status dmt_guiding_linear_tda(int32_t d, const double* aux, int32_t npts, const double* t,
                                  const double* HT, const double* FT, double cT, double* H,
                                  double* F, double* c);

/* ---------------- multi-GPU (RCCL over xGMI) ---------------- */
dmt_status dmt_comm_unique_id(uint8_t* id_out /*128 bytes*/);
dmt_status dmt_comm_init(dmt_ens* h, int32_t nranks, int32_t rank, const uint8_t* id);
/* ranks of the handle's communicator as RCCL reports them (ncclCommCount), 1 without one */
dmt_status dmt_comm_size(dmt_ens* h, int32_t* nranks);
/* Declare this handle a shard of a larger SamplingEnsemble: its local segment 0 is global
 * segment seg_base.  Device RNG streams are keyed by global segment ids, so a sharded
 * ensemble draws exactly the normals / Exp(1) variables of the unsharded one (weak-scaling
 * shards are bit-identical to the corresponding blocks of one big ensemble).  Default 0.
 * No reference counterpart (the reference is single-process). */
dmt_status dmt_set_shard(dmt_ens* h, int64_t seg_base);
/* The host step of the multi-rank fetch_ll / dmt_mcmc_run: combine every rank's all-gathered
 * partials in rank order.  all[(r·n_iter + i)·3 + c] = rank r's partial c (ll, ll°, accepted
 * count) of iteration i, as ncclAllGather of each rank's [n_iter][3] leaves them;
 * out[i·3 + c] = the complete adjacent-pair tree over ranks 0..nranks−1, padded with zeros to a
 * power of two, + 0.0.  Host-only (no device needed); the code the RCCL
 * paths run after their all-gather.  Replaces the cross-recording part of fetch_ll's
 * mapreduce (src/block_ensemble.jl:140,152), which the single-process reference never splits. */
dmt_status dmt_combine_rank_partials(const double* all, int32_t nranks, int64_t n_iter,
                                     double* out);

/* ---------------- path snapshots ----------------
 * The reference's callers keep every k-th accepted path, `append!(paths, [deepcopy(bb.b.XX)])`
 * (docs/src/tutorials/biblock/smoothing.md:55; per recording, block_ensemble/inference.md:124).
 * Snapshots are kept in HBM: a ring of n_slots copies of XX (what_mask bit 0) and/or WW
 * (bit 1, cumulative Wiener paths) of one unit, reference layout, fp64, taken on the handle's
 * stream without a host round trip (a C3-sized XX snapshot is 1.05 GB; 288 GB of HBM holds
 * a whole smoothing run's worth).  dmt_snapshot_write streams slots [s0, s1) to a file:
 *   dmt_snapshot_header, int32 n_segments[n_recordings], int32 n_points[n_segments],
 *   double t[n_t] (n_t = points of one recording when grid_shared, else n_points total),
 *   then per slot: int64 mcmciter, int64 unit, [double X[P][d]], [double W[P][m]]
 * (little-endian; P = Σ n_points; segments recording-major, as every host array here). */
typedef struct {
    char magic[8];          /* "DMTPATH1" */
    uint32_t version;       /* 1 */
    uint32_t what_mask;     /* 1 XX, 2 WW, 3 both */
    int32_t d, m;
    int32_t grid_shared;
    int32_t precision;      /* of the ensemble the paths come from (DMT_F64 / DMT_F32) */
    int64_t n_recordings, n_segments, n_points, n_t, n_slots;
    int64_t seg_base;       /* global id of local segment 0 (dmt_set_shard) */
} dmt_snapshot_header;

dmt_status dmt_snapshot_reserve(dmt_ens* h, int32_t what_mask, int64_t n_slots);
/* deepcopy(unit.XX / unit.WW) into slot (after every queued kernel), tagged with mcmciter */
dmt_status dmt_snapshot_take(dmt_ens* h, int32_t unit, int64_t slot, int64_t mcmciter);
/* Snapshots inside dmt_mcmc_run: from now on every run snapshots u (dmt_snapshot_take(h, DMT_U,
 * …)) after each iteration k with k % every == 0, into slots slot0, slot0 + 1, … (a ring over
 * the reserved slots), without host synchronisation — the reference's smoothing loop keeps
 * `deepcopy(sp.u.XX)` every few iterations (docs/src/tutorials/biblock/smoothing.md:40-44).
 * every = 0 turns it off. */
dmt_status dmt_set_run_snapshots(dmt_ens* h, int64_t every, int64_t slot0);
dmt_status dmt_snapshot_download(dmt_ens* h, int32_t what, int64_t slot, double* out,
                                 int64_t* mcmciter);
dmt_status dmt_snapshot_write(dmt_ens* h, const char* path, int64_t s0, int64_t s1);

/* ---------------- random stream counter (DMT_RNG_AUTO) ---------------- */
dmt_status dmt_rng_counter(dmt_ens* h, uint64_t* next);
dmt_status dmt_set_rng_counter(dmt_ens* h, uint64_t next);
/* The whole auto-stream state for checkpoint / resume: the next counter value, the key of the
 * last auto draw and whether the next auto accept still takes it (an accept pending after a
 * draw).  Restoring all three resumes bit for bit even between a draw and its accept
 * (dmt_set_rng_counter alone clears the pending draw). */
dmt_status dmt_rng_state(dmt_ens* h, uint64_t* next, uint64_t* last_draw, uint8_t* pending);
dmt_status dmt_set_rng_state(dmt_ens* h, uint64_t next, uint64_t last_draw, uint8_t pending);

/* ---------------- misc ---------------- */
dmt_status dmt_sync(dmt_ens* h);
/* Kernel timing with HIP events on the handle's stream: bit k of `mask` times the kernels of
 * class k (DMT_K_*); -1 = all, 0 = off.  Resets the accumulators. */
dmt_status dmt_set_timing(dmt_ens* h, int32_t mask);
/* accumulated device time (ms) and launch count of a kernel since timing was switched on */
dmt_status dmt_get_timing(dmt_ens* h, int32_t kernel, double* ms, int64_t* count);
/* bytes of device memory held by the handle */
dmt_status dmt_memory_bytes(dmt_ens* h, int64_t* bytes);
/* Debug: raw Philox4x32-10 blocks computed on the device for n counters (ctr[n][4]). */
dmt_status dmt_debug_philox(int32_t device, uint64_t seed, const uint32_t* ctr, int64_t n,
                            uint32_t* out);
/* Debug: device normal pairs (double) for n counters. */
dmt_status dmt_debug_normals(int32_t device, uint64_t seed, const uint32_t* ctr, int64_t n,
                             double* out);
/* Names (demangled) of the last kernels (up to 8) the calling thread launched through libdmt,
 * most recent first, one per line, into buf[n] (truncated, NUL-terminated): which kernel a call
 * dispatched (e.g. k_block_ps_pk or k_block_pk for a C5 draw), as the runtime chose it. */
dmt_status dmt_recent_kernels(char* buf, int64_t n);
const char* dmt_last_error(void);
const char* dmt_version(void);

#ifdef __cplusplus
}
#endif
#endif /* DMT_H */
