// dmt_kernels.hip — gfx950 kernels of the guided-bridge imputation hot path.
//
// k_block  : pCN mix + guided Euler–Maruyama + Girsanov log-weight for whole blocks
//            (replaces GP.rand!(…, ρ, Val(:ll), …) at src/biblock.jl:94-106, GP.solve_and_ll!
//            at src/block.jl:165-167,180 and rand! at src/sampling_unit.jl:119).
// k_pathll : Girsanov log-weight of a stored path (GP.loglikhd, src/block.jl:138-152).
// k_accept : per-block Metropolis–Hastings decision, selector flips, histories
//            (src/biblock.jl:121-127, broadcast src/block_collection.jl:60-64).
// k_block_sum : deterministic tree reduction for fetch_ll / fetch_ll°
//            (src/block_collection.jl:144,156, src/block_ensemble.jl:140,152).
//
// Mapping: one LANE per (recording, block): the 64 lanes of a wave run 64 independent
// Euler recursions in lock-step over a recording tile whose paths are stored
// lane-interleaved ("planes", dmt_internal.h), so every per-step load/store is one
// coalesced 512 B access per component.  Inputs of the next K steps are prefetched into
// registers while the current K steps are integrated (software pipeline, prefetch
// distance K), which is what hides HBM latency at one wave per SIMD.
#include <math.h>
#include <stdlib.h>

#include <type_traits>
#include <hip/hip_ext.h>
#include <algorithm>

#include "dmt_device.h"
#include "dmt_internal.h"
#include "dmt_filter.h"

// gfx950 only: no other target is built or validated (the persistent kernels' inter-workgroup
// hand-offs use gfx950's write-through agent-scope stores).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "dmt_kernels.hip targets gfx950 (MI355X) only"
#endif

namespace dmt {

#ifndef DMT_SPLIT  // 1: one translation unit of the split build (Makefile; see DMT_DISPATCH)
#define DMT_SPLIT 0
#endif
#ifndef DMT_TU_GROUP
#define DMT_TU_GROUP -1
#endif
// the model-independent kernels and launchers: the monolithic build, or the split build's
// common unit
#define DMT_TU_COMMON (!DMT_SPLIT || DMT_TU_GROUP < 0)

template <int K>
struct Log2 { static constexpr int v = K == 1 ? 0 : 1 + Log2<(K > 1 ? K / 2 : 1)>::v; };
template <>
struct Log2<1> { static constexpr int v = 0; };

// Adjacent-pair tree over K values (K a power of two), in place: v[0] = ((v0+v1)+(v2+v3))…
template <class T, int K>
__device__ __forceinline__ T tree_sum(T* v) {
#pragma unroll
  for (int w = K; w > 1; w >>= 1) {
#pragma unroll
    for (int j = 0; j < w / 2; ++j) v[j] = v[2 * j] + v[2 * j + 1];
  }
  return v[0];
}

// Streamed path / table accesses of the lane kernels: non-temporal hints for data a draw
// touches once per launch (C3 / C5 stream 4.7 GB per draw, ≫ L2 and MALL).  Cache hints only:
// the values are the same.  Measured (profiles/r03f, one box): non-temporal X°/W° stores take
// C3 (fp64) from 1 239 to 1 144 µs per draw, but C5 (fp32, whose mixed-selector stores write
// partial lines) from 1 878 to 1 957 µs; non-temporal loads slow both (1 414, 2 291 µs).  So:
// NT stores for fp64 (DMT_LANE_NT_STORES=1 also for fp32, 0 for none), normal loads.
#ifndef DMT_LANE_NT_LOADS
#define DMT_LANE_NT_LOADS 0
#endif
#ifndef DMT_LANE_NT_STORES
#define DMT_LANE_NT_STORES 2  // 2: fp64 only, 1: all, 0: none
#endif
template <class T>
__device__ __forceinline__ T lane_ld(const T* p) {
#if DMT_LANE_NT_LOADS
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
template <class T>
__device__ __forceinline__ void lane_st(T* p, T v) {
  if constexpr (DMT_LANE_NT_STORES == 1 || (DMT_LANE_NT_STORES == 2 && sizeof(T) == 8))
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// One lane integrates one segment.  Main loop: full chunks of K steps, branch-free, with the
// next chunk's inputs (t, H, F, accepted W, and Z in parity mode) loaded into registers
// before the current chunk is integrated (prefetch distance K; no memory operation sits in
// a branch, so the waitcnt pass can count outstanding loads exactly).  Normals of a chunk
// come in whole Box–Muller pairs (K·M even); the chunk's K Girsanov terms are summed as an
// aligned subtree and inserted into the 64-step pairwise counter.  A tail of < K steps
// runs through the single-step path.
#ifndef DMT_LANE_AHEAD  // lane kernels (row layout): chunks of K steps loaded ahead (1 or 2;
#define DMT_LANE_AHEAD 0  // 0: two when a chunk's inputs fit in 40 registers per lane, e.g. FHN)
#endif
#ifndef DMT_KCHUNK_PAIR_BASE
#define DMT_KCHUNK_PAIR_BASE 4  // pair-kernel chunk (doubled when it would hold an odd number of
                                // Philox blocks: Lorenz fp32, 3 normals per step → 8 steps)
#endif
// Two lanes of one wave (l and l + 32) holding the same recording (the pair mapping,
// k_block_pair): role 0 draws the even Philox blocks of a chunk, role 1 the odd ones, and
// v_permlane32_swap hands each half's normals to the other — both roles then run the same
// recursion on the same values (bit-identical to one lane drawing them all).
template <class T>
__device__ __forceinline__ void pair_exchange(T v, T& lo, T& hi);
template <>
__device__ __forceinline__ void pair_exchange<float>(float v, float& lo, float& hi) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  lo = __uint_as_float(r[0]);  // role 0's value in every lane
  hi = __uint_as_float(r[1]);  // role 1's value in every lane
}
template <>
__device__ __forceinline__ void pair_exchange<double>(double v, double& lo, double& hi) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const auto l = __builtin_amdgcn_permlane32_swap((uint32_t)b, (uint32_t)b, false, false);
  const auto h = __builtin_amdgcn_permlane32_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32),
                                                  false, false);
  lo = __longlong_as_double((long long)(((uint64_t)h[0] << 32) | l[0]));
  hi = __longlong_as_double((long long)(((uint64_t)h[1] << 32) | l[1]));
}

template <class Mdl, class T, int MODE, bool PARITY, int K, bool PAIR = false, bool TD = false>
__device__ __forceinline__ bool run_segment(const Law<Mdl, T>& L, const T* __restrict__ tpl,
                                            const int t_sh, const T* __restrict__ Ht,
                                            const int H_sh, const T* __restrict__ Ft,
                                            const T* __restrict__ At,
                                            const T* Ws, T* Wd, T* Xd, const double* __restrict__ Zg,
                                            const T* Xcs, T* Xcd, T* Wcd,
                                            NormalStream<T>& ns, const int64_t tq, const int64_t q0,
                                            const int np, const int lane, const T rho,
                                            const T srho, const int ll_skip, T* x, T& sl,
                                            const int role = 0) {
  constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2;
  constexpr bool DRAW = MODE != MODE_RECOMPUTE;
  constexpr bool READW = MODE != MODE_FRESH;
  static_assert((K * M) % 2 == 0 && 64 % K == 0, "chunk must hold whole normal pairs");
  const int64_t row = tq + q0;
  const T* tb = t_sh ? tpl + q0 : tpl + row * kLanes + lane;
  const int tst = t_sh ? 1 : kLanes;
  const T* Hb = H_sh ? Ht + q0 * HP : Ht + row * HP * kLanes + lane;
  const int hst = H_sh ? 1 : kLanes;
  const T* Fb = Ft + row * D * kLanes + lane;
  const T* Wsb = Ws + row * M * kLanes + lane;
  T* Wdb = Wd + row * M * kLanes + lane;
  T* Xdb = Xd + row * D * kLanes + lane;
  // time-dependent auxiliary law (DMT_LAW_AUXTD): step i's B̃(t_i), β̃(t_i) from the per-point
  // table; wave-uniform, so a time-homogeneous ensemble takes the branch-free path
  // (TD: the ensemble has a per-point table; a separate instantiation, so that a
  // time-homogeneous ensemble runs the kernel without it)
  constexpr int CA = kAuxCols<D>;
  const T* Ab = (TD && At) ? At + row * CA * kLanes + lane : nullptr;
  const bool td = TD && Ab != nullptr && __ballot(L.auxtd) != 0;
  // tile-phase repair: a lane whose u lives in the "wrong" buffer copies u.X
  // (Xcs -> Xcd) and u.W (-> Wcd) to the tile's u buffer while its proposal goes to the
  // tile's proposal buffer; nullptr = nothing to copy
  const bool cpx = Xcd != nullptr, cpw = Wcd != nullptr;
  const T* Xcsb = cpx ? Xcs + row * D * kLanes + lane : nullptr;
  T* Xcdb = cpx ? Xcd + row * D * kLanes + lane : nullptr;
  T* Wcdb = cpw ? Wcd + row * M * kLanes + lane : nullptr;

  // W planes hold increments: row 0 = W(t0), row i+1 = dW_i
  const int nst = np - 1;
  // wave-uniform: every active lane's law has σ = I (the step's fast path)
#ifdef DMT_NO_UNIT_FAST  // measurement variant: the generic path (per-lane selects) always
  const bool all_unit = false;
#else
  const bool all_unit = !Mdl::kLinear && __ballot(L.unit) == __ballot(1);
#endif
  T tcur = tb[0];
  if (cpx) {
#pragma unroll
    for (int p = 0; p < D; ++p) lane_st(&Xcdb[p * kLanes], lane_ld(&Xcsb[p * kLanes]));
  }
#pragma unroll
  for (int p = 0; p < D; ++p) lane_st(&Xdb[p * kLanes], x[p]);
  if (DRAW) {
#pragma unroll
    for (int k = 0; k < M; ++k) {
      const T w0 = READW ? lane_ld(&Wsb[k * kLanes]) : (T)0;
      if (cpw) lane_st(&Wcdb[k * kLanes], w0);
      lane_st(&Wdb[k * kLanes], rho * w0);
    }
  }
  PSum<T> ps;
  ps.init();
#ifdef DMT_PROBE_PKT  // timing probe only: a chunk's X°/W° rows as per-lane K-step packets
  constexpr bool PKT = MODE == MODE_PCN && !PAIR;
#else
  constexpr bool PKT = false;
#endif
  T pkx[K][D], pkw[K][M];

  struct Chunk {
    T t[K], H[K][HP], F[K][D], W[K][M], Z[K][M], Xu[K][D];
  };
  auto load = [&](int c0, Chunk& c) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int64_t i = c0 + j;
      c.t[j] = tb[(i + 1) * tst];
#pragma unroll
      for (int e = 0; e < HP; ++e) c.H[j][e] = lane_ld(&Hb[(i * HP + e) * hst]);
#pragma unroll
      for (int e = 0; e < D; ++e) c.F[j][e] = lane_ld(&Fb[(i * D + e) * kLanes]);
#pragma unroll
      for (int k = 0; k < M; ++k) {
        c.W[j][k] = READW ? lane_ld(&Wsb[((i + 1) * M + k) * kLanes]) : (T)0;
        c.Z[j][k] = (PARITY && DRAW) ? (T)Zg[i * M + k] : (T)0;
      }
      if (cpx) {  // u.X of the points this chunk overwrites (read before they are)
#pragma unroll
        for (int e = 0; e < D; ++e) c.Xu[j][e] = lane_ld(&Xcsb[((i + 1) * D + e) * kLanes]);
      }
    }
  };
  // one Euler step from registers; returns the Girsanov term G·dt
  auto step = [&](int i, T tn, const T* Hi, const T* Fi, const T* Wi, const T* Zi,
                  const T* Xui, const int pj) -> T {
    const T dt = tn - tcur;
    T dW[M];
    if (cpx) {
#pragma unroll
      for (int e = 0; e < D; ++e) lane_st(&Xcdb[((int64_t)(i + 1) * D + e) * kLanes], Xui[e]);
    }
    if (!DRAW) {
#pragma unroll
      for (int k = 0; k < M; ++k) dW[k] = Wi[k];
    } else {
      const T sdt = sqrt(dt);
#pragma unroll
      for (int k = 0; k < M; ++k) {
        if (cpw) lane_st(&Wcdb[((int64_t)(i + 1) * M + k) * kLanes], Wi[k]);
        dW[k] = dfma(rho, Wi[k], srho * (sdt * Zi[k]));
        if (PKT && pj >= 0) pkw[pj][k] = dW[k];
        else lane_st(&Wdb[((int64_t)(i + 1) * M + k) * kLanes], dW[k]);
      }
    }
    T r[D], b[D], sdW[D], Mg[D * D], cg[D];
    T G;
    if constexpr (TD) {
      if (td) {
        T Bq[D * D], bq[D], dq[D * (D + 1) / 2];
        bool trq;
        aux_step<Mdl, T>(L, Ab + (int64_t)i * CA * kLanes, kLanes, Bq, bq, dq, trq,
                         [](const T* p) { return lane_ld(p); });
        G = g_at_aux<Mdl, T>(L, Hi, Fi, x, r, b, Bq, bq, dq, trq);
      } else {
        G = g_at<Mdl, T>(L, Hi, Fi, x, r, b);
      }
    } else {
      G = g_at<Mdl, T>(L, Hi, Fi, x, r, b);
    }
    bool fast = false;
    if constexpr (!Mdl::kLinear && D == M) {
      if (all_unit) {  // every lane's law has σ = I: M = H, c = F, σ·dW = dW (canonical)
#pragma unroll
        for (int p = 0; p < D; ++p) sdW[p] = dW[p];
        guide_coeffs_unit<Mdl, T>(Hi, Fi, Mg, cg);
        fast = true;
      }
    }
    if (!fast) {
      sigma_dw<Mdl, T>(L, dW, sdW);
      guide_coeffs<Mdl, T>(L, Hi, Fi, Mg, cg);
    }
    euler_step<Mdl, T>(L.th, Mg, cg, b, dt, sdW, x);
#pragma unroll
    for (int p = 0; p < D; ++p) {
      if (PKT && pj >= 0) pkx[pj][p] = x[p];
      else lane_st(&Xdb[((int64_t)(i + 1) * D + p) * kLanes], x[p]);
    }
    tcur = tn;
    // recompute_path!(…; skip): the segment's last ll_skip steps add no term
    return (MODE == MODE_RECOMPUTE && i >= nst - ll_skip) ? (T)0 : G * dt;
  };

  const int nfull = nst - nst % K;
  // one chunk of K steps from registers: its normals, the steps, the chunk's subtree
  auto run_chunk = [&](const int c0, Chunk& cur) {
    if (DRAW && !PARITY) {  // whole Philox blocks of normals for this chunk, straight-line
      constexpr int NPB = NormPerBlock<T>::v;
      static_assert((K * M) % NPB == 0, "chunk must hold whole normal blocks");
      if constexpr (PAIR) {  // role r draws blocks 2j + r; the pair swaps halves
        static_assert((K * M / NPB) % 2 == 0, "a pair chunk holds an even number of blocks");
#pragma unroll
        for (int j = 0; j < K * M / NPB / 2; ++j) {
          const uint32_t bc = (uint32_t)((c0 * M) / NPB + 2 * j + role);
          T zb[NPB];
          normal_block(philox4x32_10(U4{bc, ns.seg, ns.iter, ns.c3}, ns.k0, ns.k1), zb);
#pragma unroll
          for (int e = 0; e < NPB; ++e) {
            T lo, hi;
            pair_exchange<T>(zb[e], lo, hi);
            const int n0 = NPB * (2 * j) + e, n1 = NPB * (2 * j + 1) + e;
            cur.Z[n0 / M][n0 % M] = lo;
            cur.Z[n1 / M][n1 % M] = hi;
          }
        }
      } else {
#pragma unroll
        for (int bq = 0; bq < K * M / NPB; ++bq) {
          const uint32_t bc = (uint32_t)((c0 * M) / NPB + bq);
          T zb[NPB];
          normal_block(philox4x32_10(U4{bc, ns.seg, ns.iter, ns.c3}, ns.k0, ns.k1), zb);
#pragma unroll
          for (int e = 0; e < NPB; ++e) cur.Z[(NPB * bq + e) / M][(NPB * bq + e) % M] = zb[e];
        }
      }
    }
    T gv[K];
#pragma unroll
    for (int j = 0; j < K; ++j)
      gv[j] = step(c0 + j, cur.t[j], cur.H[j], cur.F[j], cur.W[j], cur.Z[j], cur.Xu[j], j);
    ps.template add_subtree<Log2<K>::v>(tree_sum<T, K>(gv));
    if constexpr (PKT) {
      static_assert(K * sizeof(T) % 16 == 0, "packets of whole 16-byte pieces");
      typedef T v16 __attribute__((ext_vector_type(16 / sizeof(T))));
      constexpr int NV = 16 / sizeof(T);
#pragma unroll
      for (int p = 0; p < D; ++p) {
        T* q = Xd + (row + c0 + 1) * D * kLanes + ((int64_t)p * kLanes + lane) * K;
#pragma unroll
        for (int h = 0; h < K / NV; ++h) {
          v16 v;
#pragma unroll
          for (int e = 0; e < NV; ++e) v[e] = pkx[h * NV + e][p];
          __builtin_nontemporal_store(v, (v16*)(q + h * NV));
        }
      }
#pragma unroll
      for (int k = 0; k < M; ++k) {
        T* q = Wd + (row + c0 + 1) * M * kLanes + ((int64_t)k * kLanes + lane) * K;
#pragma unroll
        for (int h = 0; h < K / NV; ++h) {
          v16 v;
#pragma unroll
          for (int e = 0; e < NV; ++e) v[e] = pkw[h * NV + e][k];
          __builtin_nontemporal_store(v, (v16*)(q + h * NV));
        }
      }
    }
  };
  // chunks in flight: one, or two where a chunk's inputs (t, H, F, W, Z, u.X: one value each)
  // take few registers — C3 (FHN, fp64): 1 061-1 070 -> 1 011-1 013 µs per draw; Lorenz's
  // lane kernels spill with two (profiles/r05h)
  constexpr int kChunkVals = K * (1 + HP + D + 2 * M + D);
  constexpr int AHEAD = DMT_LANE_AHEAD ? DMT_LANE_AHEAD : (kChunkVals <= 40 ? 2 : 1);
  if (nfull > 0 && AHEAD == 2) {
    // a ring of three register sets, unrolled by three so that no set is copied (a copy would
    // wait for the loads just issued); the tile's kPadPoints spare rows keep the prefetch 2K
    // points past the segment in bounds
    static_assert(2 * K <= kPadPoints, "prefetch distance exceeds the tile's spare rows");
    Chunk c_a, c_b, c_c;
    load(0, c_a);
    load(K, c_b);
    for (int c0 = 0;;) {
      if (c0 >= nfull) break;
      load(c0 + 2 * K, c_c);
      run_chunk(c0, c_a);
      c0 += K;
      if (c0 >= nfull) break;
      load(c0 + 2 * K, c_a);
      run_chunk(c0, c_b);
      c0 += K;
      if (c0 >= nfull) break;
      load(c0 + 2 * K, c_b);
      run_chunk(c0, c_c);
      c0 += K;
    }
  } else if (nfull > 0) {
    Chunk cur, nxt;
    load(0, cur);
    for (int c0 = 0; c0 < nfull; c0 += K) {
      load(c0 + K, nxt);  // prefetch; padded rows keep the last one in bounds
      run_chunk(c0, cur);
      cur = nxt;
    }
  }
  for (int i = nfull; i < nst; ++i) {  // tail (< K steps): single-step path
    const int64_t q = i;
    T Hi[HP], Fi[D], Wi[M], Zi[M], Xui[D];
#pragma unroll
    for (int e = 0; e < D; ++e) Xui[e] = cpx ? lane_ld(&Xcsb[((q + 1) * D + e) * kLanes]) : (T)0;
#pragma unroll
    for (int e = 0; e < HP; ++e) Hi[e] = lane_ld(&Hb[(q * HP + e) * hst]);
#pragma unroll
    for (int e = 0; e < D; ++e) Fi[e] = lane_ld(&Fb[(q * D + e) * kLanes]);
#pragma unroll
    for (int k = 0; k < M; ++k) {
      Wi[k] = READW ? lane_ld(&Wsb[((q + 1) * M + k) * kLanes]) : (T)0;
      Zi[k] = DRAW ? (PARITY ? (T)Zg[q * M + k] : ns.get((uint32_t)(i * M + k))) : (T)0;
    }
    ps.add(step(i, tb[(q + 1) * tst], Hi, Fi, Wi, Zi, Xui, -1));
  }
  sl = ps.finish();
  bool ok = isfinite(sl);
#pragma unroll
  for (int p = 0; p < D; ++p) ok = ok && isfinite(x[p]);
  return ok;
}

// Common prologue: map (wave, lane) → (tile, block index, recording, flat block id).
template <class T>
__device__ __forceinline__ bool map_block(const BlockArgs<T>& a, int64_t& tile, int64_t& blk) {
  const int lane = threadIdx.x;
  const int64_t wave = blockIdx.x;
  tile = a.tile0 + wave / a.MB;
  const int b = (int)(wave % a.MB);
  if (tile >= a.tile1) return false;
  const int64_t r = tile * kLanes + lane;
  if (r >= a.R) return false;
  blk = a.blk_off[r] + b;
  if (blk >= a.blk_off[r + 1] || blk < a.b0 || blk >= a.b1) return false;
  return true;
}


// Path buffers of one container (X or W) in a MAP_LANE draw (MODE_PCN: reads u, writes u°),
// decided per wave over its active lanes from how many lanes hold their u in each buffer
// ("path buffers").  A partial line costs far more than its bytes: a wave's
// proposal stores should all go to ONE buffer.  M = the buffer holding most lanes' u.
//  * a buffer holds no active lane's u and M holds >= 3/4 of them (high acceptance: a wave's
//    lanes mostly move together): every proposal goes there, nothing is copied;
//  * three buffers all in use by <= 1/16 stragglers outside M: no copy, the smallest group's
//    lanes write to M, the rest to the smallest group's buffer;
//  * otherwise (while the off-M lanes are <= 1/repair_div of the wave and >= repair_min lanes):
//    consolidate — every lane outside M moves its u to M during the sweep (read before
//    overwritten) and every proposal goes to buffer 0 or 1 other than M (the tile-phase repair
//    of two buffers; a wave of a low-acceptance chain stays on two buffers);
//  * else each lane writes to a buffer other than its own u (mixed).
// Measured per draw (profiles/r03rep, r03pbuf2; draw + accept loops): C3 (acceptance 0.99) two
// buffers with the repair 1 137-1 164 µs, with up to 3 mixed lanes per wave 1 351, three buffers
// without copies 1 037, all lanes flipping together 1 010; C5 (0.54) two buffers mixed 1 899,
// consolidated 1 818, three buffers in use 2 264-2 284.
struct PathPlan {
  int p, src, dst;  // this lane's proposal buffer; its u moves src -> dst (src < 0: stays)
};
__device__ __forceinline__ PathPlan path_plan(const bool act, const int u, const int nbuf,
                                              const int repair_div, const int repair_min,
                                              const int full = 0) {
  const int nact = __popcll(__ballot(act));
  const int c0 = __popcll(__ballot(act && u == 0)), c1 = __popcll(__ballot(act && u == 1));
  const int c2 = nact - c0 - c1;  // 0 with two buffers
  int m = c1 > c0 ? 1 : 0, cm = c1 > c0 ? c1 : c0;
  if (nbuf == 3 && c2 > cm) { m = 2; cm = c2; }
  const int fr = c0 == 0 ? 0 : (c1 == 0 ? 1 : (nbuf == 3 && c2 == 0 ? 2 : -1));  // a free buffer
  const int off = nact - cm;
  const int other = m == 0 ? 1 : 0;  // the proposal buffer of a consolidated wave
  PathPlan r{u == m ? other : m, -1, -1};  // mixed
  if (fr >= 0 && 4 * cm >= 3 * nact) {
    r.p = fr;
  } else if (nbuf == 3 && fr < 0 && 16 * off <= nact) {
    const int o1 = m == 0 ? 1 : 0, o2 = m == 2 ? 1 : 2;  // the two buffers other than m
    const int co1 = o1 == 0 ? c0 : c1, co2 = o2 == 1 ? c1 : c2;
    const int sm = co1 <= co2 ? o1 : o2;
    r.p = u == sm ? m : sm;
  } else if (repair_div * off <= nact && off >= repair_min) {
    r.p = other;
    if (u != m || full) { r.src = u; r.dst = m; }  // full: the majority rewrites its own u too
  }
  return r;
}

// The lane kernel's body for block blk of recording tile `tile`, recording slot `lane` of the
// tile (the lane-interleaved layout's column); PAIR: two lanes (roles) per recording.
template <class Mdl, class T, int MODE, bool PARITY, int K, bool PAIR, bool TD = false>
__device__ __forceinline__ void lane_block(const BlockArgs<T>& a, const int64_t tile,
                                           const int64_t blk, const int lane, const int role) {
  constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2;
  const int64_t tq = a.tile_qoff[tile];
  auto idx = [&](int64_t q, int c, int C) -> int64_t { return ((tq + q) * C + c) * kLanes + lane; };
  const int g0 = a.gfirst[blk], g1 = a.glast[blk];
  const bool term = a.term[blk] != 0;

  T x[D];
  {
    const T* Xs = a.X[sel_buf(a.selX[g0], a.xs_flip)];
    const int64_t q = a.seg_q[g0];
#pragma unroll
    for (int p = 0; p < D; ++p) x[p] = Xs[idx(q, p, D)];
  }
  T ll;
  {
    const int ls = a.selPP[g0] ^ a.law_flip;
    const double* Lr = a.law[ls][0] + (int64_t)g0 * DMT_LAW_STRIDE;
    const T* Ht = a.H[ls][0];
    const T* Ft = a.F[ls][0];
    const int64_t q = a.seg_q[g0];
    T H0[HP], F0[D];
#pragma unroll
    for (int c = 0; c < HP; ++c) H0[c] = a.H_shared[ls][0] ? Ht[q * HP + c] : Ht[idx(q, c, HP)];
#pragma unroll
    for (int c = 0; c < D; ++c) F0[c] = Ft[idx(q, c, D)];
    ll = obs_term<D, T>(H0, F0, x, (T)Lr[DMT_LAW_C0]);
  }
  bool ok = true;
  const T rho = (MODE == MODE_FRESH) ? (T)0 : (T)a.rho[blk];
  const T srho = (MODE == MODE_FRESH) ? (T)1 : (T)a.srho[blk];
  for (int g = g0; g <= g1; ++g) {
    const int kind = (!term && g == g1) ? 1 : 0;
    const int ls = (kind ? a.selPPB[g] : a.selPP[g]) ^ a.law_flip;
    Law<Mdl, T> L;
    L.load(a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE);
    NormalStream<T> ns;
    ns.init(a.seed, (uint32_t)g + a.seg_base, a.iter, a.salt);
    const double* Zg = a.Z ? a.Z + a.st_off[g] * M : nullptr;
    const int sx = a.selX[g], sw = a.selW[g];
    T* Xd = a.X[sel_buf(sx, a.xd_flip)];
    const T* Ws = a.W[sel_buf(sw, a.ws_flip)];
    T* Wd = a.W[sel_buf(sw, a.wd_flip)];
    const T* Xcs = nullptr;
    T *Xcd = nullptr, *Wcd = nullptr;
    int nsx = sx, nsw = sw;
    if (MODE == MODE_PCN) {  // one proposal buffer per wave (path_plan)
      const PathPlan px = path_plan(true, sel_u(sx), a.nbuf, a.repair_div, a.repair_min, a.full_copy);
      const PathPlan pw = path_plan(true, sel_u(sw), a.nbuf, a.repair_div, a.repair_min, a.full_copy);
      Xd = a.X[px.p];
      Wd = a.W[pw.p];
      if (px.src >= 0) { Xcs = a.X[px.src]; Xcd = a.X[px.dst]; }
      if (pw.src >= 0) Wcd = a.W[pw.dst];
      nsx = sel_make(px.src >= 0 ? px.dst : sel_u(sx), px.p);
      nsw = sel_make(pw.src >= 0 ? pw.dst : sel_u(sw), pw.p);
    }
    T sl;
    const bool sok = run_segment<Mdl, T, MODE, PARITY, K, PAIR, TD>(
        L, a.t, a.t_shared, a.H[ls][kind], a.H_shared[ls][kind], a.F[ls][kind], a.aux[kind], Ws,
        Wd, Xd, Zg,
        Xcs, Xcd, Wcd, ns, tq, a.seg_q[g], a.seg_np[g], lane, rho, srho, a.ll_skip, x, sl, role);
    if (MODE == MODE_PCN) {
      if (nsx != sx) a.selX[g] = (uint8_t)nsx;
      if (nsw != sw) a.selW[g] = (uint8_t)nsw;
    }
    if (!sok) { ok = false; break; }
    ll = ll + sl;
  }
  if (role == 0) {
    a.ll_out[blk] = ok ? (double)ll : -INFINITY;
    if (a.success) a.success[blk] = ok ? 1 : 0;
  }
}

template <class Mdl, class T, int MODE, bool PARITY, int K, bool TD = false>
__global__ __launch_bounds__(64) void k_block(const BlockArgs<T> a) {
  int64_t tile, blk;
  if (!map_block(a, tile, blk)) return;
  lane_block<Mdl, T, MODE, PARITY, K, false, TD>(a, tile, blk, threadIdx.x, 0);
}

template <class Mdl, class T>
struct PairChunk {  // steps per chunk: an even number of whole Philox blocks of normals
  static constexpr int NPB = NormPerBlock<T>::v;
  static constexpr int v = ((DMT_KCHUNK_PAIR_BASE * Mdl::M) % (2 * NPB) == 0)
                               ? DMT_KCHUNK_PAIR_BASE : 2 * DMT_KCHUNK_PAIR_BASE;
};

// ---- MAP_LANE with lane packets (fp32 ensembles, BlockArgs::pk = kPathPacket).
// The path planes X, W hold each lane's PK consecutive points of a component as one 64-byte
// piece (plane_ix), so the per-lane buffers of u and u° (two, selected per segment exactly as
// the reference swaps its containers) never share a piece of memory: a wave whose lanes hold u
// in different buffers reads and writes whole pieces of its own, with no partial lines, no
// consolidation copies and no third buffer (the row layout's path_plan).  FAST (every active
// lane's segment starts at point ≡ PK − 1 of a packet, which dmt_create arranges for the first
// segment of every recording): per packet of PK steps the lane loads u.W's packet one packet
// ahead (NV 16-byte pieces per component, back to back) and stores the packet's X°, W° whole at
// its end; the remaining steps (and segments not so aligned) go point by point through
// plane_ix.  The arithmetic, its order and the Girsanov summation tree (K-step subtrees from
// the segment start, single steps for the last nst % K) are run_segment's, so the results are
// bit-identical to the row layout's and to the oracle's.
#ifndef DMT_PK_ROLL  // 1: u.W's next packet loaded piece by piece into the registers just consumed
#define DMT_PK_ROLL 1   // 0: the whole next packet in a second register set
#endif
#ifndef DMT_PK_SDT_TABLE  // shared grids: the packet kernel reads √dt from a per-point table
#define DMT_PK_SDT_TABLE 1
#endif
#ifndef DMT_PK_CHUNK_STORE  // 1: X°, W° pieces stored at the end of the chunk that completes them
#define DMT_PK_CHUNK_STORE 0   // (measured slower: C5 1 906-1 925 vs 1 432-1 449 µs per draw,
                               // profiles/r05b) 0: the whole packet staged in registers, stored at its end
#endif
#ifndef DMT_PK_LDS  // 1: the packet's X°, W° staged in the lane's LDS rows
#define DMT_PK_LDS 0   // 0: staged in registers (measured faster in the kernel: 1 455 vs 1 574 µs, C5)
#endif
// PAIR (k_block_pk_pair): two lanes (roles) of a wave per recording, l and l + 32 — each draws
// every other Philox block of a chunk and the pair swaps halves (pair_exchange), both run the
// recursion on the same values; role 0 stores X°, role 1 W° (every load is the same address
// for both, one request).  Fills the chip with twice the waves when the ensemble has fewer
// recording tiles than SIMDs (C5: 512 tiles, 1 024 SIMDs).  Bit-identical.
// SDT: a shared grid's √dt table (BlockArgs::sdt) read per step in place of the square root
template <class Mdl, class T, int MODE, bool PARITY, int K, bool TD, int PK, bool FAST,
          bool PAIR = false, bool SDT = false>
__device__ __forceinline__ bool run_segment_pk(const Law<Mdl, T>& L, const T* __restrict__ tpl,
                                               const int t_sh, const T* __restrict__ Ht,
                                               const int H_sh, const T* __restrict__ Ft,
                                               const T* __restrict__ At, const T* Ws, T* Wd,
                                               T* Xd, const double* __restrict__ Zg,
                                               NormalStream<T>& ns, const int64_t tq,
                                               const int64_t q0, const int np, const int lane,
                                               const T rho, const T srho, const int ll_skip,
                                               T* x, T& sl, T* stg, const int role = 0,
                                               const T* __restrict__ sdtab = nullptr) {
  constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2;
  constexpr bool DRAW = MODE != MODE_RECOMPUTE;
  constexpr bool READW = MODE != MODE_FRESH;
  const bool stx = !PAIR || role == 0, stw = DRAW && (!PAIR || role == 1);  // who stores what
  constexpr int VE = 16 / (int)sizeof(T);  // elements per 16-byte piece
  constexpr int NV = PK / VE;              // pieces per packet
  static_assert(PK % K == 0 && K % VE == 0 && (K * M) % 2 == 0 && 64 % K == 0,
                "packets of whole chunks, chunks of whole 16-byte pieces");
  typedef T v16 __attribute__((ext_vector_type(VE)));
  const int64_t row = tq + q0;
  const T* tb = t_sh ? tpl + q0 : tpl + row * kLanes + lane;
  const int tst = t_sh ? 1 : kLanes;
  const T* Hb = H_sh ? Ht + q0 * HP : Ht + row * HP * kLanes + lane;
  const int hst = H_sh ? 1 : kLanes;
  const T* Fb = Ft + row * D * kLanes + lane;
  // point i of the segment, component c, in the layout's lane packets (kPathPacket points); the
  // loop below stages PK-point pieces of them (PK divides kPathPacket)
  static_assert(kPathPacket % PK == 0, "whole pieces per layout packet");
  auto pix = [&](int64_t i, int c, int C) -> int64_t {
    return plane_ix(row + i, c, C, kLanes, lane, kPathPacket);
  };
  constexpr int CA = kAuxCols<D>;
  const T* Ab = (TD && At) ? At + row * CA * kLanes + lane : nullptr;
  const bool td = TD && Ab != nullptr && __ballot(L.auxtd) != 0;
  const int nst = np - 1;
#ifdef DMT_NO_UNIT_FAST
  const bool all_unit = false;
#else
  const bool all_unit = !Mdl::kLinear && __ballot(L.unit) == __ballot(1);
#endif
  T tcur = tb[0];
  if (stx) {
#pragma unroll
    for (int p = 0; p < D; ++p) Xd[pix(0, p, D)] = x[p];
  }
  if (stw) {
#pragma unroll
    for (int k = 0; k < M; ++k) {
      const T w0 = READW ? Ws[pix(0, k, M)] : (T)0;
      Wd[pix(0, k, M)] = rho * w0;
    }
  }
  PSum<T> ps;
  ps.init();
  // one Euler step from registers (run_segment's step): dW (in: u's increment, out: the
  // proposal's), x advanced; returns the Girsanov term G·dt
  const T* sdb = SDT ? sdtab + q0 : nullptr;  // step i's √dt at sdb[i] (shared grid)
  auto step = [&](int i, T tn, const T* Hi, const T* Fi, T* dW, const T* Zi, T sdt_i) -> T {
    const T dt = tn - tcur;
    if (DRAW) {
      const T sdt = SDT ? sdt_i : sqrt(dt);
#pragma unroll
      for (int k = 0; k < M; ++k) dW[k] = dfma(rho, dW[k], srho * (sdt * Zi[k]));
    }
    T r[D], b[D], sdW[D], Mg[D * D], cg[D];
    T G;
    if constexpr (TD) {
      if (td) {
        T Bq[D * D], bq[D], dq[D * (D + 1) / 2];
        bool trq;
        aux_step<Mdl, T>(L, Ab + (int64_t)i * CA * kLanes, kLanes, Bq, bq, dq, trq,
                         [](const T* p) { return lane_ld(p); });
        G = g_at_aux<Mdl, T>(L, Hi, Fi, x, r, b, Bq, bq, dq, trq);
      } else {
        G = g_at<Mdl, T>(L, Hi, Fi, x, r, b);
      }
    } else {
      G = g_at<Mdl, T>(L, Hi, Fi, x, r, b);
    }
    bool fast = false;
    if constexpr (!Mdl::kLinear && D == M) {
      if (all_unit) {
#pragma unroll
        for (int p = 0; p < D; ++p) sdW[p] = dW[p];
        guide_coeffs_unit<Mdl, T>(Hi, Fi, Mg, cg);
        fast = true;
      }
    }
    if (!fast) {
      sigma_dw<Mdl, T>(L, dW, sdW);
      guide_coeffs<Mdl, T>(L, Hi, Fi, Mg, cg);
    }
    euler_step<Mdl, T>(L.th, Mg, cg, b, dt, sdW, x);
    tcur = tn;
    return (MODE == MODE_RECOMPUTE && i >= nst - ll_skip) ? (T)0 : G * dt;
  };
  struct Chunk {
    T t[K], s[K], H[K][HP], F[K][D], Z[K][M];
  };
  auto load = [&](int c0, Chunk& c) {  // the chunk's grid, guiding term, caller normals
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int64_t i = c0 + j;
      c.t[j] = tb[(i + 1) * tst];
      c.s[j] = (SDT && DRAW) ? sdb[i] : (T)0;
#pragma unroll
      for (int e = 0; e < HP; ++e) c.H[j][e] = lane_ld(&Hb[(i * HP + e) * hst]);
#pragma unroll
      for (int e = 0; e < D; ++e) c.F[j][e] = lane_ld(&Fb[(i * D + e) * kLanes]);
#pragma unroll
      for (int k = 0; k < M; ++k) c.Z[j][k] = (PARITY && DRAW) ? (T)Zg[i * M + k] : (T)0;
    }
  };
  auto normals = [&](int c0, Chunk& c) {  // whole Philox blocks of the chunk, straight-line
    if (DRAW && !PARITY) {
      constexpr int NPB = NormPerBlock<T>::v;
      static_assert((K * M) % NPB == 0, "chunk must hold whole normal blocks");
      if constexpr (PAIR) {  // role r draws blocks 2j + r; the pair swaps halves
        static_assert((K * M / NPB) % 2 == 0, "a pair chunk holds an even number of blocks");
#pragma unroll
        for (int j = 0; j < K * M / NPB / 2; ++j) {
          const uint32_t bc = (uint32_t)((c0 * M) / NPB + 2 * j + role);
          T zb[NPB];
          normal_block(philox4x32_10(U4{bc, ns.seg, ns.iter, ns.c3}, ns.k0, ns.k1), zb);
#pragma unroll
          for (int e = 0; e < NPB; ++e) {
            T lo, hi;
            pair_exchange<T>(zb[e], lo, hi);
            const int n0 = NPB * (2 * j) + e, n1 = NPB * (2 * j + 1) + e;
            c.Z[n0 / M][n0 % M] = lo;
            c.Z[n1 / M][n1 % M] = hi;
          }
        }
      } else {
#pragma unroll
        for (int bq = 0; bq < K * M / NPB; ++bq) {
          const uint32_t bc = (uint32_t)((c0 * M) / NPB + bq);
          T zb[NPB];
          normal_block(philox4x32_10(U4{bc, ns.seg, ns.iter, ns.c3}, ns.k0, ns.k1), zb);
#pragma unroll
          for (int e = 0; e < NPB; ++e) c.Z[(NPB * bq + e) / M][(NPB * bq + e) % M] = zb[e];
        }
      }
    }
  };
  int i0 = 0;  // steps done by the packet loop
  if constexpr (FAST) {
    const int npk = nst / PK;
    if (npk > 0) {
      // packet j of a component: the segment's points j·PK + 1 … j·PK + PK, NV pieces
      auto wpk = [&](int j, int k) -> const v16* { return (const v16*)&Ws[pix((int64_t)j * PK + 1, k, M)]; };
      v16 wc[M][NV];
#if !DMT_PK_ROLL
      v16 wn[M][NV];
#endif
      if (READW) {
#pragma unroll
        for (int k = 0; k < M; ++k)
#pragma unroll
          for (int v = 0; v < NV; ++v) wc[k][v] = wpk(0, k)[v];
      }
      Chunk cur, nxt;
      load(0, cur);
      for (int j = 0; j < npk; ++j) {
#if !DMT_PK_ROLL
        if (READW) {  // next packet (the tile's spare rows keep the last one in bounds)
#pragma unroll
          for (int k = 0; k < M; ++k)
#pragma unroll
            for (int v = 0; v < NV; ++v) wn[k][v] = wpk(j + 1, k)[v];
        }
#endif
        // the packet's X°, W° are collected step by step and leave as whole 16-byte pieces at
        // the packet's end: in registers (default), or in the lane's LDS rows (stg[c][e][lane],
        // a 65-element row pitch; DMT_PK_LDS=1 — faster in the layout probe, slower in the kernel)
        // (a pair's roles each store one of the two, so they share NS staging rows: X° rows for
        // role 0, W° rows for role 1)
        constexpr int NS = PAIR ? (D > M ? D : M) : D + M, WR = PAIR ? 0 : D;
#if DMT_PK_LDS
        auto st = [&](int c, int e) -> T& { return stg[(c * PK + e) * 65 + lane]; };
        auto put = [&](int c, int e, T v) { st(c, e) = v; };
#elif DMT_PK_CHUNK_STORE
        // a chunk of K steps completes K / VE whole pieces of every component: they leave at
        // the chunk's end (the registers of one chunk's pieces instead of a whole packet's)
        constexpr int CP = K / VE;
        v16 ob[NS][CP];
        auto put = [&](int c, int e, T v) { ob[c][(e % K) / VE][e % VE] = v; };
#else
        v16 ob[NS][NV];
        auto put = [&](int c, int e, T v) { ob[c][e / VE][e % VE] = v; };
#endif
#pragma unroll
        for (int v = 0; v < PK / K; ++v) {
          const int c0 = j * PK + v * K;
          load(c0 + K, nxt);
          normals(c0, cur);
          T gv[K];
#pragma unroll
          for (int q = 0; q < K; ++q) {
            const int e = v * K + q;  // element of the packet
            T dW[M];
#pragma unroll
            for (int k = 0; k < M; ++k) dW[k] = READW ? wc[k][e / VE][e % VE] : (T)0;
            gv[q] = step(c0 + q, cur.t[q], cur.H[q], cur.F[q], dW, cur.Z[q], cur.s[q]);
            if constexpr (PAIR) {
#pragma unroll
              for (int c = 0; c < NS; ++c)
                put(c, e, stx ? (c < D ? x[c] : (T)0) : (c < M ? dW[c] : (T)0));
            } else {
#pragma unroll
              for (int p = 0; p < D; ++p) put(p, e, x[p]);
              if (DRAW) {
#pragma unroll
                for (int k = 0; k < M; ++k) put(D + k, e, dW[k]);
              }
            }
          }
#if !DMT_PK_LDS && DMT_PK_CHUNK_STORE
          if (stx) {
#pragma unroll
            for (int p = 0; p < D; ++p) {
              v16* dst = (v16*)&Xd[pix((int64_t)j * PK + 1, p, D)];
#pragma unroll
              for (int u = 0; u < CP; ++u) dst[v * CP + u] = ob[p][u];
            }
          }
          if (stw) {
#pragma unroll
            for (int k = 0; k < M; ++k) {
              v16* dst = (v16*)&Wd[pix((int64_t)j * PK + 1, k, M)];
#pragma unroll
              for (int u = 0; u < CP; ++u) dst[v * CP + u] = ob[WR + k][u];
            }
          }
#endif
#if DMT_PK_ROLL
          // the piece of u.W this chunk consumed is refilled with the next packet's: a prefetch
          // distance of one packet in the registers of one (the tile's spare rows keep the
          // last packet's in bounds)
          if (READW) {
#pragma unroll
            for (int k = 0; k < M; ++k)
#pragma unroll
              for (int pc = v * K / VE; pc < (v + 1) * K / VE; ++pc) wc[k][pc] = wpk(j + 1, k)[pc];
          }
#endif
          ps.template add_subtree<Log2<K>::v>(tree_sum<T, K>(gv));
          cur = nxt;
        }
#if DMT_PK_LDS || !DMT_PK_CHUNK_STORE
        auto piece = [&](int c, int v) -> v16 {
#if DMT_PK_LDS
          v16 o;
#pragma unroll
          for (int u = 0; u < VE; ++u) o[u] = st(c, v * VE + u);
          return o;
#else
          return ob[c][v];
#endif
        };
        if (stx) {
#pragma unroll
          for (int p = 0; p < D; ++p) {
            v16* dst = (v16*)&Xd[pix((int64_t)j * PK + 1, p, D)];
#pragma unroll
            for (int v = 0; v < NV; ++v) dst[v] = piece(p, v);
          }
        }
        if (stw) {
#pragma unroll
          for (int k = 0; k < M; ++k) {
            v16* dst = (v16*)&Wd[pix((int64_t)j * PK + 1, k, M)];
#pragma unroll
            for (int v = 0; v < NV; ++v) dst[v] = piece(WR + k, v);
          }
        }
#endif
#if !DMT_PK_ROLL
        if (READW) {
#pragma unroll
          for (int k = 0; k < M; ++k)
#pragma unroll
            for (int v = 0; v < NV; ++v) wc[k][v] = wn[k][v];
        }
#endif
      }
      i0 = npk * PK;
    }
  }
  // the remaining whole chunks, point by point (FAST: < PK steps; else every chunk)
  const int nfull = nst - nst % K;
  if (i0 < nfull) {
    Chunk cur, nxt;
    load(i0, cur);
    for (int c0 = i0; c0 < nfull; c0 += K) {
      load(c0 + K, nxt);
      T wu[K][M];
#pragma unroll
      for (int q = 0; q < K; ++q)
#pragma unroll
        for (int k = 0; k < M; ++k) wu[q][k] = READW ? Ws[pix(c0 + q + 1, k, M)] : (T)0;
      normals(c0, cur);
      T gv[K];
#pragma unroll
      for (int q = 0; q < K; ++q) {
        gv[q] = step(c0 + q, cur.t[q], cur.H[q], cur.F[q], wu[q], cur.Z[q], cur.s[q]);
        if (stx) {
#pragma unroll
          for (int p = 0; p < D; ++p) Xd[pix(c0 + q + 1, p, D)] = x[p];
        }
        if (stw) {
#pragma unroll
          for (int k = 0; k < M; ++k) Wd[pix(c0 + q + 1, k, M)] = wu[q][k];
        }
      }
      ps.template add_subtree<Log2<K>::v>(tree_sum<T, K>(gv));
      cur = nxt;
    }
  }
  for (int i = nfull; i < nst; ++i) {  // tail (< K steps): single steps
    const int64_t q = i;
    T Hi[HP], Fi[D], dW[M], Zi[M];
#pragma unroll
    for (int e = 0; e < HP; ++e) Hi[e] = lane_ld(&Hb[(q * HP + e) * hst]);
#pragma unroll
    for (int e = 0; e < D; ++e) Fi[e] = lane_ld(&Fb[(q * D + e) * kLanes]);
#pragma unroll
    for (int k = 0; k < M; ++k) {
      dW[k] = READW ? Ws[pix(q + 1, k, M)] : (T)0;
      Zi[k] = DRAW ? (PARITY ? (T)Zg[q * M + k] : ns.get((uint32_t)(i * M + k))) : (T)0;
    }
    ps.add(step(i, tb[(q + 1) * tst], Hi, Fi, dW, Zi, (SDT && DRAW) ? sdb[q] : (T)0));
    if (stx) {
#pragma unroll
      for (int p = 0; p < D; ++p) Xd[pix(q + 1, p, D)] = x[p];
    }
    if (stw) {
#pragma unroll
      for (int k = 0; k < M; ++k) Wd[pix(q + 1, k, M)] = dW[k];
    }
  }
  sl = ps.finish();
  bool ok = isfinite(sl);
#pragma unroll
  for (int p = 0; p < D; ++p) ok = ok && isfinite(x[p]);
  return ok;
}

template <class Mdl, class T, int MODE, bool PARITY, int K, bool TD, bool PAIR = false,
          bool SDT = false>
__device__ __forceinline__ void lane_block_pk(const BlockArgs<T>& a, const int64_t tile,
                                              const int64_t blk, const int lane, T* stg,
                                              const int role = 0) {
  constexpr int D = Mdl::D, HP = D * (D + 1) / 2, PK = kPkChunkPts;  // staged piece (points)
  const int64_t tq = a.tile_qoff[tile];
  auto idx = [&](int64_t q, int c, int C) -> int64_t { return ((tq + q) * C + c) * kLanes + lane; };
  const int g0 = a.gfirst[blk], g1 = a.glast[blk];
  const bool term = a.term[blk] != 0;
  T x[D];
  {
    const T* Xs = a.X[sel_buf(a.selX[g0], a.xs_flip)];
    const int64_t q = a.seg_q[g0];
#pragma unroll
    for (int p = 0; p < D; ++p) x[p] = Xs[plane_ix(tq + q, p, D, kLanes, lane, kPathPacket)];
  }
  T ll;
  {
    const int ls = a.selPP[g0] ^ a.law_flip;
    const double* Lr = a.law[ls][0] + (int64_t)g0 * DMT_LAW_STRIDE;
    const T* Ht = a.H[ls][0];
    const T* Ft = a.F[ls][0];
    const int64_t q = a.seg_q[g0];
    T H0[HP], F0[D];
#pragma unroll
    for (int c = 0; c < HP; ++c) H0[c] = a.H_shared[ls][0] ? Ht[q * HP + c] : Ht[idx(q, c, HP)];
#pragma unroll
    for (int c = 0; c < D; ++c) F0[c] = Ft[idx(q, c, D)];
    ll = obs_term<D, T>(H0, F0, x, (T)Lr[DMT_LAW_C0]);
  }
  bool ok = true;
  const T rho = (MODE == MODE_FRESH) ? (T)0 : (T)a.rho[blk];
  const T srho = (MODE == MODE_FRESH) ? (T)1 : (T)a.srho[blk];
  for (int g = g0; g <= g1; ++g) {
    const int kind = (!term && g == g1) ? 1 : 0;
    const int ls = (kind ? a.selPPB[g] : a.selPP[g]) ^ a.law_flip;
    Law<Mdl, T> L;
    L.load(a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE);
    NormalStream<T> ns;
    ns.init(a.seed, (uint32_t)g + a.seg_base, a.iter, a.salt);
    const double* Zg = a.Z ? a.Z + a.st_off[g] * Mdl::M : nullptr;
    const int sx = a.selX[g], sw = a.selW[g];
    T* Xd = a.X[sel_buf(sx, a.xd_flip)];
    const T* Ws = a.W[sel_buf(sw, a.ws_flip)];
    T* Wd = a.W[sel_buf(sw, a.wd_flip)];
    const int64_t q0 = a.seg_q[g];
    const bool aligned = __ballot(((tq + q0 + 1) & (PK - 1)) != 0) == 0;
    T sl;
    // SDT (a shared grid with its √dt table, launch-time choice): the aligned segments read √dt
    const bool sok =
        aligned ? run_segment_pk<Mdl, T, MODE, PARITY, K, TD, PK, true, PAIR, SDT>(
                      L, a.t, a.t_shared, a.H[ls][kind], a.H_shared[ls][kind], a.F[ls][kind],
                      a.aux[kind], Ws, Wd, Xd, Zg, ns, tq, q0, a.seg_np[g], lane, rho, srho,
                      a.ll_skip, x, sl, stg, role, SDT ? a.sdt : nullptr)
                : run_segment_pk<Mdl, T, MODE, PARITY, K, TD, PK, false, PAIR>(
                      L, a.t, a.t_shared, a.H[ls][kind], a.H_shared[ls][kind], a.F[ls][kind],
                      a.aux[kind], Ws, Wd, Xd, Zg, ns, tq, q0, a.seg_np[g], lane, rho, srho,
                      a.ll_skip, x, sl, stg, role);
    if (!sok) { ok = false; break; }
    ll = ll + sl;
  }
  if (role == 0) {
    a.ll_out[blk] = ok ? (double)ll : -INFINITY;
    if (a.success) a.success[blk] = ok ? 1 : 0;
  }
}

template <class Mdl, class T, int MODE, bool PARITY, int K, bool TD = false, bool SDT = false>
__global__ __launch_bounds__(64) void k_block_pk(const BlockArgs<T> a) {
  __shared__ T stg[DMT_PK_LDS ? (Mdl::D + Mdl::M) * kPkChunkPts * 65 : 1];  // X°, W° (DMT_PK_LDS)
  int64_t tile, blk;
  if (!map_block(a, tile, blk)) return;
  lane_block_pk<Mdl, T, MODE, PARITY, K, TD, false, SDT>(a, tile, blk, threadIdx.x, stg);
}

// lane pairs on the packet layout (device-RNG draws): two waves per (recording tile, block
// index), 32 recordings each on lanes (l, l + 32) — the mapping of k_block_pair
template <class Mdl, class T, int MODE, bool TD = false>
__global__ __launch_bounds__(64) void k_block_pk_pair(const BlockArgs<T> a) {
  __shared__ T stg[DMT_PK_LDS ? (Mdl::D + Mdl::M) * kPkChunkPts * 65 : 1];
  const int lane = threadIdx.x, role = lane >> 5;
  const int64_t wave = blockIdx.x, w2 = wave >> 1;
  const int slot = (int)(wave & 1) * 32 + (lane & 31);
  const int64_t tile = a.tile0 + w2 / a.MB;
  const int b = (int)(w2 % a.MB);
  if (tile >= a.tile1) return;
  const int64_t r = tile * kLanes + slot;
  if (r >= a.R) return;
  const int64_t blk = a.blk_off[r] + b;
  if (blk >= a.blk_off[r + 1] || blk < a.b0 || blk >= a.b1) return;
  lane_block_pk<Mdl, T, MODE, false, PairChunk<Mdl, T>::v, TD, true>(a, tile, blk, slot, stg, role);
}

// ---- MAP_LANE, pair mapping: two waves per (recording tile, block index), each
// holding 32 recordings of the tile on lane pairs (l, l + 32).  The pair draws a chunk's normals
// half each (pair_exchange) and runs the recursion redundantly, so an ensemble with fewer
// tiles than the device has SIMDs (C5: 512 tiles, 1 024 SIMDs) fills the chip with waves whose
// per-step instruction stream is the recursion plus HALF the random-number work.  Same
// operations on the same values per recording: bit-identical to k_block.


template <class Mdl, class T, int MODE>
__global__ __launch_bounds__(64) void k_block_pair(const BlockArgs<T> a) {
  const int lane = threadIdx.x, role = lane >> 5;
  const int64_t wave = blockIdx.x, w2 = wave >> 1;
  const int slot = (int)(wave & 1) * 32 + (lane & 31);
  const int64_t tile = a.tile0 + w2 / a.MB;
  const int b = (int)(w2 % a.MB);
  if (tile >= a.tile1) return;
  const int64_t r = tile * kLanes + slot;
  if (r >= a.R) return;
  const int64_t blk = a.blk_off[r] + b;
  if (blk >= a.blk_off[r + 1] || blk < a.b0 || blk >= a.b1) return;
  lane_block<Mdl, T, MODE, false, PairChunk<Mdl, T>::v, true>(a, tile, blk, slot, role);
}



// ---- MAP_LANE, split into a producer and a consumer wave.  For draws
// (MODE_PCN, device RNG) over single-segment blocks.  One workgroup of two waves per
// (recording tile, block index): the PRODUCER wave loads t and u's W, draws the normals
// (Philox/Box–Muller), forms dW° = fma(ρ, dW, √(1−ρ²)·√dt·Z), stores W° and hands (dt, dW°)
// to the CONSUMER through LDS, chunk by chunk (kPsChunk steps, double-buffered, one barrier per
// chunk); the consumer runs the Euler recursion, the Girsanov terms, the pairwise sums and the
// X° stores.  Each wave's instruction stream is about half the single-wave kernel's, which is
// what bounds the lane mapping when the ensemble has fewer tiles than the chip has SIMDs (C5).
// Same operations in the same order as k_block: bit-identical.
#ifndef DMT_PS_CHUNK
#define DMT_PS_CHUNK 16
#endif
constexpr int kPsChunk = DMT_PS_CHUNK;
#ifndef DMT_PS_MINW
#define DMT_PS_MINW 1  // 2 (with DMT_PS_CHUNK 8, no spills) measured no better: 1 877 vs 1 749–1 782 µs on C5
#endif

template <class Mdl, class T>
__global__ __launch_bounds__(128, DMT_PS_MINW) void k_block_ps(const BlockArgs<T> a) {
  constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2;
  constexpr int L = kPsChunk, K = 4;
  static_assert(L % K == 0 && (L * M) % 2 == 0, "chunk must hold whole normal pairs");
  __shared__ T s_dt[2][L][64];
  __shared__ T s_dw[2][L][M][64];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t tile = a.tile0 + blockIdx.x / a.MB;
  const int bidx = (int)(blockIdx.x % a.MB);
  if (tile >= a.tile1) return;  // whole workgroup
  const int64_t r = tile * kLanes + lane;
  int64_t blk = -1;
  if (r < a.R) {
    blk = a.blk_off[r] + bidx;
    if (blk >= a.blk_off[r + 1] || blk < a.b0 || blk >= a.b1) blk = -1;
  }
  const bool act = blk >= 0;
  const int64_t tq = a.tile_qoff[tile];
  const int g = act ? a.gfirst[blk] : 0;  // the block's only segment (host-checked), terminal
  const int nst = act ? a.seg_np[g] - 1 : 0;
  // chunks: the longest lane of the tile (both waves compute the same count)
  int nmax = nst;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) nmax = max(nmax, __shfl_xor(nmax, o, 64));
  const int nch = (__builtin_amdgcn_readfirstlane(nmax) + L - 1) / L;
  const int64_t row = tq + (act ? a.seg_q[g] : 0);
  const T rho = act ? (T)a.rho[blk] : (T)0;
  const T srho = act ? (T)a.srho[blk] : (T)1;
  // selectors and the tile-phase repair decision (k_block), identical in both waves
  const int sx = act ? a.selX[g] : kSelInit, sw = act ? a.selW[g] : kSelInit;
  const T* Ws = a.W[sel_buf(sw, a.ws_flip)];
  const T *Xcs = nullptr;
  T *Xcd = nullptr, *Wcd = nullptr;
  // one proposal buffer per wave (path_plan; MODE_PCN)
  const PathPlan px = path_plan(act, sel_u(sx), a.nbuf, a.repair_div, a.repair_min, a.full_copy);
  const PathPlan pw = path_plan(act, sel_u(sw), a.nbuf, a.repair_div, a.repair_min, a.full_copy);
  T* Xd = a.X[px.p];
  T* Wd = a.W[pw.p];
  if (px.src >= 0) { Xcs = a.X[px.src]; Xcd = a.X[px.dst]; }
  if (pw.src >= 0) Wcd = a.W[pw.dst];
  const int nsx = sel_make(px.src >= 0 ? px.dst : sel_u(sx), px.p);
  const int nsw = sel_make(pw.src >= 0 ? pw.dst : sel_u(sw), pw.p);
  auto idx = [&](int64_t q, int c, int C) -> int64_t { return ((row + q) * C + c) * kLanes + lane; };

  if (w == 0) {
    // ================= producer =================
    const T* tb = a.t_shared ? a.t + (act ? a.seg_q[g] : 0) : a.t + row * kLanes + lane;
    const int tst = a.t_shared ? 1 : kLanes;
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
    const uint32_t seg = (uint32_t)g + a.seg_base, c3 = a.salt << 1;
    T tcur = tb[0];
    if (act) {
#pragma unroll
      for (int k = 0; k < M; ++k) {
        const T w0 = Ws[idx(0, k, M)];
        if (Wcd) Wcd[idx(0, k, M)] = w0;
        Wd[idx(0, k, M)] = rho * w0;
      }
    }
    // prefetched inputs of the next chunk (rows past a segment end read padding: in bounds)
    T pt[L], pw_[L][M];
    auto load = [&](int c) {
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const int64_t i = (int64_t)c * L + j;
        const int64_t ii = min<int64_t>(i, max(nst - 1, 0));
        pt[j] = tb[(ii + 1) * tst];
#pragma unroll
        for (int k = 0; k < M; ++k) pw_[j][k] = Ws[idx(ii + 1, k, M)];
      }
    };
    load(0);
    for (int c = -1; c < nch; ++c) {
      if (c + 1 < nch) {
        const int cp = c + 1, buf = cp & 1;
        T ct[L], cw[L][M];
#pragma unroll
        for (int j = 0; j < L; ++j) {
          ct[j] = pt[j];
#pragma unroll
          for (int k = 0; k < M; ++k) cw[j][k] = pw_[j][k];
        }
        if (cp + 1 < nch) load(cp + 1);
        T z[L][M];
        constexpr int NPB = NormPerBlock<T>::v;
        static_assert((L * M) % NPB == 0, "chunk must hold whole normal blocks");
#pragma unroll
        for (int bq = 0; bq < L * M / NPB; ++bq) {
          const uint32_t bc = (uint32_t)((cp * L * M) / NPB + bq);
          T zb[NPB];
          normal_block(philox4x32_10(U4{bc, seg, a.iter, c3}, k0, k1), zb);
#pragma unroll
          for (int e = 0; e < NPB; ++e) z[(NPB * bq + e) / M][(NPB * bq + e) % M] = zb[e];
        }
#pragma unroll
        for (int j = 0; j < L; ++j) {
          const int64_t i = (int64_t)cp * L + j;
          const bool v = act && i < nst;
          const T dt = ct[j] - tcur;
          const T sdt = sqrt(dt);
          s_dt[buf][j][lane] = dt;
#pragma unroll
          for (int k = 0; k < M; ++k) {
            const T dw = dfma(rho, cw[j][k], srho * (sdt * z[j][k]));
            s_dw[buf][j][k][lane] = dw;
            if (v) {
              if (Wcd) Wcd[idx(i + 1, k, M)] = cw[j][k];
              Wd[idx(i + 1, k, M)] = dw;
            }
          }
          tcur = v ? ct[j] : tcur;
        }
      }
      __syncthreads();
    }
  } else {
    // ================= consumer =================
    Law<Mdl, T> LA;
    const int ls = act ? (a.selPP[g] ^ a.law_flip) : 0;
    LA.load(a.law[ls][0] + (int64_t)g * DMT_LAW_STRIDE);
    // wave-uniform: every active lane's law has σ = I (the step's fast path, as in k_block)
    const bool all_unit = !Mdl::kLinear && __ballot(!act || LA.unit) == __ballot(1);
    const T* Hb = a.H_shared[ls][0] ? a.H[ls][0] + (act ? a.seg_q[g] : 0) * HP : a.H[ls][0] + row * HP * kLanes + lane;
    const int hst = a.H_shared[ls][0] ? 1 : kLanes;
    const T* Fb = a.F[ls][0] + row * D * kLanes + lane;
    T x[D];
    {
      const T* Xs = a.X[sel_buf(sx, a.xs_flip)];
#pragma unroll
      for (int p = 0; p < D; ++p) x[p] = Xs[idx(0, p, D)];
    }
    T ll;
    {
      T H0[HP], F0[D];
#pragma unroll
      for (int e = 0; e < HP; ++e) H0[e] = Hb[e * hst];
#pragma unroll
      for (int e = 0; e < D; ++e) F0[e] = Fb[e * kLanes];
      ll = obs_term<D, T>(H0, F0, x, (T)a.law[ls][0][(int64_t)g * DMT_LAW_STRIDE + DMT_LAW_C0]);
    }
    if (act) {
      if (Xcd) {
#pragma unroll
        for (int p = 0; p < D; ++p) Xcd[idx(0, p, D)] = Xcs[idx(0, p, D)];
      }
#pragma unroll
      for (int p = 0; p < D; ++p) Xd[idx(0, p, D)] = x[p];
    }
    PSum<T> ps;
    ps.init();
    const int nfull = nst - nst % K;
    struct Sub { T H[K][HP], F[K][D], Xu[K][D]; };
    auto load = [&](int64_t i0, Sub& s) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const int64_t i = min<int64_t>(i0 + j, max(nst - 1, 0));
#pragma unroll
        for (int e = 0; e < HP; ++e) s.H[j][e] = Hb[(i * HP + e) * hst];
#pragma unroll
        for (int e = 0; e < D; ++e) s.F[j][e] = Fb[(i * D + e) * kLanes];
        if (Xcd) {
#pragma unroll
          for (int e = 0; e < D; ++e) s.Xu[j][e] = Xcs[idx(i + 1, e, D)];
        }
      }
    };
    Sub cur, nxt;
    load(0, cur);
    for (int c = -1; c < nch; ++c) {
      if (c >= 0) {
        const int buf = c & 1;
#pragma unroll
        for (int q = 0; q < L / K; ++q) {
          const int64_t i0 = (int64_t)c * L + q * K;
          load(i0 + K, nxt);  // prefetch (the next chunk's first sub-chunk at q = L/K - 1)
          T gv[K];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const int64_t i = i0 + j;
            const bool v = act && i < nst;
            const T dt = s_dt[buf][q * K + j][lane];
            T dW[M];
#pragma unroll
            for (int k = 0; k < M; ++k) dW[k] = s_dw[buf][q * K + j][k][lane];
            T rr[D], b[D], sdW[D], Mg[D * D], cg[D];
            const T G = g_at<Mdl, T>(LA, cur.H[j], cur.F[j], x, rr, b);
            bool fast = false;
            if constexpr (!Mdl::kLinear && D == M) {
              if (all_unit) {
#pragma unroll
                for (int p = 0; p < D; ++p) sdW[p] = dW[p];
                guide_coeffs_unit<Mdl, T>(cur.H[j], cur.F[j], Mg, cg);
                fast = true;
              }
            }
            if (!fast) {
              sigma_dw<Mdl, T>(LA, dW, sdW);
              guide_coeffs<Mdl, T>(LA, cur.H[j], cur.F[j], Mg, cg);
            }
            T xn[D];
#pragma unroll
            for (int p = 0; p < D; ++p) xn[p] = x[p];
            euler_step<Mdl, T>(LA.th, Mg, cg, b, dt, sdW, xn);
            if (v) {
              if (Xcd) {
#pragma unroll
                for (int e = 0; e < D; ++e) Xcd[idx(i + 1, e, D)] = cur.Xu[j][e];
              }
#pragma unroll
              for (int p = 0; p < D; ++p) {
                x[p] = xn[p];
                Xd[idx(i + 1, p, D)] = xn[p];
              }
            }
            gv[j] = G * dt;
          }
          if (i0 + K <= nfull) {
            ps.template add_subtree<Log2<K>::v>(tree_sum<T, K>(gv));
          } else {
#pragma unroll
            for (int j = 0; j < K; ++j)
              if (i0 + j < nst) ps.add(gv[j]);
          }
          cur = nxt;
        }
      }
      __syncthreads();
    }
    if (act) {
      const T sl = ps.finish();
      bool ok = isfinite(sl);
#pragma unroll
      for (int p = 0; p < D; ++p) ok = ok && isfinite(x[p]);
      if (nsx != sx) a.selX[g] = (uint8_t)nsx;
      if (nsw != sw) a.selW[g] = (uint8_t)nsw;
      a.ll_out[blk] = ok ? (double)(ll + sl) : -INFINITY;
      if (a.success) a.success[blk] = ok ? 1 : 0;
    }
  }
}

// ---- MAP_LANE packets, split into a producer and a consumer wave: k_block_ps's division of
// work on the lane-packet layout (fp32 ensembles).  For draws (MODE_PCN, device
// RNG, no per-point auxiliary table) over single-segment blocks whose segments start on a packet
// boundary (the first segment of every recording does).  One workgroup of two waves per
// (recording tile, block index), one packet of PK steps per hand-off (double-buffered LDS, one
// barrier per packet): the PRODUCER reads u.W's packets, draws the packet's normals (whole
// Philox blocks), forms dW° = fma(ρ, dW, √(1−ρ²)·(√dt·Z)), stores W°'s packet and hands (dt,
// dW°) over; the CONSUMER loads H, F one chunk of K steps ahead, runs the guided recursion and
// the Girsanov terms and stores X°'s packet.  The operations, their order, the normal numbering
// and the summation tree are run_segment_pk's (K-step subtrees for every whole chunk, single
// steps after), so the results are bit-identical to k_block_pk's.  A wave whose segments are
// not aligned runs lane_block_pk on the consumer wave alone.
#ifndef DMT_PSPK_STUB
#define DMT_PSPK_STUB 0
#endif
#ifndef DMT_PSPK_GLDS  // the consumer's H, F chunks by LDS-DMA (global_load_lds_dwordx4), ring of
#define DMT_PSPK_GLDS 0   // DMT_PSPK_GLDS_SLOTS slots, one fewer chunks in flight (0: register ring);
#endif                    // C5 1 282 (4 slots), 1 293 (5) vs 1 278 µs per draw (profiles/r06e)
#ifndef DMT_PSPK_GLDS_SLOTS
#define DMT_PSPK_GLDS_SLOTS 4
#endif
// One LDS-DMA wave-instruction: each lane's 16 bytes at gsrc land at the wave-uniform LDS byte
// address lds_dst + 16·lane (M0 holds the base; saved and restored in the same statement, the
// recipe of cdna_hip_programming.md §5.7).  hipcc does not count it: the caller waits with its
// own s_waitcnt vmcnt before reading the bytes.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
#ifndef DMT_PSPK_PAIR  // whole 128-byte lines per lane: a packet's first piece waits in LDS;
#define DMT_PSPK_PAIR 1   // C5 1 152 vs 1 278 µs per draw without (profiles/r06e)
#endif
#ifndef DMT_PSPK_RING  // the consumer's H, F register ring (chunks of K steps; 2 = one ahead;
#define DMT_PSPK_RING 2   // 4, three ahead, measured the same: 1 350 vs 1 341-1 343 µs, r05l)
#endif
template <class Mdl, class T, int K, bool SDT>
__global__ __launch_bounds__(128, 1) void k_block_ps_pk(const BlockArgs<T> a) {
  constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2, PK = kPkChunkPts;  // staged piece
  constexpr int VE = 16 / (int)sizeof(T), NV = PK / VE;
  constexpr int NPB = NormPerBlock<T>::v;
  static_assert(PK % K == 0 && (PK * M) % NPB == 0 && (K * M) % 2 == 0, "whole chunks, blocks");
  typedef T v16 __attribute__((ext_vector_type(VE)));
  __shared__ T s_dt[2][PK][64];
  __shared__ T s_dw[2][PK][M][64];
  // the one-wave fallback's X°, W° staging (DMT_PK_LDS builds; one element otherwise)
  __shared__ T stg[DMT_PK_LDS ? (Mdl::D + Mdl::M) * kPkChunkPts * 65 : 1];
  // whole-line stores (DMT_PSPK_PAIR): a layout packet is kPathPacket / PK pieces; the first
  // piece of each waits in LDS (each lane its own slots) until the second completes the lane's
  // 128-byte line, which then leaves in one run of stores — a half line written ≈ 16 steps
  // before its other half was often evicted in between: a partial write, read back (FETCH)
  constexpr bool PAIRW = DMT_PSPK_PAIR && kPathPacket == 2 * PK;
  __shared__ v16 stW[PAIRW ? M : 1][PAIRW ? NV : 1][64];  // producer: W° first halves
  __shared__ v16 stX[PAIRW ? D : 1][PAIRW ? NV : 1][64];  // consumer: X° first halves
  // the consumer's H, F chunks of K steps by LDS-DMA (DMT_PSPK_GLDS): slot image = the tile's
  // rows as they lie in memory, H [K][HP][64] then F [K][D][64]
  constexpr int GCH = K * HP * 64, GCF = K * D * 64;  // elements per chunk
  constexpr int NGS = DMT_PSPK_GLDS ? DMT_PSPK_GLDS_SLOTS : 1;
  [[maybe_unused]] __shared__ T hfr[NGS][DMT_PSPK_GLDS ? GCH + GCF : 1];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t tile = a.tile0 + blockIdx.x / a.MB;
  const int bidx = (int)(blockIdx.x % a.MB);
  if (tile >= a.tile1) return;  // whole workgroup
  const int64_t r = tile * kLanes + lane;
  int64_t blk = -1;
  if (r < a.R) {
    blk = a.blk_off[r] + bidx;
    if (blk >= a.blk_off[r + 1] || blk < a.b0 || blk >= a.b1) blk = -1;
  }
  const bool act = blk >= 0;
  const int64_t tq = a.tile_qoff[tile];
  const int g = act ? a.gfirst[blk] : 0;  // the block's only segment (host-checked)
  const int64_t q0 = act ? a.seg_q[g] : 0;
  const int64_t row = tq + q0;
  // both waves take the same branch (same lanes, same values).  The LDS-DMA consumer
  // (DMT_PSPK_GLDS) also needs every lane's segment at the tile's first row and per-point H
  bool glds_off = false;
  if constexpr (DMT_PSPK_GLDS) {
    const int lsu = act ? ((a.term[blk] != 0 ? a.selPP[g] : a.selPPB[g]) ^ a.law_flip) : 0;
    const int kdu = act && a.term[blk] == 0 ? 1 : 0;
    glds_off = __ballot(act && (q0 != 0 || a.H_shared[lsu][kdu] != 0)) != 0;
  }
  if (glds_off || __ballot(act && ((row + 1) & (PK - 1)) != 0) != 0) {
    if (w == 1 && act) lane_block_pk<Mdl, T, MODE_PCN, false, K, false, false, SDT>(a, tile, blk, lane, stg);
    return;
  }
  const int nst = act ? a.seg_np[g] - 1 : 0;
  int nmax = nst;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) nmax = max(nmax, __shfl_xor(nmax, o, 64));
  const int nch = (__builtin_amdgcn_readfirstlane(nmax) + PK - 1) / PK;  // packets
  const int sx = act ? a.selX[g] : kSelInit, sw = act ? a.selW[g] : kSelInit;
  // every lane's segment starts a layout packet: piece p is the first half of its packet for
  // even p (uniform; the first segment of every recording, dmt_create's tile alignment)
  const bool pair = PAIRW && __ballot(act && ((row + 1) & (kPathPacket - 1)) != 0) == 0;
  auto pix = [&](int64_t i, int c, int C) -> int64_t {  // the layout's lane packets
    return plane_ix(row + i, c, C, kLanes, lane, kPathPacket);
  };
  if (w == 0) {
    // ================= producer =================
    const T rho = act ? (T)a.rho[blk] : (T)0;
    const T srho = act ? (T)a.srho[blk] : (T)1;
    NormalStream<T> ns;
    ns.init(a.seed, (uint32_t)g + a.seg_base, a.iter, a.salt);
    const T* Ws = a.W[sel_buf(sw, a.ws_flip)];
    T* Wd = a.W[sel_buf(sw, a.wd_flip)];
    const T* tb = a.t_shared ? a.t + q0 : a.t + row * kLanes + lane;
    const int tst = a.t_shared ? 1 : kLanes;
    const T* sdb = SDT ? a.sdt + q0 : nullptr;
    const int ilast = max(nst - 1, 0);  // per-step tables are read clamped to the segment
    T tcur = tb[0];
    if (act) {
#pragma unroll
      for (int k = 0; k < M; ++k) Wd[pix(0, k, M)] = rho * Ws[pix(0, k, M)];
    }
    // packet p of a component: points p·PK + 1 … p·PK + PK (the tile's spare rows keep the last
    // packet's whole pieces in bounds); the next packet's pieces and grid prefetched
    auto wpk = [&](int p, int k) -> const v16* { return (const v16*)&Ws[pix((int64_t)p * PK + 1, k, M)]; };
    v16 wn[M][NV];
    T tn_[PK], sn_[PK];
    auto load = [&](int p) {
#pragma unroll
      for (int k = 0; k < M; ++k)
#pragma unroll
        for (int v = 0; v < NV; ++v) wn[k][v] = wpk(p, k)[v];
#pragma unroll
      for (int e = 0; e < PK; ++e) {
        const int64_t i = min((int64_t)p * PK + e, (int64_t)ilast);
        tn_[e] = tb[(i + 1) * tst];
        sn_[e] = SDT ? sdb[i] : (T)0;
      }
    };
    load(0);
    for (int c = -1; c < nch; ++c) {
      if (c + 1 < nch) {
        const int p = c + 1, buf = p & 1;
        v16 wc[M][NV];
        T tc[PK], sc[PK];
#pragma unroll
        for (int k = 0; k < M; ++k)
#pragma unroll
          for (int v = 0; v < NV; ++v) wc[k][v] = wn[k][v];
#pragma unroll
        for (int e = 0; e < PK; ++e) { tc[e] = tn_[e]; sc[e] = sn_[e]; }
        if (p + 1 < nch) load(p + 1);
        T z[PK][M];
#pragma unroll
        for (int bq = 0; bq < PK * M / NPB; ++bq) {
          const uint32_t bc = (uint32_t)((p * PK * M) / NPB + bq);
          T zb[NPB];
#if DMT_PSPK_STUB & 2  // timing stub: the consumer alone (no normals drawn; wrong results)
#pragma unroll
          for (int e = 0; e < NPB; ++e) zb[e] = (T)(bc & 7) * (T)0.125;
#else
          normal_block(philox4x32_10(U4{bc, ns.seg, ns.iter, ns.c3}, ns.k0, ns.k1), zb);
#endif
#if DMT_PSPK_STUB & 16  // timing probe (results unchanged): every normal block drawn twice
          {
            uint32_t bc2 = bc;
            asm volatile("" : "+v"(bc2));
            T zb2[NPB];
            normal_block(philox4x32_10(U4{bc2, ns.seg, ns.iter, ns.c3}, ns.k0, ns.k1), zb2);
#pragma unroll
            for (int e = 0; e < NPB; ++e) asm volatile("" ::"v"(zb2[e]));
          }
#endif
#pragma unroll
          for (int e = 0; e < NPB; ++e) z[(NPB * bq + e) / M][(NPB * bq + e) % M] = zb[e];
        }
        v16 ob[M][NV];
#pragma unroll
        for (int e = 0; e < PK; ++e) {
          const bool v = act && p * PK + e < nst;
          const T dt = tc[e] - tcur;
          const T sdt = SDT ? sc[e] : sqrt(dt);
          s_dt[buf][e][lane] = dt;
#pragma unroll
          for (int k = 0; k < M; ++k) {
            const T dw = dfma(rho, wc[k][e / VE][e % VE], srho * (sdt * z[e][k]));
            s_dw[buf][e][k][lane] = dw;
            ob[k][e / VE][e % VE] = dw;
          }
          tcur = v ? tc[e] : tcur;
        }
        if (act) {
          if ((p + 1) * PK <= nst) {  // a whole piece
            if (pair && (p & 1) == 0 && (p + 2) * PK <= nst) {  // first half: wait in LDS
#pragma unroll
              for (int k = 0; k < M; ++k)
#pragma unroll
                for (int v = 0; v < NV; ++v) stW[k][v][lane] = ob[k][v];
            } else if (pair && (p & 1) == 1) {  // second half: the lane's whole line
#pragma unroll
              for (int k = 0; k < M; ++k) {
                v16* dst = (v16*)&Wd[pix((int64_t)(p - 1) * PK + 1, k, M)];
#pragma unroll
                for (int v = 0; v < NV; ++v) dst[v] = stW[k][v][lane];
#pragma unroll
                for (int v = 0; v < NV; ++v) dst[NV + v] = ob[k][v];
              }
            } else {
#pragma unroll
              for (int k = 0; k < M; ++k) {
                v16* dst = (v16*)&Wd[pix((int64_t)p * PK + 1, k, M)];
#pragma unroll
                for (int v = 0; v < NV; ++v) dst[v] = ob[k][v];
              }
            }
          } else {
#pragma unroll
            for (int e = 0; e < PK; ++e)
              if (p * PK + e < nst)
#pragma unroll
                for (int k = 0; k < M; ++k) Wd[pix((int64_t)p * PK + e + 1, k, M)] = ob[k][e / VE][e % VE];
          }
        }
      }
      __syncthreads();
    }
  } else {
    // ================= consumer =================
    const bool term = act ? a.term[blk] != 0 : true;
    const int kind = term ? 0 : 1;  // a non-terminal block's segment takes the blocking law
    const int ls = act ? ((kind ? a.selPPB[g] : a.selPP[g]) ^ a.law_flip) : 0;
    Law<Mdl, T> LA;
    LA.load(a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE);
    const bool all_unit = !Mdl::kLinear && __ballot(!act || LA.unit) == __ballot(1);
    const T* Ht = a.H[ls][kind];
    const int hsh = a.H_shared[ls][kind];
    const T* Hb = hsh ? Ht + q0 * HP : Ht + row * HP * kLanes + lane;
    const int hst = hsh ? 1 : kLanes;
    const T* Fb = a.F[ls][kind] + row * D * kLanes + lane;
    T x[D];
    {
      const T* Xs = a.X[sel_buf(sx, a.xs_flip)];
#pragma unroll
      for (int p = 0; p < D; ++p) x[p] = Xs[pix(0, p, D)];
    }
    T ll;
    {  // the block's observation term: u's terminal-kind law of its first segment (lane_block_pk)
      const int l0 = act ? (a.selPP[g] ^ a.law_flip) : 0;
      const T* H0t = a.H[l0][0];
      T H0[HP], F0[D];
#pragma unroll
      for (int e = 0; e < HP; ++e) H0[e] = a.H_shared[l0][0] ? H0t[q0 * HP + e] : H0t[(row * HP + e) * kLanes + lane];
#pragma unroll
      for (int e = 0; e < D; ++e) F0[e] = a.F[l0][0][(row * D + e) * kLanes + lane];
      ll = obs_term<D, T>(H0, F0, x, (T)a.law[l0][0][(int64_t)g * DMT_LAW_STRIDE + DMT_LAW_C0]);
    }
    T* Xd = a.X[sel_buf(sx, a.xd_flip)];
    if (act) {
#pragma unroll
      for (int p = 0; p < D; ++p) Xd[pix(0, p, D)] = x[p];
    }
    const int ilast = max(nst - 1, 0);
    PSum<T> ps;
    ps.init();
    const int nfull = nst - nst % K;
    struct Sub { T H[K][HP], F[K][D]; };
    auto load = [&](int64_t i0, Sub& s) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const int64_t i = min<int64_t>(i0 + j, ilast);
#if DMT_PSPK_STUB & 8  // timing stub: no H, F loads (wrong results)
#pragma unroll
        for (int e = 0; e < HP; ++e) s.H[j][e] = (T)(i & 3) * (T)0.01;
#pragma unroll
        for (int e = 0; e < D; ++e) s.F[j][e] = (T)(i & 7) * (T)0.01;
#else
#pragma unroll
        for (int e = 0; e < HP; ++e) s.H[j][e] = lane_ld(&Hb[(i * HP + e) * hst]);
#pragma unroll
        for (int e = 0; e < D; ++e) s.F[j][e] = lane_ld(&Fb[(i * D + e) * kLanes]);
#endif
      }
    };
#if DMT_PSPK_GLDS
    // LDS-DMA ring (every lane's segment at the tile's first row — the first segment of every
    // recording, C5 — and per-point tables: a chunk of the tile's H, F rows is then one
    // contiguous block, copied by 1 KB wave-instructions without registers, the loads of
    // NGS - 1 chunks in flight).  The chunk's rows are read unclamped: a lane past its own
    // segment end only evaluates steps it never adds or applies (the tile's spare rows keep
    // every read inside the tile)
    constexpr int NIH = GCH * (int)sizeof(T) / 1024, NIF = GCF * (int)sizeof(T) / 1024;
    static_assert(GCH * sizeof(T) % 1024 == 0 && GCF * sizeof(T) % 1024 == 0, "whole 1 KB copies");
    static_assert((NGS - 1) * K + K <= kPadPoints && (NGS - 1) * (NIH + NIF) <= 63, "ring depth");
    const T* Ft = a.F[ls][kind];
    auto gissue = [&](int64_t i0, int slot) {  // chunk of steps [i0, i0 + K) → slot
      const T* hs = Ht + (tq + i0) * HP * kLanes + lane * (16 / (int)sizeof(T));
      const T* fs = Ft + (tq + i0) * D * kLanes + lane * (16 / (int)sizeof(T));
      const uint32_t l0 = (uint32_t)(uintptr_t)&hfr[slot][0];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's last reads retired (WAR)
#pragma unroll
      for (int j = 0; j < NIH; ++j)
        glds16(hs + j * (1024 / (int)sizeof(T)), __builtin_amdgcn_readfirstlane(l0 + 1024u * j));
#pragma unroll
      for (int j = 0; j < NIF; ++j)
        glds16(fs + j * (1024 / (int)sizeof(T)),
               __builtin_amdgcn_readfirstlane(l0 + (uint32_t)(GCH * sizeof(T)) + 1024u * j));
    };
    auto gread = [&](int slot, Sub& s) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
#pragma unroll
        for (int e = 0; e < HP; ++e) s.H[j][e] = hfr[slot][(j * HP + e) * 64 + lane];
#pragma unroll
        for (int e = 0; e < D; ++e) s.F[j][e] = hfr[slot][GCH + (j * D + e) * 64 + lane];
      }
    };
#endif
    // H, F chunks in flight: a ring of NR register sets, NR - 1 chunks ahead; NR divides the
    // packet's chunks, so the unrolled packet loop indexes the ring with constants (the consumer
    // has little arithmetic per step to cover the loads' latency with)
    constexpr int NR = DMT_PSPK_RING;
    static_assert((PK / K) % NR == 0 && (NR - 1) * K <= kPadPoints, "ring of whole packets");
#if DMT_PSPK_GLDS
#pragma unroll
    for (int u = 0; u < NGS - 1; ++u) gissue((int64_t)u * K, u);
#else
    Sub sb[NR];
#pragma unroll
    for (int u = 0; u < NR - 1; ++u) load((int64_t)u * K, sb[u]);
#endif
    for (int c = -1; c < nch; ++c) {
      if (c >= 0) {
        const int buf = c & 1;
        v16 ob[D][NV];
#pragma unroll
        for (int q = 0; q < PK / K; ++q) {
          const int64_t i0 = (int64_t)c * PK + q * K;
#if DMT_PSPK_GLDS
          // chunk jj + NGS - 1 into the slot chunk jj - 1 was read from; chunk jj's copies are
          // the oldest loads outstanding but the (NGS - 1)(NIH + NIF) issued after them
          const int jj = c * (PK / K) + q;
          gissue(i0 + (NGS - 1) * K, (jj + NGS - 1) % NGS);
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NGS - 1) * (NIH + NIF)) : "memory");
          Sub cur;
          gread(jj % NGS, cur);
#else
          load(i0 + (NR - 1) * K, sb[(q + NR - 1) % NR]);  // prefetch NR - 1 chunks ahead
          Sub& cur = sb[q % NR];
#endif
          T gv[K];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const int e = q * K + j;
            const bool v = act && i0 + j < nst;
            const T dt = s_dt[buf][e][lane];
            T dW[M];
#pragma unroll
            for (int k = 0; k < M; ++k) dW[k] = s_dw[buf][e][k][lane];
            T xn[D];
#if DMT_PSPK_STUB & 1  // timing stub: the producer alone (no recursion; wrong results)
            const T G = cur.H[j][0] + cur.F[j][0];
#pragma unroll
            for (int p = 0; p < D; ++p) xn[p] = x[p] + dW[p % M] * dt;
#else
            T rr[D], b[D], sdW[D], Mg[D * D], cg[D];
            const T G = g_at<Mdl, T>(LA, cur.H[j], cur.F[j], x, rr, b);
            bool fast = false;
            if constexpr (!Mdl::kLinear && D == M) {
              if (all_unit) {
#pragma unroll
                for (int p = 0; p < D; ++p) sdW[p] = dW[p];
                guide_coeffs_unit<Mdl, T>(cur.H[j], cur.F[j], Mg, cg);
                fast = true;
              }
            }
            if (!fast) {
              sigma_dw<Mdl, T>(LA, dW, sdW);
              guide_coeffs<Mdl, T>(LA, cur.H[j], cur.F[j], Mg, cg);
            }
#pragma unroll
            for (int p = 0; p < D; ++p) xn[p] = x[p];
            euler_step<Mdl, T>(LA.th, Mg, cg, b, dt, sdW, xn);
#if DMT_PSPK_STUB & 32  // timing probe (results unchanged): every step's arithmetic twice
            {
              T x2[D], r2[D], b2[D], M2[D * D], c2[D], H2[HP], F2[D];
#pragma unroll
              for (int p = 0; p < D; ++p) { x2[p] = x[p]; asm volatile("" : "+v"(x2[p])); }
#pragma unroll
              for (int e2 = 0; e2 < HP; ++e2) { H2[e2] = cur.H[j][e2]; asm volatile("" : "+v"(H2[e2])); }
#pragma unroll
              for (int e2 = 0; e2 < D; ++e2) { F2[e2] = cur.F[j][e2]; asm volatile("" : "+v"(F2[e2])); }
              const T G2 = g_at<Mdl, T>(LA, H2, F2, x2, r2, b2);
              guide_coeffs<Mdl, T>(LA, H2, F2, M2, c2);
              euler_step<Mdl, T>(LA.th, M2, c2, b2, dt, sdW, x2);
              asm volatile("" ::"v"(G2));
#pragma unroll
              for (int p = 0; p < D; ++p) asm volatile("" ::"v"(x2[p]));
            }
#endif
#endif
#pragma unroll
            for (int p = 0; p < D; ++p) {
              x[p] = v ? xn[p] : x[p];
              ob[p][e / VE][e % VE] = xn[p];
            }
            gv[j] = G * dt;
          }
          if (i0 + K <= nfull) {
            ps.template add_subtree<Log2<K>::v>(tree_sum<T, K>(gv));
          } else {
#pragma unroll
            for (int j = 0; j < K; ++j)
              if (i0 + j < nst) ps.add(gv[j]);
          }
        }
        if (act && !(DMT_PSPK_STUB & 4)) {  // (timing stub 4: no X° stores)
          if ((int64_t)(c + 1) * PK <= nst) {  // a whole piece
            if (pair && (c & 1) == 0 && (int64_t)(c + 2) * PK <= nst) {  // first half: LDS
#pragma unroll
              for (int p = 0; p < D; ++p)
#pragma unroll
                for (int v = 0; v < NV; ++v) stX[p][v][lane] = ob[p][v];
            } else if (pair && (c & 1) == 1) {  // second half: the lane's whole line
#pragma unroll
              for (int p = 0; p < D; ++p) {
                v16* dst = (v16*)&Xd[pix((int64_t)(c - 1) * PK + 1, p, D)];
#pragma unroll
                for (int v = 0; v < NV; ++v) dst[v] = stX[p][v][lane];
#pragma unroll
                for (int v = 0; v < NV; ++v) dst[NV + v] = ob[p][v];
              }
            } else {
#pragma unroll
              for (int p = 0; p < D; ++p) {
                v16* dst = (v16*)&Xd[pix((int64_t)c * PK + 1, p, D)];
#pragma unroll
                for (int v = 0; v < NV; ++v) dst[v] = ob[p][v];
              }
            }
          } else {
#pragma unroll
            for (int e = 0; e < PK; ++e)
              if ((int64_t)c * PK + e < nst)
#pragma unroll
                for (int p = 0; p < D; ++p) Xd[pix((int64_t)c * PK + e + 1, p, D)] = ob[p][e / VE][e % VE];
          }
        }
      }
      __syncthreads();
    }
    if (act) {
      const T sl = ps.finish();
      bool ok = isfinite(sl);
#pragma unroll
      for (int p = 0; p < D; ++p) ok = ok && isfinite(x[p]);
      a.ll_out[blk] = ok ? (double)(ll + sl) : -INFINITY;
      if (a.success) a.success[blk] = ok ? 1 : 0;
    }
  }
}

// Girsanov log-weight of a stored path (loglikhd!), same summation order as k_block.
template <class Mdl, class T, int K, bool TD = false>
__global__ __launch_bounds__(64) void k_pathll(const BlockArgs<T> a) {
  constexpr int D = Mdl::D, HP = D * (D + 1) / 2;
  int64_t tile, blk;
  if (!map_block(a, tile, blk)) return;
  const int lane = threadIdx.x;
  const int64_t tq = a.tile_qoff[tile];
  auto idx = [&](int64_t q, int c, int C) -> int64_t { return ((tq + q) * C + c) * kLanes + lane; };
  // the path planes (X): row layout or lane packets (plane_ix)
  auto pidx = [&](int64_t q, int c, int C) -> int64_t { return plane_ix(tq + q, c, C, kLanes, lane, a.pk); };
  auto tload = [&](int64_t q) -> T { return a.t_shared ? a.t[q] : a.t[idx(q, 0, 1)]; };
  const int g0 = a.gfirst[blk], g1 = a.glast[blk];
  const bool term = a.term[blk] != 0;
  T ll;
  {
    const int ls = a.selPP[g0] ^ a.law_flip;
    const double* Lr = a.law[ls][0] + (int64_t)g0 * DMT_LAW_STRIDE;
    const T* Xs = a.X[sel_buf(a.selX[g0], a.xs_flip)];
    const int64_t q = a.seg_q[g0];
    T H0[HP], F0[D], x0[D];
#pragma unroll
    for (int c = 0; c < HP; ++c)
      H0[c] = a.H_shared[ls][0] ? a.H[ls][0][q * HP + c] : a.H[ls][0][idx(q, c, HP)];
#pragma unroll
    for (int c = 0; c < D; ++c) F0[c] = a.F[ls][0][idx(q, c, D)];
#pragma unroll
    for (int c = 0; c < D; ++c) x0[c] = Xs[pidx(q, c, D)];
    ll = obs_term<D, T>(H0, F0, x0, (T)Lr[DMT_LAW_C0]);
  }
  for (int g = g0; g <= g1; ++g) {
    const int kind = (!term && g == g1) ? 1 : 0;
    const int ls = (kind ? a.selPPB[g] : a.selPP[g]) ^ a.law_flip;
    Law<Mdl, T> L;
    L.load(a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE);
    const T* __restrict__ Ht = a.H[ls][kind];
    const T* __restrict__ Ft = a.F[ls][kind];
    const int Hsh = a.H_shared[ls][kind];
    const T* __restrict__ Xs = a.X[sel_buf(a.selX[g], a.xs_flip)];
    const int64_t q0 = a.seg_q[g];
    const int nst = a.seg_np[g] - 1;
    constexpr int CA = kAuxCols<D>;  // time-dependent auxiliary law (run_segment)
    const T* At = TD ? a.aux[kind] : nullptr;
    const bool td = TD && At != nullptr && __ballot(L.auxtd) != 0;
    PSum<T> ps;
    ps.init();
    T tcur = tload(q0);
    for (int c0 = 0; c0 < nst; c0 += K) {
      T vt[K], vH[K][HP], vF[K][D], vX[K][D];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        int i = c0 + j;
        i = i < nst ? i : nst - 1;
        const int64_t q = q0 + i;
        vt[j] = tload(q + 1);
#pragma unroll
        for (int c = 0; c < HP; ++c) vH[j][c] = Hsh ? Ht[q * HP + c] : Ht[idx(q, c, HP)];
#pragma unroll
        for (int c = 0; c < D; ++c) { vF[j][c] = Ft[idx(q, c, D)]; vX[j][c] = Xs[pidx(q, c, D)]; }
      }
#pragma unroll
      for (int j = 0; j < K; ++j) {
        if (c0 + j < nst) {
          const T dt = vt[j] - tcur;
          T r[D], b[D];
          T G;
          if constexpr (TD) {
            if (td) {
              T Bq[D * D], bq[D], dq[HP];
              bool trq;
              aux_step<Mdl, T>(L, At + idx(q0 + c0 + j, 0, CA), kLanes, Bq, bq, dq, trq,
                               [](const T* p) { return *p; });
              G = g_at_aux<Mdl, T>(L, vH[j], vF[j], vX[j], r, b, Bq, bq, dq, trq);
            } else {
              G = g_at<Mdl, T>(L, vH[j], vF[j], vX[j], r, b);
            }
          } else {
            G = g_at<Mdl, T>(L, vH[j], vF[j], vX[j], r, b);
          }
          ps.add(G * dt);
          tcur = vt[j];
        }
      }
    }
    ll = ll + ps.finish();
  }
  a.ll_out[blk] = (double)ll;
}

// ================================================================ MAP_WAVE kernels
// One wavefront per block (tw = 1 layout).  Per chunk of 64 consecutive steps:
//   phase A (lane-parallel): lane j loads step c0+j's grid, guiding term and accepted W,
//            draws its normals (Philox + Box–Muller) and writes one LDS row;
//   phase S (serial, uniform): the Euler recursion over the 64 rows, every lane computing
//            the same values from broadcast LDS reads; lane j captures x_j and W°_{j+1};
//   phase B (lane-parallel): lane j evaluates G(t_j, x_j)·dt_j, a 64-lane adjacent-pair
//            xor-shuffle tree gives the chunk sum (= the canonical chunk tree), and every
//            lane stores its point: coalesced writes of the path.
// Cross-lane moves of the adjacent-pair trees: DPP for partners within a 16-lane row (no LDS
// round trip), ds_swizzle for lane ^ 16, ds_bpermute for lane ^ 32.
template <int CTRL, class T>
__device__ __forceinline__ T dpp_mov(T v) {
  if constexpr (sizeof(T) == 8) {
    int2 p = __builtin_bit_cast(int2, v);
    p.x = __builtin_amdgcn_mov_dpp(p.x, CTRL, 0xF, 0xF, false);
    p.y = __builtin_amdgcn_mov_dpp(p.y, CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(T, p);
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF,
                                                          0xF, false));
  }
}
template <int PATTERN, class T>
__device__ __forceinline__ T swizzle_mov(T v) {
  if constexpr (sizeof(T) == 8) {
    int2 p = __builtin_bit_cast(int2, v);
    p.x = __builtin_amdgcn_ds_swizzle(p.x, PATTERN);
    p.y = __builtin_amdgcn_ds_swizzle(p.y, PATTERN);
    return __builtin_bit_cast(T, p);
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), PATTERN));
  }
}
// Adjacent-pair tree over every aligned group of G lanes (G = 2 … 64, a power of two), whole
// wave active: afterwards each lane holds its group's sum, formed exactly as the xor-butterfly
// v + v[lane ^ off], off = 1, 2, …, G/2 (each level adds a lane's partial to its partner's;
// IEEE addition is commutative, so every lane's value is the canonical tree's).  Level 4 and 8
// read the mirrored lane (row_half_mirror, row_mirror): after the lower levels it holds the
// partner's partial.
template <int G, class T>
__device__ __forceinline__ T group_tree_sum(T v) {
  static_assert(G >= 2 && G <= 64 && (G & (G - 1)) == 0, "G: power of two in [2, 64]");
  v = v + dpp_mov<0xB1>(v);                                   // quad_perm(1,0,3,2): lane ^ 1
  if constexpr (G >= 4) v = v + dpp_mov<0x4E>(v);             // quad_perm(2,3,0,1): lane ^ 2
  if constexpr (G >= 8) v = v + dpp_mov<0x141>(v);            // row_half_mirror
  if constexpr (G >= 16) v = v + dpp_mov<0x140>(v);           // row_mirror
  if constexpr (G >= 32) v = v + swizzle_mov<0x401F>(v);      // lane ^ 16 (xor mode)
  if constexpr (G >= 64) v = v + __shfl_xor(v, 32, 64);       // lane ^ 32
  return v;
}
template <class T>
__device__ __forceinline__ T wave_tree_sum(T v) {
  return group_tree_sum<64, T>(v);
}

// ---- MAP_WAVE block kernel: a 2-wave workgroup per block, software-pipelined by chunk.
// Wave S (serial) integrates chunk k from LDS rows {dt, σdW, H, F} and captures x_j per lane;
// it issues no global memory operation.  Wave P, in the same period, first finishes chunk
// k-1 (Girsanov terms G(t_j, x_j)·dt_j, the 64-lane adjacent-pair tree, every global store of
// the chunk, the per-segment success test) and then prepares chunk k+1 (loads, Philox /
// Box–Muller normals, the increment-form pCN dW° = fma(ρ, dW, √(1-ρ²)·√dt·Z), σ·dW°) — all
// lane-parallel.  One __syncthreads per period.  Canonical arithmetic.
// wave S's row per step: {dt, σdW[D], M[D·D], c[D]}, or a model's step map (FHN: {A, e, −ε⁻¹dt},
// Mdl::step_map), padded to an even count
template <class Mdl>
constexpr int wave_row_len() {
  if constexpr (Mdl::kAffineStep) return (Mdl::NS + 1) & ~1;
  else return ((1 + Mdl::D + Mdl::D * Mdl::D + Mdl::D) + 1) & ~1;
}
template <class T, int D, int M, int HP, int NRR>
struct WaveLds {
  static constexpr int NR = NRR;
  static constexpr int NB = 1 + HP + D;                      // dt, H[HP], F[D] (phase B)
  T rows[2][64][NR];
  T rowsB[2][64][NB];
  alignas(16) T xcap[2][64][D];
  T wcap[2][64][M];  // dW° of each step (stored to W° by phase B)
  T xend[2][D];
  T w0[2][M];
};

struct ChunkIt {  // (segment, first step) iterator over a block's chunks of 64 steps
  int g, c0, nst;
  __device__ __forceinline__ void next(const int32_t* seg_np) {
    c0 += 64;
    if (c0 >= nst) { ++g; c0 = 0; nst = ldc(seg_np + g) - 1; }
  }
};

#ifndef DMT_S_UNROLL
#define DMT_S_UNROLL 4
#endif
#ifndef DMT_S_LDS_CAPTURE  // wave S captures x_s through an LDS store of lane 0 (1) or a
#define DMT_S_LDS_CAPTURE 1  // register select in lane s (0)
#endif
#ifndef DMT_S_FULL_UNROLL  // whole 64-step chunks straight-line (1) or the DMT_S_UNROLL loop (0)
#define DMT_S_FULL_UNROLL 1
#endif
#ifndef DMT_S_AHEAD  // rows read this many steps ahead in the straight-line chunk
#define DMT_S_AHEAD 2
#endif
// DIAG (timing diagnostics only, never selected in production): bit 0 = S skips its
// recursion, bit 1 = P skips phase A, bit 2 = P skips phase B.
template <class Mdl, class T, int MODE, int DIAG = 0>
__global__ __launch_bounds__(128) void k_block_wave(const BlockArgs<T> a) {
  constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2;
  using Lds = WaveLds<T, D, M, HP, wave_row_len<Mdl>()>;
  constexpr int NR = Lds::NR;
  __shared__ Lds sh;
  const int lane = threadIdx.x & 63;
  const bool is_s = threadIdx.x < 64;
  const int64_t blk = a.b0 + (int64_t)blockIdx.x;
  if (blk >= a.b1) return;
  const int64_t r = a.blk_rec[blk];
  const int64_t tq = a.tile_qoff[r];
  const int g0 = a.gfirst[blk], g1 = a.glast[blk];
  const bool term = a.term[blk] != 0;
  const T rho = (MODE == MODE_FRESH) ? (T)0 : (T)a.rho[blk];
  const T srho = (MODE == MODE_FRESH) ? (T)1 : (T)a.srho[blk];
  int ktot = 0;
  for (int g = g0; g <= g1; ++g) ktot += (a.seg_np[g] - 1 + 63) / 64;
  auto law_of = [&](int g, int& kind) -> int {
    kind = (!term && g == g1) ? 1 : 0;
    return (kind ? a.selPPB[g] : a.selPP[g]) ^ a.law_flip;
  };
  T x[D];
  {
    const T* Xs = a.X[sel_buf(a.selX[g0], a.xs_flip)];
    const int64_t q = a.seg_q[g0];
#pragma unroll
    for (int p = 0; p < D; ++p) x[p] = Xs[(tq + q) * D + p];
  }

  if (is_s) {
    // ======================= wave S
    ChunkIt it{g0, 0, a.seg_np[g0] - 1};
    Law<Mdl, T> L;
    int lg = -1;
    __syncthreads();  // period 0: P prepares chunk 0
    for (int k = 0; k < ktot; ++k) {
      if (it.g != lg) {
        int kind;
        const int ls = law_of(it.g, kind);
        L.load(a.law[ls][kind] + (int64_t)it.g * DMT_LAW_STRIDE);
        lg = it.g;
      }
      const int cnt = (DIAG & 1) ? 0 : min(64, it.nst - it.c0);
      const T(*rw)[NR] = sh.rows[k & 1];
      T(*const xw)[D] = sh.xcap[k & 1];
#if DMT_S_LDS_CAPTURE
      // lanes past the chunk's last step keep the chunk's start point (as the register capture)
      if (lane >= cnt) {
#pragma unroll
        for (int p = 0; p < D; ++p) xw[lane][p] = x[p];
      }
#else
      T xc[D];
#pragma unroll
      for (int p = 0; p < D; ++p) xc[p] = x[p];
#endif
      // the next step's row is read into registers one step ahead, so the LDS latency overlaps
      // the current step's dependent chain instead of preceding it
      T nx[NR];
#pragma unroll
      for (int i = 0; i < NR; ++i) nx[i] = rw[0][i];
      // step s of the chunk from its row q.  x_s is captured for phase B: lane 0 writes it to
      // the LDS row s (DMT_S_LDS_CAPTURE; an exec-masked store, no VALU), or lane s keeps it in
      // a register (four v_cndmask and a compare per step, on the serial chain's wave)
      auto body = [&](const int s, const T* q) {
#if DMT_S_LDS_CAPTURE
        if (lane == 0) {
          if constexpr (D == 2) {  // one 16/8-byte store at an immediate offset
            typedef T t2 __attribute__((ext_vector_type(2)));
            *reinterpret_cast<t2*>(&xw[s][0]) = t2{x[0], x[1]};
          } else {
#pragma unroll
            for (int p = 0; p < D; ++p) xw[s][p] = x[p];
          }
        }
#else
        const bool mine = lane == s;
#pragma unroll
        for (int p = 0; p < D; ++p) xc[p] = mine ? x[p] : xc[p];
#endif
        if constexpr (Mdl::kAffineStep) {
          Mdl::step_apply(q, x);  // the row is the step's map (Mdl::step_map, phase A)
        } else {
          T b_[D];
          if (!Mdl::kLinear) Mdl::drift(L.th, x, b_);
          euler_step<Mdl, T>(L.th, q + 1 + D, q + 1 + D + D * D, b_, q[0], q + 1, x);
        }
      };
#if DMT_S_FULL_UNROLL
      if (cnt == 64) {
        // a whole chunk (all but a segment's last): straight-line, no loop control, the rows
        // read DMT_S_AHEAD steps ahead into a register ring indexed by constants
        constexpr int AH = DMT_S_AHEAD;
        T rb[AH][NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) rb[0][i] = nx[i];
#pragma unroll
        for (int a = 1; a < AH; ++a)
#pragma unroll
          for (int i = 0; i < NR; ++i) rb[a][i] = rw[a][i];
#pragma unroll
        for (int s = 0; s < 64; ++s) {
          T q[NR];
#pragma unroll
          for (int i = 0; i < NR; ++i) q[i] = rb[s % AH][i];
          const int sn = s + AH < 64 ? s + AH : 63;
#pragma unroll
          for (int i = 0; i < NR; ++i) rb[s % AH][i] = rw[sn][i];
          body(s, q);
        }
      } else
#endif
      {
#pragma unroll DMT_S_UNROLL
        for (int s = 0; s < cnt; ++s) {  // the row read one step ahead
          T q[NR];
#pragma unroll
          for (int i = 0; i < NR; ++i) q[i] = nx[i];
          const int sn = s + 1 < cnt ? s + 1 : s;
#pragma unroll
          for (int i = 0; i < NR; ++i) nx[i] = rw[sn][i];
          body(s, q);
        }
      }
#if !DMT_S_LDS_CAPTURE
#pragma unroll
      for (int p = 0; p < D; ++p) xw[lane][p] = xc[p];
#endif
      const bool seg_end = it.c0 + 64 >= it.nst;
      if (seg_end && lane == 0) {
#pragma unroll
        for (int p = 0; p < D; ++p) sh.xend[k & 1][p] = x[p];
      }
      if (k + 1 < ktot) it.next(a.seg_np);
      __syncthreads();
    }
    __syncthreads();  // period ktot+1: P finishes the last chunk
    return;
  }

  // ======================= wave P
  ChunkIt ia{g0, 0, a.seg_np[g0] - 1};  // chunk being prepared (A)
  ChunkIt ib{g0, 0, a.seg_np[g0] - 1};  // chunk being finished (B)
  T ll;
  {
    const int64_t q = a.seg_q[g0];
    const int lsp = a.selPP[g0] ^ a.law_flip;
    T H0[HP], F0[D];
#pragma unroll
    for (int c = 0; c < HP; ++c)
      H0[c] = a.H_shared[lsp][0] ? a.H[lsp][0][q * HP + c] : a.H[lsp][0][(tq + q) * HP + c];
#pragma unroll
    for (int c = 0; c < D; ++c) F0[c] = a.F[lsp][0][(tq + q) * D + c];
    ll = obs_term<D, T>(H0, F0, x, (T)a.law[lsp][0][(int64_t)g0 * DMT_LAW_STRIDE + DMT_LAW_C0]);
  }
  bool ok = true;
  int stop_after = 0x7fffffff;  // chunks after a failed segment store nothing
  T seg_acc = (T)0;
  Law<Mdl, T> LB;
  int lgb = -1;
  Law<Mdl, T> LA;  // law of the chunk being prepared (sigma, a, linear drift)
  int lga = -1;
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32), c3 = a.salt << 1;

  auto prepare = [&](int k) {  // phase A of chunk k (iterator ia), lane-parallel
    const int g = ia.g, c0 = ia.c0, nst = ia.nst;
    int kind;
    const int ls = law_of(g, kind);
    if (g != lga) {
      LA.load(a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE);
      lga = g;
    }
    const int64_t q0 = a.seg_q[g], row = tq + q0;
    const T* tb = a.t_shared ? a.t + q0 : a.t + row;
    const T* Hb = a.H_shared[ls][kind] ? a.H[ls][kind] + q0 * HP : a.H[ls][kind] + row * HP;
    const T* Fb = a.F[ls][kind] + row * D;
    const T* Wsb = a.W[sel_buf(a.selW[g], a.ws_flip)] + row * M;
    const int cnt = min(64, nst - c0);
    const bool valid = lane < cnt;
    const int i = c0 + (valid ? lane : cnt - 1);
    if (MODE != MODE_RECOMPUTE && c0 == 0 && lane == 0) {
#pragma unroll
      for (int kk = 0; kk < M; ++kk) sh.w0[k & 1][kk] = rho * ((MODE == MODE_FRESH) ? (T)0 : Wsb[kk]);
    }
    const T dt = tb[i + 1] - tb[i];
    T dW[M];
    if (MODE == MODE_RECOMPUTE) {
#pragma unroll
      for (int kk = 0; kk < M; ++kk) dW[kk] = Wsb[(int64_t)(i + 1) * M + kk];
    } else {
      const double* Zg = a.Z ? a.Z + a.st_off[g] * M : nullptr;
      constexpr int NPB = NormPerBlock<T>::v;
      uint32_t have = 0xFFFFFFFFu;
      T zb[NPB] = {};
      const T sdt = sqrt(dt);
#pragma unroll
      for (int kk = 0; kk < M; ++kk) {
        const uint32_t n = (uint32_t)(i * M + kk);
        T z;
        if (Zg) {
          z = (T)Zg[(int64_t)i * M + kk];
        } else {
          if (n / NPB != have) {
            have = n / NPB;
            normal_block(philox4x32_10(U4{have, (uint32_t)g + a.seg_base, a.iter, c3}, k0, k1), zb);
          }
          z = pick_normal<T, NPB>(zb, n % NPB);
        }
        const T w = (MODE == MODE_FRESH) ? (T)0 : Wsb[(int64_t)(i + 1) * M + kk];
        dW[kk] = dfma(rho, w, srho * (sdt * z));
      }
    }
    T Hi[HP], Fi[D], Mg[D * D], cg[D], sdW[D];
#pragma unroll
    for (int c = 0; c < HP; ++c) Hi[c] = Hb[(int64_t)i * HP + c];
#pragma unroll
    for (int c = 0; c < D; ++c) Fi[c] = Fb[(int64_t)i * D + c];
    sigma_dw<Mdl, T>(LA, dW, sdW);
    guide_coeffs<Mdl, T>(LA, Hi, Fi, Mg, cg);
    T* rw = sh.rows[k & 1][lane];
    if constexpr (Mdl::kAffineStep) {  // the step's map, as euler_step forms it
      T sm[Mdl::NS];
      Mdl::step_map(LA.th, Mg, cg, dt, sdW, sm);
#pragma unroll
      for (int e = 0; e < Mdl::NS; ++e) rw[e] = sm[e];
    } else {
      rw[0] = dt;
#pragma unroll
      for (int p = 0; p < D; ++p) rw[1 + p] = sdW[p];
#pragma unroll
      for (int e = 0; e < D * D; ++e) rw[1 + D + e] = Mg[e];
#pragma unroll
      for (int p = 0; p < D; ++p) rw[1 + D + D * D + p] = cg[p];
    }
    T* rb = sh.rowsB[k & 1][lane];
    rb[0] = dt;
#pragma unroll
    for (int c = 0; c < HP; ++c) rb[1 + c] = Hi[c];
#pragma unroll
    for (int c = 0; c < D; ++c) rb[1 + HP + c] = Fi[c];
#pragma unroll
    for (int kk = 0; kk < M; ++kk) sh.wcap[k & 1][lane][kk] = dW[kk];
  };

  auto finish = [&](int k) {  // phase B of chunk k (iterator ib)
    const int g = ib.g, c0 = ib.c0, nst = ib.nst;
    int kind;
    const int ls = law_of(g, kind);
    if (g != lgb) {
      LB.load(a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE);
      lgb = g;
    }
    const int cnt = min(64, nst - c0);
    const bool valid = lane < cnt;
    const T* rw = sh.rowsB[k & 1][lane];
    T Hi[HP], Fi[D], xi[D], rr[D], bb[D];
#pragma unroll
    for (int c = 0; c < HP; ++c) Hi[c] = rw[1 + c];
#pragma unroll
    for (int c = 0; c < D; ++c) { Fi[c] = rw[1 + HP + c]; xi[c] = sh.xcap[k & 1][lane][c]; }
    T G;
    if (a.aux[kind] && LB.auxtd) {  // time-dependent auxiliary law: step i's B̃(t_i), β̃(t_i)
      constexpr int CA = kAuxCols<D>;
      const int i = c0 + (valid ? lane : cnt - 1);
      T Bq[D * D], bq[D], dq[HP];
      bool trq;
      aux_step<Mdl, T>(LB, a.aux[kind] + (tq + a.seg_q[g] + i) * CA, 1, Bq, bq, dq, trq,
                       [](const T* p) { return *p; });
      G = g_at_aux<Mdl, T>(LB, Hi, Fi, xi, rr, bb, Bq, bq, dq, trq);
    } else {
      G = g_at<Mdl, T>(LB, Hi, Fi, xi, rr, bb);
    }
    const bool inll = MODE != MODE_RECOMPUTE || c0 + lane < nst - a.ll_skip;  // skip
    const T csum = wave_tree_sum<T>((valid && inll) ? G * rw[0] : (T)0);
    seg_acc = seg_acc + (csum + (T)0);
    const bool seg_end = c0 + 64 >= nst;
    if (k <= stop_after) {
      const int64_t row = tq + a.seg_q[g];
      T* Xdb = a.X[sel_buf(a.selX[g], a.xd_flip)] + row * D;
      T* Wdb = a.W[sel_buf(a.selW[g], a.wd_flip)] + row * M;
      if (valid) {
        const int i = c0 + lane;
#pragma unroll
        for (int p = 0; p < D; ++p) Xdb[(int64_t)i * D + p] = xi[p];
        if (MODE != MODE_RECOMPUTE) {
#pragma unroll
          for (int kk = 0; kk < M; ++kk) Wdb[(int64_t)(i + 1) * M + kk] = sh.wcap[k & 1][lane][kk];
        }
      }
      if (lane == 0) {
        if (MODE != MODE_RECOMPUTE && c0 == 0) {
#pragma unroll
          for (int kk = 0; kk < M; ++kk) Wdb[kk] = sh.w0[k & 1][kk];
        }
        if (seg_end) {
#pragma unroll
          for (int p = 0; p < D; ++p) Xdb[(int64_t)nst * D + p] = sh.xend[k & 1][p];
        }
      }
    }
    if (seg_end) {
      if (k <= stop_after) {
        bool sok = isfinite(seg_acc);
#pragma unroll
        for (int p = 0; p < D; ++p) sok = sok && isfinite(sh.xend[k & 1][p]);
        if (sok) {
          ll = ll + seg_acc;
        } else {
          ok = false;
          stop_after = k;
        }
      }
      seg_acc = (T)0;
    }
  };

  for (int p = 0; p <= ktot; ++p) {
    if (p >= 2) {
      if (!(DIAG & 4)) finish(p - 2);
      if (p - 2 + 1 < ktot) ib.next(a.seg_np);
    }
    if (p < ktot) {
      if (!(DIAG & 2)) prepare(p);
      if (p + 1 < ktot) ia.next(a.seg_np);
    }
    __syncthreads();
  }
  finish(ktot - 1);
  __syncthreads();
  if (lane == 0) {
    a.ll_out[blk] = ok ? (double)ll : -INFINITY;
    if (a.success) a.success[blk] = ok ? 1 : 0;
  }
}

// ---- linear-drift block kernels: parallel-in-time Euler recursion.
// With a linear drift (OU) every guided Euler step is an affine map x ↦ A_i x + e_i whose
// coefficients do not depend on x.  ONE WAVEFRONT OWNS ONE BLOCK (no barriers, no serial
// carry between waves); a workgroup holds ScanCfg::WPB independent waves (one per SIMD).
// A segment is cut into chunks of kSChunk = 512 steps; per chunk:
//   phase 1 (coalesced, lane j ↔ step 64k + j, k = 0..7): normals (Philox/Box–Muller), the
//            pCN increments, σ·dW°, the guiding coefficients and the step maps → LDS, W° stored;
//   phase 2 (runs, lane j ↔ steps 8j … 8j+7): the lane composes its 8 step maps into one run
//            map, an inclusive Kogge–Stone scan over the 64 run maps gives every run's start
//            point, and the lane applies its step maps one by one → points to LDS;
//   phase 3 (coalesced again): points back, Girsanov terms G·dt, the 64-step adjacent-pair tree
//            sums (the canonical chunk sums), coalesced stores of the path.
// The scan costs one 6-level Kogge–Stone per 8 steps (instead of per step) and the chunk carry
// is the scan itself.
constexpr int kRun = 8;                                 // steps per lane run
constexpr int kSChunk = 64 * kRun;                      // steps per scan chunk
constexpr int kSStride = kSChunk + kSChunk / kRun + 8;  // LDS row: 512 steps, a pad per 8, end point

// LDS slot of chunk step s: one pad double per 8 steps, so that the run-order reads of phase 2
// (lane stride 9 doubles) and the coalesced phase-1/3 accesses are both (nearly) conflict-free
__device__ __forceinline__ int lds_ix(int s) { return s + (s >> 3); }

template <int D, class T>
struct ScanLds {
  static constexpr int NA = D * D + D;
  T map[NA][kSStride];  // step maps A (D×D), e (D) of the chunk, SoA
  T pt[D][kSStride];    // pre-step points of the chunk (+ its end point at lds_ix(cnt))
};
template <int D, class T>
struct ScanCfg {  // waves (= blocks) per workgroup: as many as 160 KiB of LDS allow, ≤ 4
  static constexpr int kBytes = (int)sizeof(ScanLds<D, T>);
  static constexpr int WPB = (4 * kBytes <= 160 * 1024) ? 4 : (2 * kBytes <= 160 * 1024) ? 2 : 1;
};

// Raw cross-lane read: the value of lane `src` (ds_bpermute, no range fix-up; the caller
// selects).  `addr` = 4 * src lane.
__device__ __forceinline__ double lane_read(double v, int addr) {
  const int2 p = __builtin_bit_cast(int2, v);
  int2 r;
  r.x = __builtin_amdgcn_ds_bpermute(addr, p.x);
  r.y = __builtin_amdgcn_ds_bpermute(addr, p.y);
  return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ float lane_read(float v, int addr) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(addr, __builtin_bit_cast(int, v)));
}

// DPP moves (VALU, no LDS round trip): lane l receives lane src(l) of the pattern CTRL in the
// rows ROWMASK enables; the other lanes keep their own value (bound_ctrl off, old = v).
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_mov(double v) {
  const int2 p = __builtin_bit_cast(int2, v);
  int2 r;
  r.x = __builtin_amdgcn_update_dpp(p.x, p.x, CTRL, ROWMASK, 0xF, false);
  r.y = __builtin_amdgcn_update_dpp(p.y, p.y, CTRL, ROWMASK, 0xF, false);
  return __builtin_bit_cast(double, r);
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_mov(float v) {
  const int p = __builtin_bit_cast(int, v);
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(p, p, CTRL, ROWMASK, 0xF, false));
}
constexpr int kDppRowShr = 0x110;    // row_shr:n = kDppRowShr + n (within rows of 16 lanes)
constexpr int kDppRowBcast15 = 0x142;  // lane 15 of a row → the next row
constexpr int kDppRowBcast31 = 0x143;  // lane 31 → rows 2 and 3
[[maybe_unused]] constexpr int kDppWaveShr1 = 0x138;    // lane l − 1 → lane l

// One level of the wave's inclusive scan of affine maps: lanes with `take` compose their map
// after the map DPP pattern CTRL brings them (An = own ∘ received, affine_compose's order).
template <int CTRL, int ROWMASK, int D, class T>
__device__ __forceinline__ void affine_scan_level(T* RA, T* Re, const bool take) {
  T Ap[D * D], ep[D], An[D * D], en[D];
#pragma unroll
  for (int c = 0; c < D * D; ++c) Ap[c] = dpp_mov<CTRL, ROWMASK>(RA[c]);
#pragma unroll
  for (int c = 0; c < D; ++c) ep[c] = dpp_mov<CTRL, ROWMASK>(Re[c]);
  affine_compose<D, T>(RA, Re, Ap, ep, An, en);
#pragma unroll
  for (int c = 0; c < D * D; ++c) RA[c] = take ? An[c] : RA[c];
#pragma unroll
  for (int c = 0; c < D; ++c) Re[c] = take ? en[c] : Re[c];
}
// Inclusive scan of the 64 lanes' maps (lane j ← map_j ∘ … ∘ map_0).  DMT_SCAN_DPP = 1: the DPP
// tree the oracle restates with ORC_SCAN_DPP = 1 (dmt_oracle.c wave_scan_dpp) — Kogge–Stone
// within each row of 16 lanes (shifts 1, 2, 4, 8), then rows 1 and 3 compose after lane 15 /
// lane 47 (row_bcast:15), then rows 2 and 3 after lane 31 (row_bcast:31); every level is VALU
// work, no ds_bpermute round trip on the chain.  0: the 64-lane Kogge–Stone over ds_bpermute.
#ifndef DMT_SCAN_DPP  // 0: the 64-lane Kogge–Stone over ds_bpermute (oracle ORC_SCAN_DPP = 0)
#define DMT_SCAN_DPP 0
#endif
template <int D, class T>
__device__ __forceinline__ void wave_affine_scan(T* RA, T* Re, const int lane) {
#if !DMT_SCAN_DPP
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T Ap[D * D], ep[D], An[D * D], en[D];
    const int src = 4 * (lane - o);  // lanes < o read garbage and keep their own map
#pragma unroll
    for (int c = 0; c < D * D; ++c) Ap[c] = lane_read(RA[c], src);
#pragma unroll
    for (int c = 0; c < D; ++c) ep[c] = lane_read(Re[c], src);
    affine_compose<D, T>(RA, Re, Ap, ep, An, en);
    const bool take = lane >= o;
#pragma unroll
    for (int c = 0; c < D * D; ++c) RA[c] = take ? An[c] : RA[c];
#pragma unroll
    for (int c = 0; c < D; ++c) Re[c] = take ? en[c] : Re[c];
  }
  return;
#endif
  const int rl = lane & 15;
  affine_scan_level<kDppRowShr + 1, 0xF, D, T>(RA, Re, rl >= 1);
  affine_scan_level<kDppRowShr + 2, 0xF, D, T>(RA, Re, rl >= 2);
  affine_scan_level<kDppRowShr + 4, 0xF, D, T>(RA, Re, rl >= 4);
  affine_scan_level<kDppRowShr + 8, 0xF, D, T>(RA, Re, rl >= 8);
  affine_scan_level<kDppRowBcast15, 0xA, D, T>(RA, Re, (lane & 16) != 0);
  affine_scan_level<kDppRowBcast31, 0xC, D, T>(RA, Re, lane >= 32);
}
// The exclusive form's start points: lane l receives lane l − 1's value (lane 0: its own)
template <class T>
__device__ __forceinline__ T wave_shr1(T v) {
#if DMT_SCAN_DPP
  return dpp_mov<kDppWaveShr1, 0xF>(v);
#else
  return lane_read(v, 4 * ((int)(threadIdx.x & 63) - 1));
#endif
}

// store_row with nontemporal stores (the path stores of the resident MCMC kernels: written
// once per iteration, read by no later iteration of the launch, DMT_PC_NT_STORES)
template <int N, class T>
__device__ __forceinline__ void store_row_nt(T* p, const T* v) {
  if constexpr (std::is_same<T, double>::value && N % 2 == 0) {
    typedef double d2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int c = 0; c < N; c += 2) __builtin_nontemporal_store(d2{v[c], v[c + 1]}, (d2*)(p + c));
  } else {
#pragma unroll
    for (int c = 0; c < N; ++c) __builtin_nontemporal_store(v[c], p + c);
  }
}
// Store one point's N components (16-byte stores when N is even and T is double).
template <int N, class T>
__device__ __forceinline__ void store_row(T* p, const T* v) {
#if defined(DMT_PATH_STORE_WT)  // experiment: write-through path stores
#pragma unroll
  for (int c = 0; c < N; ++c) __hip_atomic_store(p + c, v[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return;
#endif
  if constexpr (std::is_same<T, double>::value && N % 2 == 0) {
#pragma unroll
    for (int c = 0; c < N; c += 2) *reinterpret_cast<double2*>(p + c) = make_double2(v[c], v[c + 1]);
  } else {
#pragma unroll
    for (int c = 0; c < N; ++c) p[c] = v[c];
  }
}

#ifndef DMT_PC_NT_STORES
#define DMT_PC_NT_STORES 1
#endif
template <int N, class T>
__device__ __forceinline__ void store_row_pc(T* p, const T* v) {
#if DMT_PC_NT_STORES
  store_row_nt<N, T>(p, v);
#else
  store_row<N, T>(p, v);
#endif
}

// Path selectors of the scan kernels: read from the ensemble arrays (one launch per call;
// scalar loads) or kept as wave-uniform bit masks (k_mcmc_scan flips them between its
// iterations; bit g - g0 = selector of segment g).
struct SelGlobal {
  const uint8_t* sx;
  const uint8_t* sw;
  // u's buffer (0/1: linear models keep two path buffers, u° = u ^ 1)
  __device__ __forceinline__ int x(int g) const { return sel_u(ldc(sx + g)); }
  __device__ __forceinline__ int w(int g) const { return sel_u(ldc(sw + g)); }
};
struct SelMask {
  uint64_t mx, mw;
  int g0;
  __device__ __forceinline__ int x(int g) const { return (int)((mx >> (g - g0)) & 1u); }
  __device__ __forceinline__ int w(int g) const { return (int)((mw >> (g - g0)) & 1u); }
};

// A value every lane of the wave holds (the compiler cannot always prove it): lane 0's copy
// in SGPRs, so that branches, selectors and pointers derived from it stay scalar.
__device__ __forceinline__ double wave_uniform(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ float wave_uniform(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, v)));
}
// lane `l`'s value (l wave-uniform), in SGPRs
__device__ __forceinline__ double lane_value(double v, int l) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ float lane_value(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(uint32_t, v), l));
}

__device__ __forceinline__ void wave_lds_sync() {
  // LDS accesses of one wave are performed in order; this only keeps the compiler from moving
  // an access across the phase boundary (other lanes' data)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef DMT_AUX_CHECK
#define DMT_AUX_CHECK 0
#endif
#if DMT_AUX_CHECK
// Measurement build (DMT_AUX_CHECK=1): an aux-table read outside the table is not made; the
// first kAuxDbg such reads are recorded (dmt_debug_aux_check).
constexpr int kAuxDbg = 16;
static __device__ unsigned long long g_aux_dbg[1 + 8 * kAuxDbg];
__device__ __forceinline__ void aux_check_record(int64_t blk, int g, int kind, int64_t row,
                                                 int64_t i, int c0, int cnt, int64_t nonnull) {
  const unsigned long long n = atomicAdd(&g_aux_dbg[0], 1ull);
  if (n < kAuxDbg) {
    unsigned long long* r = &g_aux_dbg[1 + 8 * n];
    r[0] = (unsigned long long)blk; r[1] = (unsigned long long)g; r[2] = (unsigned long long)kind;
    r[3] = (unsigned long long)row; r[4] = (unsigned long long)i; r[5] = (unsigned long long)c0;
    r[6] = (unsigned long long)cnt; r[7] = (unsigned long long)nonnull;
  }
}
#endif

// One block's draw / re-solve by one wave; every lane returns the block's ll and success.
// TD: time-dependent auxiliary laws (an aux table is present) — the recursion is the target
// law's and does not change; phase 3 takes step i's B̃(t_i), β̃(t_i) (and a − ã(t_i)) in G where
// the segment's law record says so (DMT_LAW_AUXTD).
template <class Mdl, class T, int MODE, class Sel, bool TD = false>
__device__ __forceinline__ void scan_block(const BlockArgs<T>& a, const int64_t blk,
                                           const uint32_t iter, const Sel& sel,
                                           ScanLds<Mdl::D, T>& S, T& ll_res, bool& ok_res) {
  constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2;
  static_assert(Mdl::kLinear, "scan_block needs a linear drift");
  // D ≤ 2: the phase-1 guiding-table values stay in registers for phase 3; D = 3 re-reads them
  constexpr bool kKeep = D <= 2;
  const int lane = threadIdx.x & 63;
  const BlkInfo* bi = a.binfo + blk;
  const int64_t tq = ldc(&bi->tq);
  const int g0 = ldc(&bi->g0), g1 = ldc(&bi->g1);
  const int bq0 = ldc(&bi->q0);
  const bool term = ldc(&bi->term) != 0;
  const T rho = (MODE == MODE_FRESH) ? (T)0 : (T)ldc(&bi->rho);
  const T srho = (MODE == MODE_FRESH) ? (T)1 : (T)ldc(&bi->srho);
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32), c3 = a.salt << 1;
  // law slot / kind of segment g (uniform)
  auto law_sel = [&](int g, int& kind) -> int {
    kind = (!term && g == g1) ? 1 : 0;
    return (kind ? ldc(a.selPPB + g) : ldc(a.selPP + g)) ^ a.law_flip;
  };
  // block start point (u's path; every lane holds it) and loglikhd_obs of the first segment
  T xc[D], ll;
  {
    const T* Xs = a.X[sel.x(g0) ^ a.xs_flip];
    const int lsp = ldc(a.selPP + g0) ^ a.law_flip;
    const int64_t q = bq0;
    T H0[HP], F0[D];
#pragma unroll
    for (int p = 0; p < D; ++p) xc[p] = wave_uniform(Xs[(tq + q) * D + p]);
#pragma unroll
    for (int c = 0; c < HP; ++c)
      H0[c] = a.H_shared[lsp][0] ? a.H[lsp][0][q * HP + c] : a.H[lsp][0][(tq + q) * HP + c];
#pragma unroll
    for (int c = 0; c < D; ++c) F0[c] = a.F[lsp][0][(tq + q) * D + c];
    const T c00 = (T)ldc(a.law[lsp][0] + (int64_t)g0 * DMT_LAW_STRIDE + DMT_LAW_C0);
    ll = obs_term<D, T>(H0, F0, xc, c00);
  }
  bool ok = true;
  for (int g = g0; g <= g1; ++g) {
    int kind;
    const int ls = law_sel(g, kind);
    const int nst = ldc(a.seg_np + g) - 1;
    const int64_t q0 = g == g0 ? (int64_t)bq0 : (int64_t)ldc(a.seg_q + g);
    const int64_t row = tq + q0;
    const T* tb = a.t_shared ? a.t + q0 : a.t + row;
    const T* Hb = a.H_shared[ls][kind] ? a.H[ls][kind] + q0 * HP : a.H[ls][kind] + row * HP;
    const T* Fb = a.F[ls][kind] + row * D;
    Law<Mdl, T> LA;
    LA.load(a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE);
    const T* Wsb = a.W[sel.w(g) ^ a.ws_flip] + row * M;
    T* const Xdb = a.X[sel.x(g) ^ a.xd_flip] + row * D;
    T* const Wdb = a.W[sel.w(g) ^ a.wd_flip] + row * M;
    const double* Zg = a.Z ? a.Z + ldc(a.st_off + g) * M : nullptr;
    // the segment's aux-table rows (TD): one uniform base per segment, not a kernel-argument
    // slot chosen by `kind` and re-read inside the chunk loop
    const T* const auxb = (TD && LA.auxtd) ? a.aux[kind] + row * kAuxCols<D> : nullptr;
    if (MODE != MODE_RECOMPUTE && lane == 0) {  // W°(t0) = ρ·W(t0)
      T w0v[M];
#pragma unroll
      for (int k = 0; k < M; ++k) w0v[k] = rho * ((MODE == MODE_FRESH) ? (T)0 : Wsb[k]);
      store_row<M, T>(Wdb, w0v);
    }
    T seg_acc = (T)0;
    for (int c0 = 0; c0 < nst; c0 += kSChunk) {
      const int cnt = min(kSChunk, nst - c0);
      // ---- phase 1 (coalesced): step maps of the chunk → LDS.  Every input of the chunk is
      // loaded first: the W° stores below may alias u's W as far as the compiler knows, so a
      // load placed after one of them could not be hoisted above it (one exposed memory
      // latency per row otherwise)
      T Hk[kRun][HP], Fk[kRun][D], dtk[kRun], Wk[kRun][M], Zk[kRun][M];
#pragma unroll
      for (int k = 0; k < kRun; ++k) {
        const int s = 64 * k + lane;
        const int i = c0 + (s < cnt ? s : cnt - 1);
        dtk[k] = tb[i + 1] - tb[i];
#pragma unroll
        for (int c = 0; c < HP; ++c) Hk[k][c] = Hb[(int64_t)i * HP + c];
#pragma unroll
        for (int c = 0; c < D; ++c) Fk[k][c] = Fb[(int64_t)i * D + c];
#pragma unroll
        for (int kk = 0; kk < M; ++kk) {
          Wk[k][kk] = (MODE == MODE_FRESH) ? (T)0 : Wsb[(int64_t)(i + 1) * M + kk];
          Zk[k][kk] = (MODE != MODE_RECOMPUTE && Zg) ? (T)Zg[(int64_t)i * M + kk] : (T)0;
        }
      }
#pragma unroll
      for (int k = 0; k < kRun; ++k) {
        const int s = 64 * k + lane;
        const bool v = s < cnt;
        const int i = c0 + (v ? s : cnt - 1);
        const T dt = dtk[k];
        T dW[M];
        if (MODE == MODE_RECOMPUTE) {
#pragma unroll
          for (int kk = 0; kk < M; ++kk) dW[kk] = Wk[k][kk];
        } else {
          constexpr int NPB = NormPerBlock<T>::v;
          uint32_t have = 0xFFFFFFFFu;
          T zb[NPB] = {};
          const T sdt = sqrt(dt);
#pragma unroll
          for (int kk = 0; kk < M; ++kk) {
            const uint32_t n = (uint32_t)(i * M + kk);
            T z;
            if (Zg) {
              z = Zk[k][kk];
            } else {
              if (n / NPB != have) {
                have = n / NPB;
                normal_block(philox4x32_10(U4{have, (uint32_t)g + a.seg_base, iter, c3}, k0, k1), zb);
              }
              z = pick_normal<T, NPB>(zb, n % NPB);
            }
            dW[kk] = dfma(rho, Wk[k][kk], srho * (sdt * z));
          }
          if (v) store_row<M, T>(Wdb + (int64_t)(i + 1) * M, dW);
        }
        T sdW[D], Mg[D * D], cg[D], A[D * D], e[D];
        sigma_dw<Mdl, T>(LA, dW, sdW);
        guide_coeffs<Mdl, T>(LA, Hk[k], Fk[k], Mg, cg);
        affine_step<D, T>(Mg, cg, dt, sdW, A, e);
        const int li = lds_ix(s);
#pragma unroll
        for (int c = 0; c < D * D; ++c) S.map[c][li] = v ? A[c] : (c % (D + 1) == 0 ? (T)1 : (T)0);
#pragma unroll
        for (int c = 0; c < D; ++c) S.map[D * D + c][li] = v ? e[c] : (T)0;
      }
      wave_lds_sync();
      // ---- phase 2 (runs): run maps, Kogge–Stone scan, start points, points
      const int nv = max(0, min(kRun, cnt - kRun * lane));  // valid steps of this lane's run
      T A8[kRun][D * D], e8[kRun][D];
#pragma unroll
      for (int r = 0; r < kRun; ++r) {
        const int li = lds_ix(kRun * lane + r);
#pragma unroll
        for (int c = 0; c < D * D; ++c) A8[r][c] = S.map[c][li];
#pragma unroll
        for (int c = 0; c < D; ++c) e8[r][c] = S.map[D * D + c][li];
      }
      T RA[D * D], Re[D];
#pragma unroll
      for (int c = 0; c < D * D; ++c) RA[c] = A8[0][c];
#pragma unroll
      for (int c = 0; c < D; ++c) Re[c] = e8[0][c];
      // run map = step_7 ∘ … ∘ step_0; identity maps past the segment end (exact for finite
      // maps; only the lane holding the last step has any, and its run map feeds only the
      // prefixes of lanes with no valid step, so no stored value depends on them)
#pragma unroll
      for (int r = 1; r < kRun; ++r) {
        T An[D * D], en[D];
        affine_compose<D, T>(A8[r], e8[r], RA, Re, An, en);
#pragma unroll
        for (int c = 0; c < D * D; ++c) RA[c] = An[c];
#pragma unroll
        for (int c = 0; c < D; ++c) Re[c] = en[c];
      }
      // inclusive scan over the lanes: lane j ← run_j ∘ … ∘ run_0
      wave_affine_scan<D, T>(RA, Re, lane);
      // start of run j = prefix_{j-1} applied to the chunk start (lane 0: the chunk start)
      T x[D];
      {
        T y[D];
        affine_apply<D, T>(RA, Re, xc, y);
#pragma unroll
        for (int p = 0; p < D; ++p) {
          const T up = wave_shr1<T>(y[p]);
          x[p] = lane == 0 ? xc[p] : up;
        }
      }
#pragma unroll
      for (int r = 0; r < kRun; ++r) {
        if (r < nv) {
          const int li = lds_ix(kRun * lane + r);
#pragma unroll
          for (int p = 0; p < D; ++p) S.pt[p][li] = x[p];
          T xn[D];
          affine_apply<D, T>(A8[r], e8[r], x, xn);
#pragma unroll
          for (int p = 0; p < D; ++p) x[p] = xn[p];
        }
      }
      if (nv > 0 && kRun * lane + nv == cnt) {  // the lane holding the chunk's last step
#pragma unroll
        for (int p = 0; p < D; ++p) S.pt[p][lds_ix(cnt)] = x[p];
      }
      wave_lds_sync();
      // ---- phase 3 (coalesced): Girsanov terms, 64-step chunk sums, path stores.  The 8 rows'
      // terms first, then their 8 xor-shuffle trees level by level (independent shuffles in
      // flight together instead of 8 dependent 6-level chains), then the stores
      T gk[kRun], xk[kRun][D];
#pragma unroll
      for (int k = 0; k < kRun; ++k) {
        const int s = 64 * k + lane;
        const bool v = s < cnt;
        const int li = lds_ix(s);
#pragma unroll
        for (int p = 0; p < D; ++p) xk[k][p] = S.pt[p][li];
        T Hi[HP], Fi[D], dt;
        if constexpr (kKeep) {
          dt = dtk[k];
#pragma unroll
          for (int c = 0; c < HP; ++c) Hi[c] = Hk[k][c];
#pragma unroll
          for (int c = 0; c < D; ++c) Fi[c] = Fk[k][c];
        } else {
          const int i = c0 + (v ? s : cnt - 1);
          dt = tb[i + 1] - tb[i];
#pragma unroll
          for (int c = 0; c < HP; ++c) Hi[c] = Hb[(int64_t)i * HP + c];
#pragma unroll
          for (int c = 0; c < D; ++c) Fi[c] = Fb[(int64_t)i * D + c];
        }
        T rr[D], bb[D];
        T G;
        if constexpr (TD) {
          if (LA.auxtd) {  // uniform: the segment's law
            constexpr int CA = kAuxCols<D>;
            const int i = c0 + (v ? s : cnt - 1);
            T Bq[D * D], bq[D], dq[HP];
            bool trq;
#if DMT_AUX_CHECK
            const int64_t ix = (row + i) * CA;
            if (a.aux[kind] == nullptr || ix < 0 || ix + CA > a.aux_n) {
              aux_check_record(blk, g, kind, row, i, c0, cnt, (int64_t)(a.aux[kind] != nullptr));
              G = g_at<Mdl, T>(LA, Hi, Fi, xk[k], rr, bb);
            } else
#endif
            {
            aux_step<Mdl, T>(LA, auxb + (int64_t)i * CA, 1, Bq, bq, dq, trq,
                             [](const T* p) { return *p; });
            G = g_at_aux<Mdl, T>(LA, Hi, Fi, xk[k], rr, bb, Bq, bq, dq, trq);
            }
          } else {
            G = g_at<Mdl, T>(LA, Hi, Fi, xk[k], rr, bb);
          }
        } else {
          G = g_at<Mdl, T>(LA, Hi, Fi, xk[k], rr, bb);
        }
        const bool inll = MODE != MODE_RECOMPUTE || c0 + s < nst - a.ll_skip;  // skip
        gk[k] = (v && inll) ? G * dt : (T)0;
      }
#pragma unroll
      for (int k = 0; k < kRun; ++k) gk[k] = wave_tree_sum<T>(gk[k]);
#pragma unroll
      for (int k = 0; k < kRun; ++k)
        if (64 * k < cnt) seg_acc = seg_acc + (wave_uniform(gk[k]) + (T)0);  // uniform
#pragma unroll
      for (int k = 0; k < kRun; ++k) {
        const int s = 64 * k + lane;
        if (s < cnt) store_row<D, T>(Xdb + (int64_t)(c0 + s) * D, xk[k]);
      }
#pragma unroll
      for (int p = 0; p < D; ++p) xc[p] = wave_uniform(S.pt[p][lds_ix(cnt)]);
      wave_lds_sync();
    }
    if (lane == 0) store_row<D, T>(Xdb + (int64_t)nst * D, xc);
    bool sok = isfinite(seg_acc);
#pragma unroll
    for (int p = 0; p < D; ++p) sok = sok && isfinite(xc[p]);
    if (!sok) {  // a failed segment ends the block (later segments untouched)
      ok = false;
      break;
    }
    ll = ll + seg_acc;
  }
  ll_res = ll;
  ok_res = ok;
}

// The persistent kernel's time-dependent iterations call scan_block out of line (DESIGN.md §7,
// "the round-4 k_mcmc_scan<TD> fault"): inlined into k_mcmc_scan's iteration loop, the round-4/5
// TD body gave wrong Girsanov terms from the third iteration on, or an illegal address,
// depending on the build; the cause was not found (its SGPR spill lanes are consistent,
// scripts/spill_flow.py), so the inline form is no longer built and dmt_mcmc_run with an aux
// table runs the per-iteration kernels unless DMT_MCMC_SCAN_TD=1 (dmt_runtime.hip).
template <class Mdl, class T, int MODE, class Sel, bool TD>
__device__ __attribute__((noinline)) void scan_block_ni(const BlockArgs<T>& a, const int64_t blk,
                                                       const uint32_t iter, const Sel& sel,
                                                       ScanLds<Mdl::D, T>& S, T& ll_res,
                                                       bool& ok_res) {
  scan_block<Mdl, T, MODE, Sel, TD>(a, blk, iter, sel, S, ll_res, ok_res);
}

template <class Mdl, class T, int MODE, bool TD = false>
__global__ __launch_bounds__((64 * ScanCfg<Mdl::D, T>::WPB), 1) void k_block_scan(const BlockArgs<T> a) {
  using Cfg = ScanCfg<Mdl::D, T>;
  __shared__ ScanLds<Mdl::D, T> lds[Cfg::WPB];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t blk = a.b0 + (int64_t)blockIdx.x * Cfg::WPB + w;
  if (blk >= a.b1) return;  // whole wave: the waves of a workgroup never synchronise
  T ll;
  bool ok;
  scan_block<Mdl, T, MODE, SelGlobal, TD>(a, blk, a.iter, SelGlobal{a.selX, a.selW}, lds[w], ll, ok);
  if ((threadIdx.x & 63) == 0) {
    a.ll_out[blk] = ok ? (double)ll : -INFINITY;
    if (a.success) a.success[blk] = ok ? 1 : 0;
  }
}

// The fetch_ll trees of every iteration of a persistent run, formed inside the launch (no
// separate tree launch), as the complete adjacent-pair tree over the zero-padded blocks of
// launch_block_sum (padding further with zeros changes nothing but the sign of a zero, and the
// ll sums are canonicalised with + 0.0), in three levels over the rows (iteration, component)
// of part[n_iter][3][nb]:
//   1. every workgroup folds its WPB consecutive leaves (the blocks of its waves) → node1;
//   2. the last workgroup to finish of each group of kTreeGroup workgroups (an arrival counter
//      per group) folds the group's node1s → node2 (16-lane DPP trees, all rows at once);
//   3. the last group to finish (one more counter) folds every row's node2s → out3.
// Levels 2-3 run on the workgroups that arrive last, so the reads of other CUs' nodes are
// spread over the groups instead of one CU reading them all.  Hand-offs without a release
// fence (an agent-scope release writes back the XCD L2's dirty lines — here the run's paths:
// ≈25 µs per 20-iteration C2 launch measured): nodes are stored write-through (relaxed
// agent-scope atomic stores, sc1), every storing wave drains its stores, one lane per workgroup
// adds to the arrival counter (agent-scope atomic) after a workgroup barrier, and the last
// arriver — told by the value its add returned — reads the nodes with sc1 loads
// (MI355X_MICROARCH.md, inter-workgroup visibility: one workgroup per CU, hipMalloc memory).
constexpr int kTreeGroup = 16;

__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// drain this wave's stores, join the workgroup, one lane adds to *cnt; true in every thread of
// the workgroup whose add completed the count `expect`
// The form is the guide's measured one (MI355X_MICROARCH.md, inter-workgroup visibility,
// "Hand-offs measured with sc1 loads", row 1: sc1 stores drained by every storing wave, one
// lane per workgroup adds to one unsharded counter after a barrier, the last adder — told by
// its add's return — loads with sc1; hipMalloc memory, one workgroup per CU), not an API
// guarantee.  DMT_TREE_FENCES=1 (measurement build) adds the API's agent-scope release before
// the add and acquire after it (their price per C2 launch).
#ifndef DMT_TREE_FENCES
#define DMT_TREE_FENCES 0
#endif
__device__ __forceinline__ bool arrive_last(unsigned* cnt, unsigned expect, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
#if DMT_TREE_FENCES
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    *s_flag = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                      expect - 1 ? 1 : 0;
#if DMT_TREE_FENCES
    if (*s_flag) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#endif
  }
  __syncthreads();
  return *s_flag != 0;
}

#ifndef DMT_TREE_ONEHOP  // persistent_tree_tail: one arrival hop for <= 256 workgroups (1) —
#define DMT_TREE_ONEHOP 0  // measured 2 µs slower per C2 launch than the two hops (profiles/r03end)
#endif
// nodes: node1 [rows][ng] then node2 [rows][ng2]; counters: [ng2] group counters then the top
// counter, zero on entry and left zero.  WPB = blocks (tree leaves) per workgroup, NW = waves
// per workgroup (every thread of the workgroup calls this)
template <int WPB, int NW = WPB, bool L1 = false>
__device__ __forceinline__ void persistent_tree_tail(const double* __restrict__ part,
                                                     double* __restrict__ nodes, int64_t nb,
                                                     int64_t n_iter,
                                                     unsigned* __restrict__ counters,
                                                     double* __restrict__ out3) {
  __shared__ int s_flag;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr int NT = 64 * NW;
  const int64_t ng = (nb + WPB - 1) / WPB, ng2 = (ng + kTreeGroup - 1) / kTreeGroup;
  const int64_t x = blockIdx.x, g = x / kTreeGroup, rows = 3 * n_iter;
  double* node1 = nodes;
  double* node2 = nodes + rows * ng;
  // ---- level 1: this workgroup's leaves (L1: formed and stored iteration by iteration during
  // the run — the stores are drained by arrive_last)
  if (!L1) __syncthreads();  // every wave's part[] stores of the run are done
  for (int64_t row = tid; row < (L1 ? 0 : rows); row += NT) {
    double v[WPB];
#pragma unroll
    for (int k = 0; k < WPB; ++k) {
      const int64_t j = x * WPB + k;
      v[k] = j < nb ? part[row * nb + j] : 0.0;
    }
#pragma unroll
    for (int w = WPB; w > 1; w >>= 1)
#pragma unroll
      for (int k = 0; k < w / 2; ++k) v[k] = v[2 * k] + v[2 * k + 1];
    st_sc1(&node1[row * ng + x], v[0]);
  }
#if DMT_TREE_ONEHOP
  if (ng <= 256 && rows * ng <= 32768) {
    // few workgroups and rows (C2 at the driver's 20 iterations: 256 x 60): one arrival over all of them, then each row's tree over its ng
    // level-1 nodes as 64 lanes x 4 adjacent leaves (zero-padded to 256) — the same complete
    // adjacent-pair tree as the two-hop form below, whose 16 x 16 grouping it skips
    if (!arrive_last(&counters[ng2], (unsigned)ng, &s_flag)) return;
    constexpr int RB = 8;  // rows per wave per batch (4 RB loads per lane in flight)
    for (int64_t r0 = (int64_t)wv * RB; r0 < rows; r0 += (int64_t)NW * RB) {
      double v[RB][4];
#pragma unroll
      for (int b = 0; b < RB; ++b)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t row = r0 + b, nd = 4 * lane + k;
          v[b][k] = (row < rows && nd < ng) ? ld_sc1(&node1[row * ng + nd]) : 0.0;
        }
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const double t = wave_tree_sum<double>((v[b][0] + v[b][1]) + (v[b][2] + v[b][3]));
        const int64_t row = r0 + b;
        if (lane == 0 && row < rows) out3[row] = (row % 3 == 2) ? t : t + 0.0;
      }
    }
    __syncthreads();
    if (tid == 0)  // ready for the next launch (stream-ordered)
      __hip_atomic_store(&counters[ng2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
#endif
  const int64_t gsize = ng - g * kTreeGroup < kTreeGroup ? ng - g * kTreeGroup : kTreeGroup;
  if (!arrive_last(&counters[g], (unsigned)gsize, &s_flag)) return;
  // ---- level 2: group g's nodes, 16 lanes per row, NT/16 rows per pass, U passes in flight
  {
    constexpr int RPP = NT / kTreeGroup, U = 8;
    const int k = tid % kTreeGroup;
    const int64_t col = g * kTreeGroup + k;
    for (int64_t r0 = 0; r0 < rows; r0 += (int64_t)RPP * U) {
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t row = r0 + (int64_t)u * RPP + tid / kTreeGroup;
        v[u] = (row < rows && col < ng) ? ld_sc1(&node1[row * ng + col]) : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v[u] = group_tree_sum<kTreeGroup, double>(v[u]);
        const int64_t row = r0 + (int64_t)u * RPP + tid / kTreeGroup;
        if (k == 0 && row < rows) st_sc1(&node2[row * ng2 + g], v[u]);
      }
    }
  }
  if (tid == 0) __hip_atomic_store(&counters[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!arrive_last(&counters[ng2], (unsigned)ng2, &s_flag)) return;
  // ---- level 3: every row's group nodes, zero-padded
  if (ng2 <= 64) {
    constexpr int RB = 8;  // rows per wave per batch (loads in flight)
    for (int64_t r0 = (int64_t)wv * RB; r0 < rows; r0 += (int64_t)NW * RB) {
      double v[RB];
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const int64_t row = r0 + b;
        v[b] = (row < rows && lane < ng2) ? ld_sc1(&node2[row * ng2 + lane]) : 0.0;
      }
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const double t = wave_tree_sum<double>(v[b]);
        const int64_t row = r0 + b;
        if (lane == 0 && row < rows) out3[row] = (row % 3 == 2) ? t : t + 0.0;
      }
    }
  } else {
    // very many blocks: each lane folds an aligned run of the padded node2 row (binary
    // counter), then the 64-lane tree
    int64_t P = 64;
    while (P < ng2) P <<= 1;
    const int64_t run = P / 64;
    constexpr int kLv = 24;
    for (int64_t row = wv; row < rows; row += NW) {
      double stk[kLv];
#pragma unroll
      for (int l = 0; l < kLv; ++l) stk[l] = 0.0;
      double acc = 0.0;
      for (int64_t k = 0; k < run; ++k) {
        const int64_t nd = (int64_t)lane * run + k;
        double xv = nd < ng2 ? ld_sc1(&node2[row * ng2 + nd]) : 0.0;
        bool carry = true;
#pragma unroll
        for (int l = 0; l < kLv; ++l) {
          const bool bit = (k >> l) & 1;
          const double y = stk[l] + xv;
          const bool add = carry && bit;
          stk[l] = (carry && !bit) ? xv : stk[l];
          carry = add;
          xv = add ? y : xv;
        }
        acc = xv;
      }
      acc = wave_tree_sum<double>(acc);
      if (lane == 0) out3[row] = (row % 3 == 2) ? acc : acc + 0.0;
    }
  }
  __syncthreads();
  if (tid == 0)  // ready for the next launch (stream-ordered)
    __hip_atomic_store(&counters[ng2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// dmt_mcmc_run for linear drifts: n_iter path-MCMC iterations in ONE launch.  Blocks are
// independent across iterations (a block's next proposal depends only on its own accepted
// state), so each wave loops over the iterations of its block: draw (scan_block, device RNG),
// then — uniformly, exactly as k_accept — the MH decision, selector flips (bit masks in
// SGPRs), histories and the ll swap.  Per-iteration (ll, ll°, accepted) go to
// part[n_iter][3][nb]; persistent_tree_tail forms every iteration's fetch_ll from them.
template <class Mdl, class T, bool TD = false>
__device__ __forceinline__ void mcmc_scan_block(const BlockArgs<T>& a, const AcceptArgs& c,
                                                const int64_t iter0, const int64_t n_iter,
                                                double* __restrict__ part, const int64_t blk,
                                                ScanLds<Mdl::D, T>& L) {
  const int lane = threadIdx.x & 63;
  const int g0 = ldc(&a.binfo[blk].g0), g1 = ldc(&a.binfo[blk].g1);
  const int nseg = g1 - g0 + 1;  // ≤ kPersistMaxSegments = 64 (host-checked)
  const bool own = lane < nseg;
  SelMask sel{__ballot(own && sel_u(a.selX[g0 + (own ? lane : 0)]) != 0),
              __ballot(own && sel_u(a.selW[g0 + (own ? lane : 0)]) != 0), g0};
  const uint64_t all = nseg >= 64 ? ~(uint64_t)0 : (((uint64_t)1 << nseg) - 1);
  double ll = wave_uniform(c.ll[blk]), llp = 0.0;
  const int64_t nb = a.b1 - a.b0, j = blk - a.b0;
  for (int64_t r = 0; r < n_iter; ++r) {
    const int64_t it = iter0 + r;
    const double E = exp1_draw(c.seed, (uint32_t)g0 + c.seg_base, (uint32_t)(it + c.key_delta), c.salt);
    T lp;
    bool ok;
    if constexpr (TD)
      scan_block_ni<Mdl, T, MODE_PCN, SelMask, TD>(a, blk, (uint32_t)(it + c.key_delta), sel, L, lp, ok);
    else
      scan_block<Mdl, T, MODE_PCN, SelMask, TD>(a, blk, (uint32_t)(it + c.key_delta), sel, L, lp, ok);
    llp = ok ? (double)lp : -INFINITY;
    const bool acc = E > -(llp - ll);
    if (acc) {
      sel.mx ^= all;
      sel.mw ^= all;
    }
    if (lane == 0) {
      if (c.hist_len > 0) {
        const int64_t o = (it - 1) * c.nblocks + blk;
        c.acc_hist[o] = acc ? 1 : 0;
        c.ll_hist[o] = ll;
        c.llp_hist[o] = llp;
      }
      part[(3 * r + 0) * nb + j] = acc ? llp : ll;
      part[(3 * r + 1) * nb + j] = acc ? ll : llp;
      part[(3 * r + 2) * nb + j] = acc ? 1.0 : 0.0;
    }
    if (acc) {
      const double t = ll;
      ll = llp;
      llp = t;
    }
    // this wave's path stores of the iteration are complete before the next iteration reads
    // the accepted path back
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  if (own) {
    a.selX[g0 + lane] = sel_two(sel.x(g0 + lane));
    a.selW[g0 + lane] = sel_two(sel.w(g0 + lane));
  }
  if (lane == 0) {
    c.ll[blk] = ll;
    c.llp[blk] = llp;
  }
}

template <class Mdl, class T, bool TD = false>
__global__ __launch_bounds__((64 * ScanCfg<Mdl::D, T>::WPB), 1) void k_mcmc_scan(
    const BlockArgs<T> a, const AcceptArgs c, const int64_t iter0, const int64_t n_iter,
    double* __restrict__ part, double* __restrict__ nodes, unsigned* __restrict__ counter,
    double* __restrict__ out3) {
  using Cfg = ScanCfg<Mdl::D, T>;
  __shared__ ScanLds<Mdl::D, T> lds[Cfg::WPB];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t blk = a.b0 + (int64_t)blockIdx.x * Cfg::WPB + w;
  if (blk < a.b1) mcmc_scan_block<Mdl, T, TD>(a, c, iter0, n_iter, part, blk, lds[w]);
  persistent_tree_tail<Cfg::WPB>(part, nodes, a.b1 - a.b0, n_iter, counter, out3);
}



// dmt_mcmc_run for linear drifts whose blocks are ONE segment of at most kSChunk steps (e.g.
// C2): the same canonical arithmetic as scan_block, but the block's per-step constants stay
// in registers for the whole run, in run order (lane j ↔ steps 8j … 8j+7): the step matrices
// A_i, the guiding offsets c_i, dt_i, √dt_i, H_i, F_i, and u's Wiener increments (after a
// decision they are the proposal's dW° or stay, both already in registers).  Per iteration the
// wave only draws normals, forms e_i = fma(c_i, dt_i, σdW°_i), composes / scans / applies the
// maps, evaluates G at the points (register-local 8-leaf trees + 3 cross-lane levels = the
// 64-step chunk trees) and stores X°, W° — transposed through LDS so that the stores stay
// coalesced.  Global memory is read once per launch.  The Exp(1) draws of 64 iterations are
// computed at once, one per lane.
template <int D, int M, class T>
struct ResLds {
  T pt[kSStride][D];  // pre-step points by LDS slot of the step (+ end point)
  T dw[kSStride][M];  // W° increments by LDS slot of the step
  // H_i, F_i of each lane's run (G's inputs), lane-minor: in LDS rather than registers, which
  // the run's other constants fill (fewer AGPR round trips, −5 % VALU instructions)
  T hf[kRun][D * (D + 1) / 2 + D][64];
};

// MCMC: n_iter iterations with the in-kernel MH decision (dmt_mcmc_run); otherwise one draw /
// re-solve in mode MODE (k_block_resident: dmt_draw_proposal, dmt_draw_unit,
// dmt_recompute_path), ll and success written like k_block_scan.
template <class Mdl, class T, int MODE, bool MCMC>
__device__ __forceinline__ void resident_block(const BlockArgs<T>& a, const AcceptArgs& c,
                                               const int64_t iter0, const int64_t n_iter,
                                               double* __restrict__ part, const int64_t blk,
                                               ResLds<Mdl::D, Mdl::M, T>& S) {
  constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2;
  static_assert(Mdl::kLinear, "resident_block needs a linear drift");
  static_assert(!MCMC || MODE == MODE_PCN, "MCMC runs draw pCN proposals");
  const int lane = threadIdx.x & 63;
  const BlkInfo* bi = a.binfo + blk;
  const int64_t tq = ldc(&bi->tq);
  const int g = ldc(&bi->g0);  // the block's only segment (host-checked)
  const int q0 = ldc(&bi->q0);
  const bool term = ldc(&bi->term) != 0;  // a single-segment block: P_last law if non-terminal
  const T rho = (MODE == MODE_FRESH) ? (T)0 : (T)ldc(&bi->rho);
  const T srho = (MODE == MODE_FRESH) ? (T)1 : (T)ldc(&bi->srho);
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32), c3 = a.salt << 1;
  const int nst = ldc(a.seg_np + g) - 1;  // ≤ kSChunk
  const int64_t row = tq + q0;
  const int kind = term ? 0 : 1;
  const int ls = (kind ? ldc(a.selPPB + g) : ldc(a.selPP + g)) ^ a.law_flip;
  Law<Mdl, T> LA;
  LA.load(a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE);
  const T* tb = a.t_shared ? a.t + q0 : a.t + row;
  const T* Hb = a.H_shared[ls][kind] ? a.H[ls][kind] + (int64_t)q0 * HP : a.H[ls][kind] + row * HP;
  const T* Fb = a.F[ls][kind] + row * D;
  SelMask sel{(uint64_t)sel_u(a.selX[g]), (uint64_t)sel_u(a.selW[g]), g};
  T* const Xd[2] = {a.X[0] + row * D, a.X[1] + row * D};
  T* const Wd[2] = {a.W[0] + row * M, a.W[1] + row * M};
  // ---- per-launch state: start point, loglikhd_obs, per-step constants (run order)
  T x0[D], w0[M], llobs;
  {
    const T* Xs = a.X[sel.x(g) ^ a.xs_flip] + row * D;
    const T* Ws = a.W[sel.w(g) ^ a.ws_flip] + row * M;
    const int lsp = ldc(a.selPP + g) ^ a.law_flip;  // loglikhd_obs uses PP[1] (block.jl:178)
    T H0[HP], F0[D];
#pragma unroll
    for (int p = 0; p < D; ++p) x0[p] = Xs[p];
#pragma unroll
    for (int k = 0; k < M; ++k) w0[k] = (MODE == MODE_FRESH) ? (T)0 : Ws[k];
#pragma unroll
    for (int cc = 0; cc < HP; ++cc)
      H0[cc] = a.H_shared[lsp][0] ? a.H[lsp][0][(int64_t)q0 * HP + cc] : a.H[lsp][0][row * HP + cc];
#pragma unroll
    for (int cc = 0; cc < D; ++cc) F0[cc] = a.F[lsp][0][row * D + cc];
    const T c00 = (T)ldc(a.law[lsp][0] + (int64_t)g * DMT_LAW_STRIDE + DMT_LAW_C0);
    llobs = obs_term<D, T>(H0, F0, x0, c00);
  }
  const int nv = max(0, min(kRun, nst - kRun * lane));  // valid steps of this lane's run
  T Ac[kRun][D * D], cgs[kRun][D], dts[kRun], sdts[kRun], wv[kRun][M];
  {
    const T* Ws = a.W[sel.w(g) ^ a.ws_flip] + row * M;
#pragma unroll
    for (int r = 0; r < kRun; ++r) {
      const int s = min(kRun * lane + r, nst - 1);
      dts[r] = tb[s + 1] - tb[s];
      sdts[r] = sqrt(dts[r]);
      T Hs[kRun][HP], Fs[kRun][D];
#pragma unroll
      for (int cc = 0; cc < HP; ++cc) Hs[r][cc] = Hb[(int64_t)s * HP + cc];
#pragma unroll
      for (int cc = 0; cc < D; ++cc) Fs[r][cc] = Fb[(int64_t)s * D + cc];
#pragma unroll
      for (int k = 0; k < M; ++k) wv[r][k] = (MODE == MODE_FRESH) ? (T)0 : Ws[(int64_t)(s + 1) * M + k];
      T Mg[D * D], zero[D] = {}, e_unused[D];
      guide_coeffs<Mdl, T>(LA, Hs[r], Fs[r], Mg, cgs[r]);
#pragma unroll
      for (int cc = 0; cc < HP; ++cc) S.hf[r][cc][lane] = Hs[r][cc];
#pragma unroll
      for (int cc = 0; cc < D; ++cc) S.hf[r][HP + cc][lane] = Fs[r][cc];
      affine_step<D, T>(Mg, cgs[r], dts[r], zero, Ac[r], e_unused);
    }
  }
  const uint64_t all = 1;
  double ll = MCMC ? c.ll[blk] : 0.0, llp = 0.0;
  const double* Zg = a.Z ? a.Z + ldc(a.st_off + g) * M : nullptr;  // parity-mode normals
  const int64_t nb = a.b1 - a.b0, j = blk - a.b0;
  const int last_lane = (nst - 1) / kRun;
  double Ev = 0.0;
  // the normals of one iteration for this lane's run: normal n = s·M + k of step s = 8·lane + r
  // is entry n % NPB of Philox block n / NPB; the run's 8M normals are exactly
  // the blocks (8M/NPB)·lane … (8M/NPB)·(lane + 1) − 1, so every index below is a compile-time
  // offset
  auto draw_z = [&](uint32_t itv, T (&z)[kRun][M]) {
    constexpr int NPB = NormPerBlock<T>::v, NB = kRun * M / NPB;  // Philox blocks per run
    static_assert((kRun * M) % NPB == 0, "a run must hold whole normal blocks");
    T zz[kRun * M];
#pragma unroll
    for (int q = 0; q < NB; ++q)
      normal_block(philox4x32_10(U4{(uint32_t)(NB * lane + q), (uint32_t)g + a.seg_base, itv, c3},
                                 k0, k1),
                   zz + NPB * q);
#pragma unroll
    for (int r = 0; r < kRun; ++r)
#pragma unroll
      for (int kk = 0; kk < M; ++kk) z[r][kk] = zz[r * M + kk];
  };
  // (drawing iteration r + 1's normals inside iteration r, to interleave them with its scan,
  // measured slower: 8.46 vs 8.12 µs per C2 iteration — register pressure)
  for (int64_t r0 = 0; r0 < n_iter; ++r0) {
    const int64_t it = iter0 + r0;
    if (MCMC && (r0 & 63) == 0)  // Exp(1) draws of the next 64 iterations, one per lane
      Ev = exp1_draw(c.seed, (uint32_t)g + c.seg_base, (uint32_t)(it + c.key_delta + lane), c.salt);
    const double E = __builtin_bit_cast(
        double, ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(
                     (int)(__builtin_bit_cast(uint64_t, Ev) >> 32), (int)(r0 & 63)) << 32) |
                    (uint32_t)__builtin_amdgcn_readlane((int)__builtin_bit_cast(uint64_t, Ev),
                                                        (int)(r0 & 63)));
    T* const Xdb = (sel.x(g) ^ a.xd_flip) ? Xd[1] : Xd[0];
    T* const Wdb = (sel.w(g) ^ a.wd_flip) ? Wd[1] : Wd[0];
    // ---- normals, pCN increments, e maps; run map
    T dW[kRun][M], e[kRun][D];
    T zc[kRun][M];
    if (MODE != MODE_RECOMPUTE) {
      if (Zg) {
#pragma unroll
        for (int r = 0; r < kRun; ++r)
#pragma unroll
          for (int kk = 0; kk < M; ++kk)
            zc[r][kk] = (T)Zg[(int64_t)min(kRun * lane + r, nst - 1) * M + kk];
      } else {
        draw_z((uint32_t)(it + c.key_delta), zc);
      }
    }
#pragma unroll
    for (int r = 0; r < kRun; ++r) {
#pragma unroll
      for (int kk = 0; kk < M; ++kk)
        dW[r][kk] = (MODE == MODE_RECOMPUTE) ? wv[r][kk]
                                              : dfma(rho, wv[r][kk], srho * (sdts[r] * zc[r][kk]));
      T sdW[D];
      sigma_dw<Mdl, T>(LA, dW[r], sdW);
#pragma unroll
      for (int p = 0; p < D; ++p) e[r][p] = dfma(cgs[r][p], dts[r], sdW[p]);
    }
    T RA[D * D], Re[D];
#pragma unroll
    for (int cc = 0; cc < D * D; ++cc) RA[cc] = Ac[0][cc];
#pragma unroll
    for (int p = 0; p < D; ++p) Re[p] = e[0][p];
    // steps past the segment end are composed too: only the lane holding the segment's last
    // step has any, and its run map feeds only the prefixes of lanes with no valid step
#pragma unroll
    for (int r = 1; r < kRun; ++r) {
      T An[D * D], en[D];
      affine_compose<D, T>(Ac[r], e[r], RA, Re, An, en);
#pragma unroll
      for (int cc = 0; cc < D * D; ++cc) RA[cc] = An[cc];
#pragma unroll
      for (int p = 0; p < D; ++p) Re[p] = en[p];
    }
    wave_affine_scan<D, T>(RA, Re, lane);
    T x[D];
    {
      T y[D];
      affine_apply<D, T>(RA, Re, x0, y);
#pragma unroll
      for (int p = 0; p < D; ++p) {
        const T up = wave_shr1<T>(y[p]);
        x[p] = lane == 0 ? x0[p] : up;
      }
    }
    // ---- points, Girsanov terms (8-leaf register tree), LDS staging of X° and W°
    T gl[kRun];
#pragma unroll
    for (int r = 0; r < kRun; ++r) {
      const int li = lds_ix(kRun * lane + r);
      const bool v = r < nv;
      T rr[D], bb[D];
      T Hr[HP], Fr[D];
#pragma unroll
      for (int cc = 0; cc < HP; ++cc) Hr[cc] = S.hf[r][cc][lane];
#pragma unroll
      for (int cc = 0; cc < D; ++cc) Fr[cc] = S.hf[r][HP + cc][lane];
      const T G = g_at<Mdl, T>(LA, Hr, Fr, x, rr, bb);
      gl[r] = (v && (MODE != MODE_RECOMPUTE || kRun * lane + r < nst - a.ll_skip)) ? G * dts[r] : (T)0;
      // branch-free: slots of steps past the segment end are written but never read
#pragma unroll
      for (int p = 0; p < D; ++p) S.pt[li][p] = x[p];
#pragma unroll
      for (int k = 0; k < M; ++k) S.dw[li][k] = dW[r][k];
      T xn[D];
      affine_apply<D, T>(Ac[r], e[r], x, xn);
#pragma unroll
      for (int p = 0; p < D; ++p) x[p] = v ? xn[p] : x[p];
    }
    // end point of the segment (held by the lane of the last step) → every lane
    T xe[D];
#pragma unroll
    for (int p = 0; p < D; ++p) xe[p] = lane_read(x[p], 4 * last_lane);
    T tsum = ((gl[0] + gl[1]) + (gl[2] + gl[3])) + ((gl[4] + gl[5]) + (gl[6] + gl[7]));
    tsum = group_tree_sum<8, T>(tsum);
    T seg_acc = (T)0;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (64 * q < nst) seg_acc = seg_acc + (lane_read(tsum, 4 * 8 * q) + (T)0);
    wave_lds_sync();
    // ---- coalesced stores of the proposal: X°[0..nst], W°[0..nst]
#pragma unroll
    for (int k = 0; k < kRun; ++k) {
      const int s = 64 * k + lane;
      if (s < nst) {
        const int li = lds_ix(s);
        T xv[D], wd[M];
#pragma unroll
        for (int p = 0; p < D; ++p) xv[p] = S.pt[li][p];
#pragma unroll
        for (int kk = 0; kk < M; ++kk) wd[kk] = S.dw[li][kk];
        store_row<D, T>(Xdb + (int64_t)s * D, xv);
        if (MODE != MODE_RECOMPUTE) store_row<M, T>(Wdb + (int64_t)(s + 1) * M, wd);
      }
    }
    T w0n[M];
#pragma unroll
    for (int k = 0; k < M; ++k) w0n[k] = rho * w0[k];
    if (lane == 0) {
      store_row<D, T>(Xdb + (int64_t)nst * D, xe);
      if (MODE != MODE_RECOMPUTE) store_row<M, T>(Wdb, w0n);
    }
    wave_lds_sync();
    bool sok = isfinite(seg_acc);
#pragma unroll
    for (int p = 0; p < D; ++p) sok = sok && isfinite(xe[p]);
    if constexpr (!MCMC) {  // one draw / re-solve: ll and success, as k_block_scan
      if (lane == 0) {
        a.ll_out[blk] = sok ? (double)(llobs + seg_acc) : -INFINITY;
        if (a.success) a.success[blk] = sok ? 1 : 0;
      }
      return;
    }
    // ---- MH decision (k_accept's order), selectors, histories, partials
    llp = sok ? (double)(llobs + seg_acc) : -INFINITY;
    if (lane == 0 && a.success) a.success[blk] = sok ? 1 : 0;  // the run's last draw's flag
    const bool acc = E > -(llp - ll);
    if (acc) {
      sel.mx ^= all;
      sel.mw ^= all;
#pragma unroll
      for (int r = 0; r < kRun; ++r)
#pragma unroll
        for (int k = 0; k < M; ++k) wv[r][k] = dW[r][k];
#pragma unroll
      for (int k = 0; k < M; ++k) w0[k] = w0n[k];
    }
    if (lane == 0) {
      if (c.hist_len > 0) {
        const int64_t o = (it - 1) * c.nblocks + blk;
        c.acc_hist[o] = acc ? 1 : 0;
        c.ll_hist[o] = ll;
        c.llp_hist[o] = llp;
      }
      part[(3 * r0 + 0) * nb + j] = acc ? llp : ll;
      part[(3 * r0 + 1) * nb + j] = acc ? ll : llp;
      part[(3 * r0 + 2) * nb + j] = acc ? 1.0 : 0.0;
    }
    if (acc) {
      const double t = ll;
      ll = llp;
      llp = t;
    }
  }
  if (MCMC && lane == 0) {
    a.selX[g] = sel_two(sel.x(g));
    a.selW[g] = sel_two(sel.w(g));
    c.ll[blk] = ll;
    c.llp[blk] = llp;
  }
}

template <class Mdl, class T>
__global__ __launch_bounds__(256, 1) void k_mcmc_resident(const BlockArgs<T> a,
                                                          const AcceptArgs c,
                                                          const int64_t iter0,
                                                          const int64_t n_iter,
                                                          double* __restrict__ part,
                                                          double* __restrict__ nodes,
                                                          unsigned* __restrict__ counter,
                                                          double* __restrict__ out3) {
  __shared__ ResLds<Mdl::D, Mdl::M, T> lds[4];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t blk = a.b0 + (int64_t)blockIdx.x * 4 + w;
#ifdef DMT_VARIANT_EARLY_RETURN  // measurement variant: no in-kernel trees (out3 not written)
  if (blk >= a.b1) return;
  resident_block<Mdl, T, MODE_PCN, true>(a, c, iter0, n_iter, part, blk, lds[w]);
#else
  if (blk < a.b1) resident_block<Mdl, T, MODE_PCN, true>(a, c, iter0, n_iter, part, blk, lds[w]);
  persistent_tree_tail<4>(part, nodes, a.b1 - a.b0, n_iter, counter, out3);
#endif
}

// ---- k_mcmc_resident split over two waves per block (producer / consumer).
// One wave per block leaves one wave per SIMD for C2's 1 024 blocks: a lone wave issues a VALU
// instruction every 4 cycles at best and exposes every LDS / cross-lane latency (SQ counters:
// VALU active 0.58 of wave cycles).  Here each block has two waves on the same arithmetic:
//   producer — the normals of the NEXT iteration (Philox4x32-10 + Box–Muller, ≈ 60 % of the
//              single-wave kernel's VALU), u's Wiener increments (register-resident, updated by
//              the decision), the pCN increments dW° = fma(ρ, dW, √(1−ρ²)·(√dt·Z)) → LDS (run
//              order, the consumer's layout), and the coalesced W° stores;
//   consumer — everything else of resident_block: e maps, run maps, the scan, the points, G and
//              its trees, the X° stores, the MH decision (→ LDS for the producer).
// Two workgroup barriers per iteration: B1 (dW° of iteration n ready) and B2 (decision n
// made).  Between B1 and B2 the producer draws iteration n+1's normals while the consumer runs
// iteration n, so the two waves of every SIMD issue concurrently.  The operations and their
// order are resident_block's: bit-identical results (the GPU tests run both).
// Measurement build only (-DDMT_PC_STAMPS, scripts/pc_stamps.py): device wall-clock stamps of
// one k_mcmc_resident_pc launch per workgroup — entry, the consumer's and the producer's set-up
// done, B1 of iteration 0 passed, the loop's end, the tail's end (dmt_probe_pc_stamps).
#ifdef DMT_PC_STAMPS
__device__ uint64_t g_pc_stamps[8192 * 8];
#define PC_STAMP(TID, K)                                                                  \
  do {                                                                                    \
    if (threadIdx.x == (TID) && blockIdx.x < 8192)                                        \
      g_pc_stamps[blockIdx.x * 8 + (K)] = (uint64_t)wall_clock64();                        \
  } while (0)
extern "C" int dmt_probe_pc_stamps(uint64_t* out, int64_t n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pc_stamps), (size_t)std::min<int64_t>(n, 8192 * 8) * 8);
}
// per iteration r < 64 of workgroup 0: consumer after B1 (0), its decision made (1), at B2 (2),
// after B2 (3); producer after B1 (4), at B2 with the next normals drawn (5), after B2 (6), at
// B1 with the next proposal handed over (7)
__device__ uint64_t g_pc_it[64 * 8];
#define PC_ITSTAMP(TID, R, K)                                                             \
  do {                                                                                    \
    if (threadIdx.x == (TID) && blockIdx.x == 0 && (R) < 64)                              \
      g_pc_it[(R) * 8 + (K)] = (uint64_t)wall_clock64();                                   \
  } while (0)
extern "C" int dmt_probe_pc_iter_stamps(uint64_t* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pc_it), 64 * 8 * 8);
}
#else
#define PC_STAMP(TID, K) \
  do {                   \
  } while (0)
#define PC_ITSTAMP(TID, R, K) \
  do {                        \
  } while (0)
#endif
#ifndef DMT_PC_DRAW_GROUP
#define DMT_PC_DRAW_GROUP 8
#endif
#ifndef DMT_PC_LATE_C  // the consumer forms its own steps' next proposal after B2
#define DMT_PC_LATE_C 1
#endif
#ifndef DMT_PC_SPEC  // the producer forms both candidates of the next proposal before B2
#define DMT_PC_SPEC 1
#endif
#ifndef DMT_PC_SETUP_OVERLAP  // set-up loads in flight while the first normals are drawn
#define DMT_PC_SETUP_OVERLAP 1
#endif
#ifndef DMT_PC_CONS_STEPS
#define DMT_PC_CONS_STEPS 2
#endif
// With one producer, the consumer draws the normals (and forms dW°, e) of the last CR steps of
// every lane run itself, filling its own latency bubbles and shortening the producer's chain;
// only when those steps hold whole Philox blocks.
template <class T, int M, int NP>
struct PcConsSteps {
  static constexpr int v = (NP == 1 && (DMT_PC_CONS_STEPS * M) % NormPerBlock<T>::v == 0)
                               ? DMT_PC_CONS_STEPS : 0;
};
template <int D, int M, class T>
struct ResPcLds {
  ResLds<D, M, T> r;  // pt: X° staging; dw: the dW° hand-off and W° staging; hf: H_i, F_i
  int acc;            // the consumer's decision of the current iteration
};

// ---- the resident MCMC service (SvcArgs): iterations posted by the host one at a time.
struct SvcLds {
  int go;             // the gate's answer
  double row[3][4];   // the iteration's (ll, ll°, accepted) of the workgroup's 4 blocks
};
#ifndef DMT_SVC_PEEK  // the gate's host words read ahead (svc_peek): 1 after the iteration's
#define DMT_SVC_PEEK 1   // points, 2 after its scan; 0: at the gate only
#endif
// Gate of iteration r (in place of its B1 barrier).  Workgroup 0's thread 0 is the launch's one
// reader of host memory: it waits until the host has posted iteration r, asked the launch to
// stop, or stayed silent for idle_ticks, and publishes the answer in device memory — go word
// = base + r + 1, or exit word = base + r + 1 — which the other workgroups' thread 0 wait for
// (agent scope: no PCIe traffic from 256 pollers; one decision, so every workgroup leaves at
// the same gate and the launch's state is exactly that of its first r iterations).  The grid
// is co-resident (launch_mcmc_service checks), so the reader always reaches the gate.  The
// barrier hands the answer to every wave.  Nothing global is written for an iteration before
// its gate opens.
// spec_stop, spec_posted: workgroup 0's thread 0 read the two host words once already, late in
// the iteration's arithmetic (svc_peek); a post seen there opens the gate without another PCIe
// round trip (the loop below reads them again otherwise)
struct SvcPeek {
  uint32_t stop = 1u;
  uint64_t posted = 0;
};
__device__ __forceinline__ SvcPeek svc_peek(const SvcArgs& sv) {
  SvcPeek p;
#if DMT_SVC_PEEK
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    p.stop = __hip_atomic_load(sv.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    p.posted = __hip_atomic_load(sv.posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
#endif
  return p;
}
__device__ __forceinline__ bool svc_gate(const SvcArgs& sv, int64_t r, SvcLds* sl,
                                         const SvcPeek pk = SvcPeek{}) {
  if (threadIdx.x == 0) {
    const uint64_t want = sv.base + (uint64_t)r + 1;
    int go = 0;
    if (blockIdx.x == 0) {
      const uint64_t t0 = (uint64_t)wall_clock64();
      if (pk.stop == 0u && pk.posted >= want) go = 1;
      for (; !go;) {
        if (__hip_atomic_load(sv.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) break;
        if (__hip_atomic_load(sv.posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= want) {
          go = 1;
          break;
        }
        if ((uint64_t)wall_clock64() - t0 > sv.idle_ticks) break;
        __builtin_amdgcn_s_sleep(4);
      }
      __hip_atomic_store(go ? sv.go : sv.quit, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef DMT_SVC_PROBE
      if (go) sv.probe[8 * (want - 1) + 0] = (uint64_t)wall_clock64();
#endif
    } else {
      for (;;) {
        if (__hip_atomic_load(sv.go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) {
          go = 1;
          break;
        }
        if (__hip_atomic_load(sv.quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == want) break;
        __builtin_amdgcn_s_sleep(2);
      }
    }
    sl->go = go;
#ifdef DMT_SVC_PROBE
    if (go) __hip_atomic_fetch_max(&sv.probe[8 * (want - 1) + 1], (uint64_t)wall_clock64(),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
  }
  __syncthreads();
  return sl->go != 0;
}

// Iteration r's gate has opened: the workgroup's 4 consumer waves left their blocks' (ll, ll°,
// accepted) in row[c][0..3] before it (0.0 for a block past b1).  Lanes 0..2 of wave 0 fold them — the
// aligned 4-leaf subtree ((x0 + x1) + (x2 + x3)) of the canonical fetch_ll tree — and send each
// sum to the host as ONE 16-byte store (value bits, value bits ^ svc_mix(iteration + 1)): the
// host takes a record once its two words agree for the iteration it waits for (a torn read does
// not, dmt_internal.h) and folds the workgroups' sums in the canonical order (svc_fold in
// dmt_runtime.hip).  No counter, no wait: the workgroup goes on.
// Records alternate between two sets by the iteration's parity; the host reads set s & 1 of
// iteration s before it posts s + 1, so set s & 1 is free again when iteration s + 2 writes it.
__device__ __forceinline__ void svc_record(const SvcArgs& sv, const SvcLds* sl, int64_t r) {
  const int lane = threadIdx.x & 63;
  if (lane < 3) {
    const double v = (sl->row[lane][0] + sl->row[lane][1]) + (sl->row[lane][2] + sl->row[lane][3]);
    const uint64_t slot = sv.base + (uint64_t)r;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint64_t vb = __builtin_bit_cast(uint64_t, v), chk = vb ^ svc_mix(slot + 1);
    const u32x4 rec = {(uint32_t)vb, (uint32_t)(vb >> 32), (uint32_t)chk, (uint32_t)(chk >> 32)};
    uint64_t* dst = sv.rec + (((slot & 1) * gridDim.x + blockIdx.x) * 4 + lane) * 2;
    // one 16-byte vector store, system-coherent (sc0 sc1: written through to host memory now,
    // not held in L2 until the launch ends)
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(dst), "v"(rec) : "memory");
  }
#ifdef DMT_SVC_PROBE
  if (lane == 0)
    __hip_atomic_fetch_max(&sv.probe[8 * (sv.base + r) + 2], (uint64_t)wall_clock64(),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

#ifndef DMT_PC_L1_LOOP  // 1: level 1 of the fetch_ll trees formed during the run (after B2);
                        // 0: read back from part[] by persistent_tree_tail
#define DMT_PC_L1_LOOP 1
#endif
template <class Mdl, class T, int NP, bool SVC, int BPW = 4>
__device__ __forceinline__ void resident_pc_consumer(const BlockArgs<T>& a, const AcceptArgs& c,
                                                     const int64_t iter0, const int64_t n_iter,
                                                     double* __restrict__ part, const int64_t blk,
                                                     const bool valid,
                                                     ResPcLds<Mdl::D, Mdl::M, T>& P,
                                                     const SvcArgs& sv, SvcLds* sl,
                                                     double* __restrict__ nodes = nullptr) {
  constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2;
  constexpr int CR = PcConsSteps<T, M, NP>::v, RC0 = kRun - CR, CRA = CR > 0 ? CR : 1;
  ResLds<D, M, T>& S = P.r;
  const int lane = threadIdx.x & 63;
  const int64_t vb = valid ? blk : a.b0;  // an idle wave reads a valid block's metadata
  const BlkInfo* bi = a.binfo + vb;
  const int64_t tq = ldc(&bi->tq);
  const int g = ldc(&bi->g0);
  const int q0 = ldc(&bi->q0);
  const bool term = ldc(&bi->term) != 0;
  const int nst = ldc(a.seg_np + g) - 1;  // ≤ kSChunk
  const T rho = (T)ldc(&bi->rho), srho = (T)ldc(&bi->srho);
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32), c3 = a.salt << 1;
  const double* Zg = a.Z ? a.Z + ldc(a.st_off + g) * M : nullptr;
  T wvC[CRA][M], sdtC[CRA], zC[CRA][M], dWC[CRA][M];
  auto draw_c = [&](uint32_t itv) {
    if constexpr (CR > 0) {
      if (Zg) {
#pragma unroll
        for (int r = 0; r < CR; ++r)
#pragma unroll
          for (int k = 0; k < M; ++k)
            zC[r][k] = (T)Zg[(int64_t)min(kRun * lane + RC0 + r, nst - 1) * M + k];
        return;
      }
      constexpr int NPB = NormPerBlock<T>::v, NB = CR * M / NPB, NBR = kRun * M / NPB;
      T zz[CR * M];
      uint32_t ln = (uint32_t)(NBR * lane + RC0 * M / NPB);  // opaque: no hoisting (producer)
      asm volatile("" : "+v"(ln));
#pragma unroll
      for (int q = 0; q < NB; ++q)
        normal_block(philox4x32_10(U4{ln + q, (uint32_t)g + a.seg_base, itv, c3}, k0, k1),
                     zz + NPB * q);
#pragma unroll
      for (int r = 0; r < CR; ++r)
#pragma unroll
        for (int k = 0; k < M; ++k) zC[r][k] = zz[r * M + k];
    }
  };
#if DMT_PC_SETUP_OVERLAP
  // the first iteration's normals of the consumer's steps: they need the block's segment
  // only, so their arithmetic runs while the metadata and per-step loads below are in flight
  draw_c((uint32_t)(iter0 + c.key_delta));
#endif
  const int64_t row = tq + q0;
  const int kind = term ? 0 : 1;
  const int ls = (kind ? ldc(a.selPPB + g) : ldc(a.selPP + g)) ^ a.law_flip;
  Law<Mdl, T> LA;
  LA.load(a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE);
  const T* tb = a.t_shared ? a.t + q0 : a.t + row;
  const T* Hb = a.H_shared[ls][kind] ? a.H[ls][kind] + (int64_t)q0 * HP : a.H[ls][kind] + row * HP;
  const T* Fb = a.F[ls][kind] + row * D;
  SelMask sel{(uint64_t)sel_u(a.selX[g]), (uint64_t)sel_u(a.selW[g]), g};
  T* const Xd[2] = {a.X[0] + row * D, a.X[1] + row * D};
  T x0[D], llobs;
  {
    const T* Xs = a.X[sel.x(g) ^ a.xs_flip] + row * D;
    const int lsp = ldc(a.selPP + g) ^ a.law_flip;
    T H0[HP], F0[D];
#pragma unroll
    for (int p = 0; p < D; ++p) x0[p] = Xs[p];
#pragma unroll
    for (int cc = 0; cc < HP; ++cc)
      H0[cc] = a.H_shared[lsp][0] ? a.H[lsp][0][(int64_t)q0 * HP + cc] : a.H[lsp][0][row * HP + cc];
#pragma unroll
    for (int cc = 0; cc < D; ++cc) F0[cc] = a.F[lsp][0][row * D + cc];
    const T c00 = (T)ldc(a.law[lsp][0] + (int64_t)g * DMT_LAW_STRIDE + DMT_LAW_C0);
    llobs = obs_term<D, T>(H0, F0, x0, c00);
  }
  PC_STAMP(0, 6);
  const int nv = max(0, min(kRun, nst - kRun * lane));
  // ---- the consumer's own steps r in [RC0, kRun) of every run (PcConsSteps): u's increments,
  // √dt, the normals of the next iteration, its pCN increments dW° (handed to the producer's
  // W° stores through the dw slots after B2) and e maps (into its own pt slots)
  // set-up: the run's per-step inputs, loaded before any of them is used
  T tl[kRun], tr[kRun], Hs[kRun][HP], Fs[kRun][D];
#pragma unroll
  for (int r = 0; r < kRun; ++r) {
    const int s = min(kRun * lane + r, nst - 1);
    tl[r] = tb[s];
    tr[r] = tb[s + 1];
#pragma unroll
    for (int cc = 0; cc < HP; ++cc) Hs[r][cc] = Hb[(int64_t)s * HP + cc];
#pragma unroll
    for (int cc = 0; cc < D; ++cc) Fs[r][cc] = Fb[(int64_t)s * D + cc];
  }
  if constexpr (CR > 0) {
    const T* Ws = a.W[sel.w(g) ^ a.ws_flip] + row * M;
#pragma unroll
    for (int r = 0; r < CR; ++r) {
      const int s = min(kRun * lane + RC0 + r, nst - 1);
#pragma unroll
      for (int k = 0; k < M; ++k) wvC[r][k] = Ws[(int64_t)(s + 1) * M + k];
    }
  }
  T Ac[kRun][D * D], dts[kRun], cgC[CRA][D];
#pragma unroll
  for (int r = 0; r < kRun; ++r) {
    dts[r] = tr[r] - tl[r];
    T Mg[D * D], cg_unused[D], zero[D] = {}, e_unused[D];
    guide_coeffs<Mdl, T>(LA, Hs[r], Fs[r], Mg, cg_unused);
#pragma unroll
    for (int cc = 0; cc < HP; ++cc) S.hf[r][cc][lane] = Hs[r][cc];
#pragma unroll
    for (int cc = 0; cc < D; ++cc) S.hf[r][HP + cc][lane] = Fs[r][cc];
    affine_step<D, T>(Mg, cg_unused, dts[r], zero, Ac[r], e_unused);
    if (r >= RC0) {
#pragma unroll
      for (int p = 0; p < D; ++p) cgC[r >= RC0 ? r - RC0 : 0][p] = cg_unused[p];
    }
  }
  if constexpr (CR > 0) {
#pragma unroll
    for (int r = 0; r < CR; ++r) sdtC[r] = sqrt(dts[RC0 + r]);
  }
  // dW° and e of the consumer's steps for the iteration whose normals are in zC; e → pt slots
  auto propose_c = [&]() {
    if constexpr (CR > 0) {
#pragma unroll
      for (int r = 0; r < CR; ++r) {
        T sdW[D];
#pragma unroll
        for (int k = 0; k < M; ++k) dWC[r][k] = dfma(rho, wvC[r][k], srho * (sdtC[r] * zC[r][k]));
        sigma_dw<Mdl, T>(LA, dWC[r], sdW);
        const int li = lds_ix(kRun * lane + RC0 + r);
#pragma unroll
        for (int p = 0; p < D; ++p) S.pt[li][p] = dfma(cgC[r][p], dts[RC0 + r], sdW[p]);
      }
    }
  };
  auto hand_dw = [&]() {
    if constexpr (CR > 0) {
#pragma unroll
      for (int r = 0; r < CR; ++r)
#pragma unroll
        for (int k = 0; k < M; ++k) S.dw[lds_ix(kRun * lane + RC0 + r)][k] = dWC[r][k];
    }
  };
  PC_STAMP(0, 7);
#if !DMT_PC_SETUP_OVERLAP
  draw_c((uint32_t)(iter0 + c.key_delta));
#endif
  propose_c();
  hand_dw();
  const uint64_t all = 1;
  double ll = valid ? c.ll[blk] : 0.0, llp = 0.0;
  const int64_t nb = a.b1 - a.b0, j = blk - a.b0;
  const int last_lane = (nst - 1) / kRun;
  double Ev = 0.0;
  PC_STAMP(0, 1);
  __syncthreads();  // B1 of iteration 0
  PC_STAMP(0, 3);
  for (int64_t r0 = 0; r0 < n_iter; ++r0) {
    const int64_t it = iter0 + r0;
    if ((r0 & 63) == 0)
      Ev = exp1_draw(c.seed, (uint32_t)g + c.seg_base, (uint32_t)(it + c.key_delta + lane), c.salt);
    const double E = __builtin_bit_cast(
        double, ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(
                     (int)(__builtin_bit_cast(uint64_t, Ev) >> 32), (int)(r0 & 63)) << 32) |
                    (uint32_t)__builtin_amdgcn_readlane((int)__builtin_bit_cast(uint64_t, Ev),
                                                        (int)(r0 & 63)));
    T* const Xdb = (sel.x(g) ^ a.xd_flip) ? Xd[1] : Xd[0];
    // the next iteration's normals of the consumer's steps (unconditional: no branch around
    // them, so they can fill the scan's latency; the last iteration's are never used).  The
    // service draws them after B2 instead: there the iteration's latency is what the caller
    // waits for, and the host's round trip to the next post hides them.
    PC_ITSTAMP(0, r0, 0);
    if constexpr (!SVC) draw_c((uint32_t)(it + 1 + c.key_delta));
    // the run map of the e maps the producer (and, for its steps, the consumer) left in the pt slots
    T RA[D * D], Re[D];
#pragma unroll
    for (int r = 0; r < kRun; ++r) {
      const int li = lds_ix(kRun * lane + r);
      T er[D];
#pragma unroll
      for (int p = 0; p < D; ++p) er[p] = S.pt[li][p];
      if (r == 0) {
#pragma unroll
        for (int cc = 0; cc < D * D; ++cc) RA[cc] = Ac[0][cc];
#pragma unroll
        for (int p = 0; p < D; ++p) Re[p] = er[p];
      } else {
        T An[D * D], en[D];
        affine_compose<D, T>(Ac[r], er, RA, Re, An, en);
#pragma unroll
        for (int cc = 0; cc < D * D; ++cc) RA[cc] = An[cc];
#pragma unroll
        for (int p = 0; p < D; ++p) Re[p] = en[p];
      }
    }
    wave_affine_scan<D, T>(RA, Re, lane);
    SvcPeek peek;  // (the service: the gate's host words, requested ahead — svc_peek)
    if constexpr (SVC && DMT_SVC_PEEK == 2) peek = svc_peek(sv);
    T x[D];
    {
      T y[D];
      affine_apply<D, T>(RA, Re, x0, y);
#pragma unroll
      for (int p = 0; p < D; ++p) {
        const T up = wave_shr1<T>(y[p]);
        x[p] = lane == 0 ? x0[p] : up;
      }
    }
    T gl[kRun];
#pragma unroll
    for (int r = 0; r < kRun; ++r) {
      const int li = lds_ix(kRun * lane + r);
      const bool v = r < nv;
      T rr[D], bb[D], Hr[HP], Fr[D], er[D];
#pragma unroll
      for (int cc = 0; cc < HP; ++cc) Hr[cc] = S.hf[r][cc][lane];
#pragma unroll
      for (int cc = 0; cc < D; ++cc) Fr[cc] = S.hf[r][HP + cc][lane];
#pragma unroll
      for (int p = 0; p < D; ++p) er[p] = S.pt[li][p];
      const T G = g_at<Mdl, T>(LA, Hr, Fr, x, rr, bb);
      gl[r] = v ? G * dts[r] : (T)0;
#pragma unroll
      for (int p = 0; p < D; ++p) S.pt[li][p] = x[p];
      T xn[D];
      affine_apply<D, T>(Ac[r], er, x, xn);
#pragma unroll
      for (int p = 0; p < D; ++p) x[p] = v ? xn[p] : x[p];
    }
    // (the service: the gate's host words requested now, answered while the trees finish)
    if constexpr (SVC && DMT_SVC_PEEK == 1) peek = svc_peek(sv);
    T xe[D];
#pragma unroll
    for (int p = 0; p < D; ++p) xe[p] = lane_value(x[p], last_lane);  // uniform: v_readlane
    T tsum = ((gl[0] + gl[1]) + (gl[2] + gl[3])) + ((gl[4] + gl[5]) + (gl[6] + gl[7]));
    tsum = group_tree_sum<8, T>(tsum);
    T seg_acc = (T)0;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (64 * q < nst) seg_acc = seg_acc + (lane_value(tsum, 8 * q) + (T)0);
    // the service computes an iteration ahead of its post (registers and LDS only) and
    // publishes it — stores, flags, selectors, the decision — once the host has posted it.  The
    // block's fetch_ll leaves go to LDS before the gate, and the workgroup's records to the host
    // as soon as it opens, ahead of the path stores
    if constexpr (SVC) {
      if (lane == 0) {
        bool ok = isfinite(seg_acc);
#pragma unroll
        for (int p = 0; p < D; ++p) ok = ok && isfinite(xe[p]);
        const double lp = ok ? (double)(llobs + seg_acc) : -INFINITY;
        const bool ac = valid && E > -(lp - ll);
        const int w4 = (int)(threadIdx.x >> 6) & 3;
        sl->row[0][w4] = valid ? (ac ? lp : ll) : 0.0;
        sl->row[1][w4] = valid ? (ac ? ll : lp) : 0.0;
        sl->row[2][w4] = ac ? 1.0 : 0.0;
      }
      if (!svc_gate(sv, r0, sl, peek)) break;
      if (threadIdx.x < 64) svc_record(sv, sl, r0);  // the workgroup's fetch_ll sums → host
    }
    wave_lds_sync();
    if (valid) {
#pragma unroll
      for (int k = 0; k < kRun; ++k) {
        const int s = 64 * k + lane;
        if (s < nst) {
          T xv[D];
#pragma unroll
          for (int p = 0; p < D; ++p) xv[p] = S.pt[lds_ix(s)][p];
          store_row_pc<D, T>(Xdb + (int64_t)s * D, xv);
        }
      }
      if (lane == 0) store_row_pc<D, T>(Xdb + (int64_t)nst * D, xe);
    }
    bool sok = isfinite(seg_acc);
#pragma unroll
    for (int p = 0; p < D; ++p) sok = sok && isfinite(xe[p]);
    llp = sok ? (double)(llobs + seg_acc) : -INFINITY;
    if (lane == 0 && valid && a.success) a.success[blk] = sok ? 1 : 0;  // last draw's flag
    const bool acc = valid && E > -(llp - ll);
    if (acc) {
      sel.mx ^= all;
      sel.mw ^= all;
    }
    PC_ITSTAMP(0, r0, 1);
    if (lane == 0) {
      P.acc = acc ? 1 : 0;
      if (valid) {
        if (c.hist_len > 0) {
          const int64_t o = (it - 1) * c.nblocks + blk;
          c.acc_hist[o] = acc ? 1 : 0;
          c.ll_hist[o] = ll;
          c.llp_hist[o] = llp;
        }
        if constexpr (!SVC && !DMT_PC_L1_LOOP) {
          part[(3 * r0 + 0) * nb + j] = acc ? llp : ll;
          part[(3 * r0 + 1) * nb + j] = acc ? ll : llp;
          part[(3 * r0 + 2) * nb + j] = acc ? 1.0 : 0.0;
        }
      }
      if constexpr (!SVC && DMT_PC_L1_LOOP) {  // the workgroup's fetch_ll leaves (0: no block)
        const int wi = (int)(threadIdx.x >> 6) % BPW;
        sl->row[0][wi] = valid ? (acc ? llp : ll) : 0.0;
        sl->row[1][wi] = valid ? (acc ? ll : llp) : 0.0;
        sl->row[2][wi] = acc ? 1.0 : 0.0;
      }
    }
    if (acc) {
      const double t = ll;
      ll = llp;
      llp = t;
    }
    if constexpr (CR > 0) {  // own steps of iteration n + 1: u's increments, then dW° and e
      if (acc) {
#pragma unroll
        for (int r = 0; r < CR; ++r)
#pragma unroll
          for (int k = 0; k < M; ++k) wvC[r][k] = dWC[r][k];
      }
      if constexpr (!SVC && !DMT_PC_LATE_C) {
        wave_lds_sync();  // this wave's pt reads of the X° stores above are done
        propose_c();
      }
    }
    PC_ITSTAMP(0, r0, 2);
    __syncthreads();  // B2: decision n → producer; pt reads of this iteration done
    PC_ITSTAMP(0, r0, 3);
    if constexpr (!SVC && DMT_PC_L1_LOOP) {
      // level 1 of iteration n's fetch_ll trees (persistent_tree_tail): the workgroup's BPW
      // leaves, adjacent pairs, stored write-through now instead of read back after the run
      if (threadIdx.x < 3) {
        double v[BPW];
#pragma unroll
        for (int k = 0; k < BPW; ++k) v[k] = sl->row[threadIdx.x][k];
#pragma unroll
        for (int w = BPW; w > 1; w >>= 1)
#pragma unroll
          for (int k = 0; k < w / 2; ++k) v[k] = v[2 * k] + v[2 * k + 1];
        const int64_t ng = (a.b1 - a.b0 + BPW - 1) / BPW;
        st_sc1(&nodes[(3 * r0 + threadIdx.x) * ng + blockIdx.x], v[0]);
      }
    }
    // (DMT_PC_LATE_C: the consumer's own steps of iteration n + 1 after B2, beside the producer's
    // proposal — the consumer, not the producer, is the one late at B2)
    if constexpr (!SVC && DMT_PC_LATE_C && CR > 0) propose_c();
    if constexpr (SVC) {
      if constexpr (CR > 0) {
        draw_c((uint32_t)(it + 1 + c.key_delta));
        propose_c();
      }
    }
    if (r0 + 1 < n_iter) {
      hand_dw();  // the producer's W° stores of iteration n are done (before its B2)
      __syncthreads();  // B1: dW° of iteration n + 1 ready
    }
  }
  PC_STAMP(0, 4);
  if (valid && lane == 0) {
    a.selX[g] = sel_two(sel.x(g));
    a.selW[g] = sel_two(sel.w(g));
    c.ll[blk] = ll;
    c.llp[blk] = llp;
  }
}

// NP producer waves per block: producer h owns the steps r in [h·RR, (h+1)·RR) of every lane's
// run (their Philox blocks, u's increments, the pCN and e maps) and the coalesced W° rows
// k in [h·RR, (h+1)·RR); producer 0 also W(t0).
template <class Mdl, class T, int NP, bool SVC>
__device__ __forceinline__ void resident_pc_producer(const BlockArgs<T>& a, const AcceptArgs& c,
                                                     const int64_t iter0, const int64_t n_iter,
                                                     const int64_t blk, const bool valid,
                                                     const int h,
                                                     ResPcLds<Mdl::D, Mdl::M, T>& P,
                                                     const SvcArgs& sv, SvcLds* sl) {
  constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2;
  constexpr int CR = PcConsSteps<T, M, NP>::v;  // trailing run steps the consumer draws
  constexpr int RR = (kRun - CR) / NP, RW = kRun / NP;  // steps / W° rows of one producer
  static_assert((kRun - CR) % NP == 0 && kRun % NP == 0, "whole steps per producer");
  const int r0h = h * RR;
  ResLds<D, M, T>& S = P.r;
  const int lane = threadIdx.x & 63;
  const int64_t vb = valid ? blk : a.b0;
  const BlkInfo* bi = a.binfo + vb;
  const int64_t tq = ldc(&bi->tq);
  const int g = ldc(&bi->g0);
  const int q0 = ldc(&bi->q0);
  const T rho = (T)ldc(&bi->rho);
  const T srho = (T)ldc(&bi->srho);
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32), c3 = a.salt << 1;
  const int nst = ldc(a.seg_np + g) - 1;
  const double* Zg = a.Z ? a.Z + ldc(a.st_off + g) * M : nullptr;  // parity-mode normals
  auto draw_z = [&](uint32_t itv, T (&z)[RR][M]) {
    if (Zg) {
#pragma unroll
      for (int r = 0; r < RR; ++r)
#pragma unroll
        for (int kk = 0; kk < M; ++kk)
          z[r][kk] = (T)Zg[(int64_t)min(kRun * lane + r0h + r, nst - 1) * M + kk];
      return;
    }
    constexpr int NPB = NormPerBlock<T>::v, NB = RR * M / NPB;  // this producer's blocks
    constexpr int NBR = kRun * M / NPB;                          // blocks of a whole run
    static_assert((RR * M) % NPB == 0, "a producer's steps must hold whole normal blocks");
    T zz[RR * M];
    // the blocks' first counter words are loop-invariant: derived from an opaque copy of the
    // lane id so that the compiler does not hoist every block's first Philox round (or the
    // words themselves) out of the iteration loop into spilled registers
    uint32_t ln = (uint32_t)(NBR * lane + h * NB);  // the run's first block of this producer
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int q = 0; q < NB; ++q) {
#if defined(DMT_PROBE_NO_BM)  // timing probes only (wrong normals): Philox without Box–Muller
      {
        const U4 o = philox4x32_10(U4{ln + q, (uint32_t)g + a.seg_base, itv, c3}, k0, k1);
        zz[NPB * q] = (T)(o.x ^ o.y) * (T)0x1p-32;
        zz[NPB * q + 1] = (T)(o.z ^ o.w) * (T)0x1p-32;
      }
#elif defined(DMT_PROBE_NO_PHILOX)  // Box–Muller without Philox
      normal_block(U4{(ln + q) ^ itv, (ln + q) * 0x9E3779B9u ^ itv, itv * 3u + q, c3 ^ ln},
                   zz + NPB * q);
#else
      normal_block(philox4x32_10(U4{ln + q, (uint32_t)g + a.seg_base, itv, c3}, k0, k1),
                   zz + NPB * q);
#endif
      // DMT_PC_DRAW_GROUP Philox blocks + Box–Muller interleaved at a time
      if ((q + 1) % DMT_PC_DRAW_GROUP == 0) __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < RR; ++r)
#pragma unroll
      for (int kk = 0; kk < M; ++kk) z[r][kk] = zz[r * M + kk];
  };
  T z[RR][M], w0n[M];
#if DMT_PC_SETUP_OVERLAP
  // the first iteration's normals: they need the block's segment only, so their arithmetic
  // runs while the metadata and per-step loads below are in flight (bit-identical)
  draw_z((uint32_t)(iter0 + c.key_delta), z);
#endif
  const int64_t row = tq + q0;
  const bool term = ldc(&bi->term) != 0;
  const int kind = term ? 0 : 1;
  const int ls = (kind ? ldc(a.selPPB + g) : ldc(a.selPP + g)) ^ a.law_flip;
  Law<Mdl, T> LA;
  LA.load(a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE);
  const T* tb = a.t_shared ? a.t + q0 : a.t + row;
  const T* Hb = a.H_shared[ls][kind] ? a.H[ls][kind] + (int64_t)q0 * HP : a.H[ls][kind] + row * HP;
  const T* Fb = a.F[ls][kind] + row * D;
  SelMask sel{(uint64_t)sel_u(a.selX[g]), (uint64_t)sel_u(a.selW[g]), g};
  T* const Wd[2] = {a.W[0] + row * M, a.W[1] + row * M};
  T w0[M], dts[RR], sdts[RR], wv[RR][M], cgs[RR][D];
  {
    // the per-step inputs, loaded before any of them is used
    const T* Ws = a.W[sel.w(g) ^ a.ws_flip] + row * M;
#pragma unroll
    for (int k = 0; k < M; ++k) w0[k] = Ws[k];
    T tl[RR], tr[RR], Hs[RR][HP], Fs[RR][D];
#pragma unroll
    for (int r = 0; r < RR; ++r) {
      const int s = min(kRun * lane + r0h + r, nst - 1);
      tl[r] = tb[s];
      tr[r] = tb[s + 1];
#pragma unroll
      for (int k = 0; k < M; ++k) wv[r][k] = Ws[(int64_t)(s + 1) * M + k];
#pragma unroll
      for (int cc = 0; cc < HP; ++cc) Hs[r][cc] = Hb[(int64_t)s * HP + cc];
#pragma unroll
      for (int cc = 0; cc < D; ++cc) Fs[r][cc] = Fb[(int64_t)s * D + cc];
    }
#pragma unroll
    for (int r = 0; r < RR; ++r) {
      dts[r] = tr[r] - tl[r];
      sdts[r] = sqrt(dts[r]);
      T Mg_unused[D * D];
      guide_coeffs<Mdl, T>(LA, Hs[r], Fs[r], Mg_unused, cgs[r]);
    }
  }
  // dW° of the iteration whose normals are in z → dw slots, its e maps
  // e_i = fma(c_i, dt_i, σ·dW°_i) → pt slots (run order), w0n = ρ·W(t0)
  // (dWp keeps this producer's dW° in registers: u's increments after an acceptance)
  T dWp[RR][M];
  auto propose_from = [&](const T (&dWs)[RR][M]) {
#pragma unroll
    for (int r = 0; r < RR; ++r) {
      const int li = lds_ix(kRun * lane + r0h + r);
      T sdW[D];
#pragma unroll
      for (int kk = 0; kk < M; ++kk) {
        S.dw[li][kk] = dWs[r][kk];
        dWp[r][kk] = dWs[r][kk];
      }
      sigma_dw<Mdl, T>(LA, dWs[r], sdW);
#pragma unroll
      for (int p = 0; p < D; ++p) S.pt[li][p] = dfma(cgs[r][p], dts[r], sdW[p]);
    }
#pragma unroll
    for (int k = 0; k < M; ++k) w0n[k] = rho * w0[k];
  };
  auto propose = [&]() {
    T dW[RR][M];
#pragma unroll
    for (int r = 0; r < RR; ++r)
#pragma unroll
      for (int kk = 0; kk < M; ++kk) dW[r][kk] = dfma(rho, wv[r][kk], srho * (sdts[r] * z[r][kk]));
    propose_from(dW);
  };
  // coalesced W° stores of the proposal just handed over (after B1)
  auto store_w = [&]() {
    if (!valid) return;
    T* const Wdb = (sel.w(g) ^ a.wd_flip) ? Wd[1] : Wd[0];
#pragma unroll
    for (int k = 0; k < RW; ++k) {
      const int s = 64 * (h * RW + k) + lane;
      if (s < nst) {
        T wd[M];
#pragma unroll
        for (int kk = 0; kk < M; ++kk) wd[kk] = S.dw[lds_ix(s)][kk];
        store_row_pc<M, T>(Wdb + (int64_t)(s + 1) * M, wd);
      }
    }
    if (h == 0 && lane == 0) store_row_pc<M, T>(Wdb, w0n);
  };
#if !DMT_PC_SETUP_OVERLAP
  draw_z((uint32_t)(iter0 + c.key_delta), z);
#endif
  propose();
  PC_STAMP(256, 2);  // producer 0 of workgroup block 0 (BPW = 4)
  __syncthreads();  // B1 of iteration 0
  if constexpr (!SVC) store_w();
  for (int64_t r0 = 0; r0 < n_iter; ++r0) {
    const bool more = r0 + 1 < n_iter;
    PC_ITSTAMP(256, r0, 4);
    // the next iteration's normals (they depend on the stream key alone), while the consumer
    // runs this one, and both candidates of its pCN increments — u's increments are the
    // current proposal's if the consumer accepts it, else they stay — so that after B2 only a
    // selection, σ·dW° and the e maps stand between the decision and B1 (DMT_PC_SPEC)
    T dWa[RR][M], dWr[RR][M];
    if (more) {
      draw_z((uint32_t)(iter0 + r0 + 1 + c.key_delta), z);
#if DMT_PC_SPEC
#pragma unroll
      for (int r = 0; r < RR; ++r)
#pragma unroll
        for (int kk = 0; kk < M; ++kk) {
          const T q = srho * (sdts[r] * z[r][kk]);
          dWa[r][kk] = dfma(rho, dWp[r][kk], q);
          dWr[r][kk] = dfma(rho, wv[r][kk], q);
        }
#endif
    }
    if constexpr (SVC) {  // the service: W° of iteration n once the host has posted it
      if (!svc_gate(sv, r0, sl)) break;
      store_w();
    }
    PC_ITSTAMP(256, r0, 5);
    __syncthreads();  // B2: decision n
    PC_ITSTAMP(256, r0, 6);
    const bool acc = P.acc != 0;
    if (acc) {  // u's increments ← the accepted proposal's
      sel.mx ^= 1;
      sel.mw ^= 1;
#pragma unroll
      for (int k = 0; k < M; ++k) w0[k] = w0n[k];
    }
#pragma unroll
    for (int r = 0; r < RR; ++r)
#pragma unroll
      for (int k = 0; k < M; ++k) wv[r][k] = acc ? dWp[r][k] : wv[r][k];
    if (more) {
#if DMT_PC_SPEC
      T dWn[RR][M];
#pragma unroll
      for (int r = 0; r < RR; ++r)
#pragma unroll
        for (int k = 0; k < M; ++k) dWn[r][k] = acc ? dWa[r][k] : dWr[r][k];
      propose_from(dWn);
#else
      propose();
#endif
      PC_ITSTAMP(256, r0, 7);
      __syncthreads();  // B1: dW° of iteration n + 1 ready
      if constexpr (!SVC) store_w();
    }
  }
}

// BPW blocks per workgroup (4; 1: every block's waves synchronise only with each other, four
// workgroups per CU — DMT_PC_BPW=1, the service keeps 4)
template <class Mdl, class T, int NP, bool SVC = false, int BPW = 4>
__global__ __launch_bounds__(64 * BPW * (NP + 1), BPW == 4 ? 1 : 2) void k_mcmc_resident_pc(const BlockArgs<T> a,
                                                                      const AcceptArgs c,
                                                                      const int64_t iter0,
                                                                      const int64_t n_iter,
                                                                      double* __restrict__ part,
                                                                      double* __restrict__ nodes,
                                                                      unsigned* __restrict__ counter,
                                                                      double* __restrict__ out3,
                                                                      const SvcArgs sv) {
  __shared__ ResPcLds<Mdl::D, Mdl::M, T> lds[BPW];
  __shared__ SvcLds s_svc;
  if (n_iter <= 0) return;
  PC_STAMP(0, 0);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t blk = a.b0 + (int64_t)blockIdx.x * BPW + (w % BPW);
  const bool valid = blk < a.b1;
  const int role = w / BPW;  // 0: consumer, 1 + h: producer h
#if defined(DMT_PC_STUB_P)  // timing probes (scripts/res_usage.sh, gpu_variants.sh): one role only
  if (role == 0)
    resident_pc_consumer<Mdl, T, NP, SVC>(a, c, iter0, n_iter, part, blk, valid, lds[w & 3], sv, &s_svc);
  else for (int64_t i = 0; i < 2 * n_iter; ++i) __syncthreads();
#elif defined(DMT_PC_STUB_C)
  if (role > 0)
    resident_pc_producer<Mdl, T, NP, SVC>(a, c, iter0, n_iter, blk, valid, role - 1, lds[w & 3], sv, &s_svc);
  else for (int64_t i = 0; i < 2 * n_iter; ++i) __syncthreads();
#else
  if (role == 0)
    resident_pc_consumer<Mdl, T, NP, SVC, BPW>(a, c, iter0, n_iter, part, blk, valid, lds[w % BPW],
                                               sv, &s_svc, nodes);
  else
    resident_pc_producer<Mdl, T, NP, SVC>(a, c, iter0, n_iter, blk, valid, role - 1, lds[w % BPW],
                                          sv, &s_svc);
#endif
#ifndef DMT_PC_NO_TAIL  // timing probe: no in-kernel fetch_ll trees
  if constexpr (!SVC)  // the service forms each iteration's tree as the iteration ends
    persistent_tree_tail<BPW, BPW * (NP + 1), DMT_PC_L1_LOOP != 0>(part, nodes, a.b1 - a.b0,
                                                                    n_iter, counter, out3);
#endif
  PC_STAMP(0, 5);
}

// One draw / re-solve (dmt_draw_proposal, dmt_draw_unit, dmt_recompute_path) of single-segment
// blocks of at most kSChunk steps (d <= 2) with the resident kernel's run-order arithmetic:
// no LDS transposition of the step maps, register-local run trees.
template <class Mdl, class T, int MODE>
__global__ __launch_bounds__(256, 1) void k_block_resident(const BlockArgs<T> a) {
  __shared__ ResLds<Mdl::D, Mdl::M, T> lds[4];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t blk = a.b0 + (int64_t)blockIdx.x * 4 + w;
  if (blk >= a.b1) return;
  resident_block<Mdl, T, MODE, false>(a, AcceptArgs{}, (int64_t)a.iter, 1, nullptr, blk, lds[w]);
}

template <class Mdl, class T>
__global__ __launch_bounds__(64) void k_pathll_wave(const BlockArgs<T> a) {
  constexpr int D = Mdl::D, HP = D * (D + 1) / 2;
  const int lane = threadIdx.x;
  const int64_t blk = a.b0 + (int64_t)blockIdx.x;
  if (blk >= a.b1) return;
  const int64_t r = a.blk_rec[blk];
  const int64_t tq = a.tile_qoff[r];
  const int g0 = a.gfirst[blk], g1 = a.glast[blk];
  const bool term = a.term[blk] != 0;
  T ll;
  {
    const int ls = a.selPP[g0] ^ a.law_flip;
    const double* Lr = a.law[ls][0] + (int64_t)g0 * DMT_LAW_STRIDE;
    const T* Xs = a.X[sel_buf(a.selX[g0], a.xs_flip)];
    const int64_t q = a.seg_q[g0];
    T H0[HP], F0[D], x0[D];
#pragma unroll
    for (int c = 0; c < HP; ++c)
      H0[c] = a.H_shared[ls][0] ? a.H[ls][0][q * HP + c] : a.H[ls][0][(tq + q) * HP + c];
#pragma unroll
    for (int c = 0; c < D; ++c) { F0[c] = a.F[ls][0][(tq + q) * D + c]; x0[c] = Xs[(tq + q) * D + c]; }
    ll = obs_term<D, T>(H0, F0, x0, (T)Lr[DMT_LAW_C0]);
  }
  for (int g = g0; g <= g1; ++g) {
    const int kind = (!term && g == g1) ? 1 : 0;
    const int ls = (kind ? a.selPPB[g] : a.selPP[g]) ^ a.law_flip;
    Law<Mdl, T> L;
    L.load(a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE);
    const int64_t q0 = a.seg_q[g], row = tq + q0;
    const T* tb = a.t_shared ? a.t + q0 : a.t + row;
    const T* Hb = a.H_shared[ls][kind] ? a.H[ls][kind] + q0 * HP : a.H[ls][kind] + row * HP;
    const T* Fb = a.F[ls][kind] + row * D;
    const T* Xb = a.X[sel_buf(a.selX[g], a.xs_flip)] + row * D;
    const int nst = a.seg_np[g] - 1;
    T acc = (T)0;
    for (int c0 = 0; c0 < nst; c0 += 64) {
      const int cnt = nst - c0 < 64 ? nst - c0 : 64;
      const bool valid = lane < cnt;
      const int i = c0 + (valid ? lane : cnt - 1);
      const T dt = tb[i + 1] - tb[i];
      T Hi[HP], Fi[D], xi[D], rr[D], bb[D];
#pragma unroll
      for (int c = 0; c < HP; ++c) Hi[c] = Hb[(int64_t)i * HP + c];
#pragma unroll
      for (int c = 0; c < D; ++c) { Fi[c] = Fb[(int64_t)i * D + c]; xi[c] = Xb[(int64_t)i * D + c]; }
      T G;
      if (a.aux[kind] && L.auxtd) {  // time-dependent auxiliary law (k_block_wave)
        constexpr int CA = kAuxCols<D>;
        T Bq[D * D], bq[D], dq[HP];
        bool trq;
        aux_step<Mdl, T>(L, a.aux[kind] + (row + i) * CA, 1, Bq, bq, dq, trq,
                         [](const T* p) { return *p; });
        G = g_at_aux<Mdl, T>(L, Hi, Fi, xi, rr, bb, Bq, bq, dq, trq);
      } else {
        G = g_at<Mdl, T>(L, Hi, Fi, xi, rr, bb);
      }
      const T csum = wave_tree_sum<T>(valid ? G * dt : (T)0);
      acc = acc + (csum + (T)0);
    }
    ll = ll + acc;
  }
  if (lane == 0) a.ll_out[blk] = (double)ll;
}

// ---------------------------------------------------------------- accept / reject
#if DMT_TU_COMMON
__global__ __launch_bounds__(256) void k_accept(const AcceptArgs a) {
  const int64_t blk = a.b0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= a.b1) return;
  const double E = a.E ? a.E[blk - a.b0]
                       : exp1_draw(a.seed, (uint32_t)a.gfirst[blk] + a.seg_base, a.key_iter, a.salt);
  const double ll = a.ll[blk], llp = a.llp[blk];
  const bool acc = E > -(llp - ll);
  if (acc) {
    for (int g = a.gfirst[blk]; g <= a.glast[blk]; ++g) {
      a.selX[g] = sel_swap(a.selX[g]);
      a.selW[g] = sel_swap(a.selW[g]);
    }
  }
  if (a.hist_len > 0) {
    const int64_t o = (a.mcmciter - 1) * a.nblocks + blk;
    a.acc_hist[o] = acc ? 1 : 0;
    a.ll_hist[o] = ll;
    a.llp_hist[o] = llp;
  }
  if (acc) {
    a.ll[blk] = llp;
    a.llp[blk] = ll;
  }
  if (a.acc_out) a.acc_out[blk - a.b0] = acc ? 1 : 0;
}
#endif  // DMT_TU_COMMON

// accept_reject + the first level of the fetch_ll tree in one pass: each thread decides its
// block (as k_accept), then the 1024-block group reduces (ll, ll°, accepted) exactly as
// k_tree_level<true> does on the post-decision values.  With one group the final
// canonicalised result is written directly.
#if DMT_TU_COMMON
__global__ __launch_bounds__(1024) void k_accept_reduce(const AcceptArgs a, double* __restrict__ out,
                                                        int64_t nout, double* __restrict__ out3) {
  __shared__ double w0[16], w1[16], w2[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t blk = a.b0 + (int64_t)blockIdx.x * 1024 + tid;
  double v0 = 0.0, v1 = 0.0, v2 = 0.0;
  if (blk < a.b1) {
    const double E = a.E ? a.E[blk - a.b0]
                         : exp1_draw(a.seed, (uint32_t)a.gfirst[blk] + a.seg_base, a.key_iter, a.salt);
    double ll = a.ll[blk], llp = a.llp[blk];
    const bool acc = E > -(llp - ll);
    if (acc) {
      for (int g = a.gfirst[blk]; g <= a.glast[blk]; ++g) {
        a.selX[g] = sel_swap(a.selX[g]);
        a.selW[g] = sel_swap(a.selW[g]);
      }
    }
    if (a.hist_len > 0) {
      const int64_t o = (a.mcmciter - 1) * a.nblocks + blk;
      a.acc_hist[o] = acc ? 1 : 0;
      a.ll_hist[o] = ll;
      a.llp_hist[o] = llp;
    }
    if (acc) {
      a.ll[blk] = llp;
      a.llp[blk] = ll;
      const double t = ll; ll = llp; llp = t;
    }
    if (a.acc_out) a.acc_out[blk - a.b0] = acc ? 1 : 0;
    v0 = ll;
    v1 = llp;
    v2 = acc ? 1.0 : 0.0;
  }
  v0 = wave_tree_sum<double>(v0);
  v1 = wave_tree_sum<double>(v1);
  v2 = wave_tree_sum<double>(v2);
  if (lane == 0) { w0[wv] = v0; w1[wv] = v1; w2[wv] = v2; }
  __syncthreads();
  if (wv == 0) {
    v0 = lane < 16 ? w0[lane] : 0.0;
    v1 = lane < 16 ? w1[lane] : 0.0;
    v2 = lane < 16 ? w2[lane] : 0.0;
    v0 = group_tree_sum<16, double>(v0);
    v1 = group_tree_sum<16, double>(v1);
    v2 = group_tree_sum<16, double>(v2);
    if (lane == 0) {
      if (nout == 1) {
        out3[0] = v0 + 0.0;
        out3[1] = v1 + 0.0;
        out3[2] = v2;
      } else {
        out[blockIdx.x] = v0;
        out[nout + blockIdx.x] = v1;
        out[2 * nout + blockIdx.x] = v2;
      }
    }
  }
}
#endif  // DMT_TU_COMMON

// Single-launch form for up to 256 groups of 256 blocks: every workgroup decides its 256
// blocks and reduces them (4 wave trees + one 4-leaf tree = the aligned 256-leaf subtree of
// the fetch_ll tree); the last workgroup to finish (device-scope counter) reduces the group
// partials in group order with the same tree and writes the canonicalised result.
[[maybe_unused]] constexpr int kAccGroup = 256;
#if DMT_TU_COMMON
__global__ __launch_bounds__(kAccGroup) void k_accept_reduce_lb(const AcceptArgs a,
                                                                double* __restrict__ part,
                                                                unsigned* __restrict__ counter,
                                                                double* __restrict__ out3) {
  __shared__ double w0[4], w1[4], w2[4];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t blk = a.b0 + (int64_t)blockIdx.x * kAccGroup + tid;
  double v0 = 0.0, v1 = 0.0, v2 = 0.0;
  if (blk < a.b1) {
    const double E = a.E ? a.E[blk - a.b0]
                         : exp1_draw(a.seed, (uint32_t)a.gfirst[blk] + a.seg_base, a.key_iter, a.salt);
    double ll = a.ll[blk], llp = a.llp[blk];
    const bool acc = E > -(llp - ll);
    if (acc) {
      for (int g = a.gfirst[blk]; g <= a.glast[blk]; ++g) {
        a.selX[g] = sel_swap(a.selX[g]);
        a.selW[g] = sel_swap(a.selW[g]);
      }
    }
    if (a.hist_len > 0) {
      const int64_t o = (a.mcmciter - 1) * a.nblocks + blk;
      a.acc_hist[o] = acc ? 1 : 0;
      a.ll_hist[o] = ll;
      a.llp_hist[o] = llp;
    }
    if (acc) {
      a.ll[blk] = llp;
      a.llp[blk] = ll;
      const double t = ll; ll = llp; llp = t;
    }
    if (a.acc_out) a.acc_out[blk - a.b0] = acc ? 1 : 0;
    v0 = ll;
    v1 = llp;
    v2 = acc ? 1.0 : 0.0;
  }
  v0 = wave_tree_sum<double>(v0);
  v1 = wave_tree_sum<double>(v1);
  v2 = wave_tree_sum<double>(v2);
  if (lane == 0) { w0[wv] = v0; w1[wv] = v1; w2[wv] = v2; }
  __syncthreads();
  if (tid == 0) {
    part[3 * blockIdx.x + 0] = (w0[0] + w0[1]) + (w0[2] + w0[3]);
    part[3 * blockIdx.x + 1] = (w1[0] + w1[1]) + (w1[2] + w1[3]);
    part[3 * blockIdx.x + 2] = (w2[0] + w2[1]) + (w2[2] + w2[3]);
    __threadfence();
    s_last = atomicAdd(counter, 1u) == gridDim.x - 1 ? 1 : 0;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  const int G = (int)gridDim.x;
  v0 = tid < G ? part[3 * tid + 0] : 0.0;
  v1 = tid < G ? part[3 * tid + 1] : 0.0;
  v2 = tid < G ? part[3 * tid + 2] : 0.0;
  v0 = wave_tree_sum<double>(v0);
  v1 = wave_tree_sum<double>(v1);
  v2 = wave_tree_sum<double>(v2);
  __syncthreads();
  if (lane == 0) { w0[wv] = v0; w1[wv] = v1; w2[wv] = v2; }
  __syncthreads();
  if (tid == 0) {
    out3[0] = ((w0[0] + w0[1]) + (w0[2] + w0[3])) + 0.0;
    out3[1] = ((w1[0] + w1[1]) + (w1[2] + w1[3])) + 0.0;
    out3[2] = (w2[0] + w2[1]) + (w2[2] + w2[3]);
    *counter = 0u;  // ready for the next launch (stream-ordered)
  }
}
#endif  // DMT_TU_COMMON

// ---------------------------------------------------------------- guiding term on the device
// recompute_guiding_term!(b) for linear auxiliary laws (src/block.jl:102-110), in the
// canonical chunked form of dmt_filter.h (guiding term; identical to the host
// dmt_guiding_linear).  Three launches per batch of blocks:
//   k_filter_mark   which law (PP / PPb of a non-terminal block's last segment) each segment uses
//   k_filter_scan   one wave per 64-step chunk: the step transitions, their suffix scan → qbuf
//                   (independent of the guiding terms, so every chunk of every block in parallel)
//   k_filter_chain  one wave per block: segments backward from the block end, chunks backward
//                   within a segment; all points of a chunk combine in parallel from the chunk
//                   end's guiding term, lane 0's result is the next chunk's end
// The last segment of a non-terminal block uses its PPb law with the artificial end
// observation frozen by set_obs!.
#if DMT_TU_COMMON
__global__ void k_filter_mark(const FilterArgs a) {
  const int64_t blk = a.b0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= a.b1) return;
  const int g0 = a.gfirst[blk], g1 = a.glast[blk];
  const bool on = !a.only || a.only[blk];
  const bool term = a.term[blk] != 0;
  for (int g = g0; g <= g1; ++g) a.segsel[g] = on ? ((!term && g == g1) ? 2 : 1) : 0;
}
#endif  // DMT_TU_COMMON

template <int D>
__device__ __forceinline__ void filt_law(const FilterArgs& a, int g, int kind, flt::Mat<D>& B,
                                         double* beta, flt::Mat<D>& At, int& slot, bool& td,
                                         bool& tda) {
  slot = (kind ? a.selPPB[g] : a.selPP[g]) ^ a.unit;
  const double* lr = a.law[slot][kind] + (int64_t)g * DMT_LAW_STRIDE;
  td = a.aux[kind] != nullptr && lr[DMT_LAW_AUXTD] != 0.0;
  tda = a.aux[kind] != nullptr && lr[DMT_LAW_AUXTD] == 2.0;
#pragma unroll
  for (int p = 0; p < D; ++p) {
    beta[p] = lr[DMT_LAW_BETA + p];
#pragma unroll
    for (int q = 0; q < D; ++q) {
      B(p, q) = lr[DMT_LAW_BT + p * D + q];
      const int e = flt::packed_ix(D, p, q);
      At(p, q) = lr[DMT_LAW_A + e] - lr[DMT_LAW_DA + e];  // ã = a − (a − ã)
    }
  }
}

// A time-dependent auxiliary law's coefficients of the filter's step q → q + 1 (the per-point
// table, element c of point q at tab[ix(q, c)]), as doubles: the trapezoidal averages
// (v(t_q) + v(t_q+1))·0.5 of B̃ and β̃, which make the exact step transition a second-order
// scheme for the filter ODEs (a constant table gives the table's value exactly)
template <int D, class T, class Ix>
__device__ __forceinline__ void filt_aux_step(const T* tab, Ix ix, int64_t q, flt::Mat<D>& B,
                                              double* beta, flt::Mat<D>& A, bool tda) {
#pragma unroll
  for (int c = 0; c < D * D; ++c) B.a[c] = ((double)tab[ix(q, c)] + (double)tab[ix(q + 1, c)]) * 0.5;
#pragma unroll
  for (int p = 0; p < D; ++p)
    beta[p] = ((double)tab[ix(q, D * D + p)] + (double)tab[ix(q + 1, D * D + p)]) * 0.5;
  if (tda) {  // ã(t) from the table as well (DMT_LAW_AUXTD = 2), its trapezoidal average
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int r = 0; r < D; ++r) {
        const int c = D * D + D + flt::packed_ix(D, p, r);
        A(p, r) = ((double)tab[ix(q, c)] + (double)tab[ix(q + 1, c)]) * 0.5;
      }
  }
}

// chunk j of a segment with np points: steps [lo, lo + cnt), counted from the segment end
__device__ __forceinline__ void filt_chunk(int np, int j, int& lo, int& cnt) {
  const int hi = (np - 1) - flt::kFiltChunk * j;
  lo = hi > flt::kFiltChunk ? hi - flt::kFiltChunk : 0;
  cnt = hi - lo;
}
__device__ __forceinline__ int filt_nchunks(int np) {
  return (np - 1 + flt::kFiltChunk - 1) / flt::kFiltChunk;
}

template <int D>
__device__ __forceinline__ flt::Trans<D> shfl_down_trans(const flt::Trans<D>& x, int k) {
  flt::Trans<D> r;
#pragma unroll
  for (int i = 0; i < D * D; ++i) {
    r.Phi.a[i] = __shfl_down(x.Phi.a[i], k, 64);
    r.K.a[i] = __shfl_down(x.K.a[i], k, 64);
  }
#pragma unroll
  for (int i = 0; i < D; ++i) r.mu[i] = __shfl_down(x.mu[i], k, 64);
  return r;
}

template <class T, int D>
__global__ __launch_bounds__(256) void k_filter_scan(const FilterArgs a, int64_t item0,
                                                     int64_t item1) {
  const int lane = threadIdx.x & 63;
  const int64_t item = item0 + (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (item >= item1) return;
  int lo_g = a.gA, hi_g = a.gB + 1;  // largest g with fchunk_off[g] <= item
  while (hi_g - lo_g > 1) {
    const int mid = (lo_g + hi_g) >> 1;
    if (a.fchunk_off[mid] <= item) lo_g = mid; else hi_g = mid;
  }
  const int g = lo_g;
  const int sel = a.segsel[g];
  if (!sel) return;
  flt::Mat<D> B, At;
  double beta[D];
  int slot;
  bool td, tda;
  filt_law<D>(a, g, sel - 1, B, beta, At, slot, td, tda);
  int lo, cnt;
  filt_chunk(a.seg_np[g], (int)(item - a.fchunk_off[g]), lo, cnt);
  const int64_t r = a.seg_rec[g];
  const int64_t tq = a.tile_qoff[r / a.tw] + a.seg_q[g];
  const int rl = (int)(r % a.tw);
  const T* tt = (const T*)a.t;
  auto tat = [&](int i) -> double {
    return a.t_shared ? (double)tt[a.seg_q[g] + i] : (double)tt[(tq + i) * a.tw + rl];
  };
  flt::Trans<D> q;
  if (lane < cnt) {
    if (td) {
      constexpr int CA = kAuxCols<D>;
      filt_aux_step<D>((const T*)a.aux[sel - 1],
                       [&](int64_t qq, int c) { return ((tq + qq) * CA + c) * a.tw + rl; },
                       lo + lane, B, beta, At, tda);
    }
    q = flt::step_trans<D>(B, beta, At, tat(lo + lane + 1) - tat(lo + lane));
  } else {
    q.Phi = flt::meye<D>();
    q.K = flt::mzero<D>();
#pragma unroll
    for (int i = 0; i < D; ++i) q.mu[i] = 0.0;
  }
#pragma unroll
  for (int k = 1; k < flt::kFiltChunk; k *= 2) {
    const flt::Trans<D> o = shfl_down_trans<D>(q, k);
    if (lane + k < cnt) q = flt::compose<D>(q, o);
  }
  if (lane < cnt) {
    const int64_t p = a.pt_off[g] + lo + lane - a.pA;
    double* Q = a.qbuf + p;
    int c = 0;
#pragma unroll
    for (int i = 0; i < D * D; ++i) Q[(c++) * a.qcap] = q.Phi.a[i];
#pragma unroll
    for (int i = 0; i < D; ++i) Q[(c++) * a.qcap] = q.mu[i];
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int j = i; j < D; ++j) Q[(c++) * a.qcap] = q.K(i, j);
  }
}

// lane 0's double, broadcast through v_readfirstlane (no LDS traffic; every lane is active)
__device__ __forceinline__ double bcast0(double v) {
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}

// per-segment inputs of the chain, all wave-uniform; loaded one segment ahead so that their
// latency overlaps the current segment's chunks
template <int D>
struct FiltSeg {
  static constexpr int HP = D * (D + 1) / 2;
  int np, slot, kind;
  int64_t pt, q0, tq, rl, s;  // s: the segment's first chunk item (fchunk_off)
  double oH[HP], oF[D], oc, ov[D];
};

template <int D>
__device__ __forceinline__ FiltSeg<D> filt_seg(const FilterArgs& a, int g, int g1, bool term) {
  FiltSeg<D> m;
  m.np = a.seg_np[g];
  m.kind = (!term && g == g1) ? 1 : 0;
  m.slot = (m.kind ? a.selPPB[g] : a.selPP[g]) ^ a.unit;
  m.pt = a.pt_off[g];
  m.q0 = a.seg_q[g];
  m.s = a.fchunk_off ? a.fchunk_off[g] : 0;
  const int64_t r = a.seg_rec[g];
  m.tq = a.tile_qoff[r / a.tw];
  m.rl = r % a.tw;
#pragma unroll
  for (int c = 0; c < FiltSeg<D>::HP; ++c) m.oH[c] = a.obsH[(int64_t)g * FiltSeg<D>::HP + c];
#pragma unroll
  for (int p = 0; p < D; ++p) {
    m.oF[p] = a.obsF[(int64_t)g * D + p];
    m.ov[p] = m.kind ? a.obsv[(int64_t)g * D + p] : 0.0;
  }
  m.oc = a.obsc[g];
  return m;
}

// readlane of a wave-uniform lane index (v_readlane_b32 with an SGPR index: no LDS traffic)
__device__ __forceinline__ double rl_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ int64_t rl_i64(int64_t v, int l) {
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, l);
  const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int D>
__device__ __forceinline__ FiltSeg<D> rl_seg(const FiltSeg<D>& m, int l) {
  FiltSeg<D> r;
  r.np = __builtin_amdgcn_readlane(m.np, l);
  r.slot = __builtin_amdgcn_readlane(m.slot, l);
  r.kind = __builtin_amdgcn_readlane(m.kind, l);
  r.pt = rl_i64(m.pt, l);
  r.q0 = rl_i64(m.q0, l);
  r.tq = rl_i64(m.tq, l);
  r.rl = rl_i64(m.rl, l);
  r.s = rl_i64(m.s, l);
#pragma unroll
  for (int c = 0; c < FiltSeg<D>::HP; ++c) r.oH[c] = rl_f64(m.oH[c], l);
#pragma unroll
  for (int p = 0; p < D; ++p) { r.oF[p] = rl_f64(m.oF[p], l); r.ov[p] = rl_f64(m.ov[p], l); }
  r.oc = rl_f64(m.oc, l);
  return r;
}

// The serial part of the few-blocks filter: one wave per block walks its chunks (segments
// backward, chunks backward in time) and carries the guiding term from chunk end to chunk start
// with one combine per chunk, all lanes computing the same values.  The inputs come in lane
// windows — lane k holds the k-th chunk's whole-chunk transition (the scan's Q at the chunk's
// first step) and the k-th segment's observation data — read with v_readlane, so the chain
// itself issues no memory load.  Every chunk's end value goes to tbuf for k_filter_points.
template <class T, int D>
__global__ __launch_bounds__(64) void k_filter_chain(const FilterArgs a) {
  const int64_t blk = a.b0 + blockIdx.x;
  if (blk >= a.b1) return;
  if (a.only && !a.only[blk]) return;
  constexpr int d = D, hp = d * (d + 1) / 2;
  const int lane = threadIdx.x;
  const int g0 = a.gfirst[blk], g1 = a.glast[blk];
  const bool term = a.term[blk] != 0;
  using M = flt::Mat<D>;
  const int64_t ilo = a.fchunk_off[g0], ihi = a.fchunk_off[g1 + 1];
  // chunk window: lane k ↔ item wbase + k
  int64_t wbase = INT64_MIN / 4;  // nothing loaded yet
  flt::Trans<D> wq;
  auto load_window = [&](int64_t base) {
    wbase = base;
    const int64_t item = base + lane;
    if (item >= ilo && item < ihi) {
      int lo_g = g0, hi_g = g1 + 1;  // largest g with fchunk_off[g] <= item
      while (hi_g - lo_g > 1) {
        const int mid = (lo_g + hi_g) >> 1;
        if (a.fchunk_off[mid] <= item) lo_g = mid; else hi_g = mid;
      }
      int lo, cnt;
      filt_chunk(a.seg_np[lo_g], (int)(item - a.fchunk_off[lo_g]), lo, cnt);
      const double* Q = a.qbuf + (a.pt_off[lo_g] + lo - a.pA);
      int c = 0;
#pragma unroll
      for (int i = 0; i < D * D; ++i) wq.Phi.a[i] = Q[(c++) * a.qcap];
#pragma unroll
      for (int i = 0; i < D; ++i) wq.mu[i] = Q[(c++) * a.qcap];
#pragma unroll
      for (int i = 0; i < D; ++i)
#pragma unroll
        for (int j2 = i; j2 < D; ++j2) { const double v = Q[(c++) * a.qcap]; wq.K(i, j2) = v; wq.K(j2, i) = v; }
    } else {
      wq.Phi = flt::meye<D>();
      wq.K = flt::mzero<D>();
#pragma unroll
      for (int i = 0; i < D; ++i) wq.mu[i] = 0.0;
    }
  };
  // segment window: lane k ↔ segment stop − k
  int stop = -1;
  FiltSeg<D> wseg;
  auto load_segs = [&](int top) {
    stop = top;
    const int g = top - lane;
    wseg = filt_seg<D>(a, g >= g0 ? g : g0, g1, term);
  };
  M Hc = flt::mzero<D>();
  double Fc[D], cc = 0.0;
#pragma unroll
  for (int p = 0; p < d; ++p) Fc[p] = 0.0;
  for (int g = g1; g >= g0; --g) {
    if (g > stop || g <= stop - 64) load_segs(g);
    const FiltSeg<D> cur = rl_seg<D>(wseg, stop - g);
    M HT;
    double FT[D], cT = cur.oc;
#pragma unroll
    for (int p = 0; p < d; ++p) {
      FT[p] = cur.oF[p];
#pragma unroll
      for (int q = 0; q < d; ++q) HT(p, q) = cur.oH[flt::packed_ix(d, p, q)];
    }
    if (cur.kind == 1) {
      const double inv = 1.0 / a.art_eps;
      double vv = 0.0;
#pragma unroll
      for (int p = 0; p < d; ++p) {
        const double v = cur.ov[p];
        HT(p, p) += inv;
        FT[p] += inv * v;
        vv += v * v;
      }
      cT += 0.5 * inv * vv + 0.5 * d * (0x1.d67f1c864beb4p+0 + flt::flt_log(a.art_eps));
    } else if (g < g1) {
      HT = flt::madd(HT, Hc);
#pragma unroll
      for (int p = 0; p < d; ++p) FT[p] += Fc[p];
      cT += cc;
    }
    Hc = HT;
#pragma unroll
    for (int p = 0; p < d; ++p) Fc[p] = FT[p];
    cc = cT;
    if (lane == 0) {  // the segment's end point
      T* Ht = (T*)a.H[cur.slot][cur.kind];
      T* Ft = (T*)a.F[cur.slot][cur.kind];
      const int64_t q = cur.tq + cur.q0 + cur.np - 1;
#pragma unroll
      for (int p = 0; p < d; ++p)
#pragma unroll
        for (int r = p; r < d; ++r) Ht[(q * hp + flt::packed_ix(d, p, r)) * a.tw + cur.rl] = (T)Hc(p, r);
#pragma unroll
      for (int p = 0; p < d; ++p) Ft[(q * d + p) * a.tw + cur.rl] = (T)Fc[p];
    }
    const int nch = filt_nchunks(cur.np);
    for (int j = 0; j < nch; ++j) {
      const int64_t item = cur.s + j;
      if (item < wbase || item >= wbase + 64)
        load_window(j == 0 ? max(ilo, item + min(nch, 64) - 64) : item);
      const int wl = (int)(item - wbase);
      flt::Trans<D> q;
#pragma unroll
      for (int i = 0; i < D * D; ++i) { q.Phi.a[i] = rl_f64(wq.Phi.a[i], wl); q.K.a[i] = rl_f64(wq.K.a[i], wl); }
#pragma unroll
      for (int i = 0; i < D; ++i) q.mu[i] = rl_f64(wq.mu[i], wl);
      if (lane == 0) {  // the chunk end's guiding term, for k_filter_points
        double* tb = a.tbuf + (item - a.fchunk_off_h0) * (hp + d + 1);
        int c = 0;
#pragma unroll
        for (int p = 0; p < d; ++p)
#pragma unroll
          for (int r = p; r < d; ++r) tb[c++] = Hc(p, r);
#pragma unroll
        for (int p = 0; p < d; ++p) tb[c++] = Fc[p];
        tb[c] = cc;
      }
      if (!flt::filter_combine<D>(q, Hc, Fc, cc)) {
        if (lane == 0) *a.fail = 1;
        return;
      }
    }
    if (lane == 0) a.law[cur.slot][cur.kind][(int64_t)g * DMT_LAW_STRIDE + DMT_LAW_C0] = cc;
  }
}

// The parallel part of the few-blocks filter: one wave per chunk, every point of the chunk
// combined from the chunk end's guiding term (tbuf) — the same combine the chain made for the
// chunk's first point, so that point is written with the chain's own value.
template <class T, int D>
__global__ __launch_bounds__(256) void k_filter_points(const FilterArgs a, int64_t item0,
                                                       int64_t item1) {
  const int lane = threadIdx.x & 63;
  const int64_t item = item0 + (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (item >= item1) return;
  int lo_g = a.gA, hi_g = a.gB + 1;
  while (hi_g - lo_g > 1) {
    const int mid = (lo_g + hi_g) >> 1;
    if (a.fchunk_off[mid] <= item) lo_g = mid; else hi_g = mid;
  }
  const int g = lo_g;
  const int sel = a.segsel[g];
  if (!sel) return;
  constexpr int d = D, hp = d * (d + 1) / 2;
  const int kind = sel - 1;
  const int slot = (kind ? a.selPPB[g] : a.selPP[g]) ^ a.unit;
  int lo, cnt;
  filt_chunk(a.seg_np[g], (int)(item - a.fchunk_off[g]), lo, cnt);
  if (lane >= cnt) return;
  const double* tb = a.tbuf + (item - a.fchunk_off_h0) * (hp + d + 1);
  flt::Mat<D> H;
  double F[D], c;
  {
    int k = 0;
#pragma unroll
    for (int p = 0; p < d; ++p)
#pragma unroll
      for (int r = p; r < d; ++r) { const double v = tb[k++]; H(p, r) = v; H(r, p) = v; }
#pragma unroll
    for (int p = 0; p < d; ++p) F[p] = tb[k++];
    c = tb[k];
  }
  flt::Trans<D> q;
  {
    const double* Q = a.qbuf + (a.pt_off[g] + lo + lane - a.pA);
    int k = 0;
#pragma unroll
    for (int i = 0; i < D * D; ++i) q.Phi.a[i] = Q[(k++) * a.qcap];
#pragma unroll
    for (int i = 0; i < D; ++i) q.mu[i] = Q[(k++) * a.qcap];
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
      for (int j2 = i; j2 < D; ++j2) { const double v = Q[(k++) * a.qcap]; q.K(i, j2) = v; q.K(j2, i) = v; }
  }
  if (!flt::filter_combine<D>(q, H, F, c)) {
    *a.fail = 1;
    return;
  }
  const int64_t r = a.seg_rec[g];
  const int64_t qq = a.tile_qoff[r / a.tw] + a.seg_q[g] + lo + lane;
  const int rl = (int)(r % a.tw);
  T* Ht = (T*)a.H[slot][kind];
  T* Ft = (T*)a.F[slot][kind];
#pragma unroll
  for (int p = 0; p < d; ++p)
#pragma unroll
    for (int r2 = p; r2 < d; ++r2) Ht[(qq * hp + flt::packed_ix(d, p, r2)) * a.tw + rl] = (T)H(p, r2);
#pragma unroll
  for (int p = 0; p < d; ++p) Ft[(qq * d + p) * a.tw + rl] = (T)F[p];
}

// Many blocks (throughput): one wave per block does everything — the chunk's step
// transitions (lane-parallel), the suffix scan (shuffles) and the combines — with no scratch
// round trip; other waves hide the latency.  Same arithmetic as k_filter_scan + k_filter_chain.
template <class T, int D>
__global__ __launch_bounds__(256) void k_filter_fused(const FilterArgs a) {
  const int64_t blk = a.b0 + (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (blk >= a.b1) return;
  if (a.only && !a.only[blk]) return;
  constexpr int d = D, hp = d * (d + 1) / 2;
  const int lane = threadIdx.x & 63;
  const int g0 = a.gfirst[blk], g1 = a.glast[blk];
  const bool term = a.term[blk] != 0;
  using M = flt::Mat<D>;
  const T* tt = (const T*)a.t;
  M Hc = flt::mzero<D>();
  double Fc[D], cc = 0.0;
#pragma unroll
  for (int p = 0; p < d; ++p) Fc[p] = 0.0;
  for (int g = g1; g >= g0; --g) {
    const FiltSeg<D> cur = filt_seg<D>(a, g, g1, term);
    M B, At;
    double beta[D];
    int slot;
    bool td, tda;
    filt_law<D>(a, g, cur.kind, B, beta, At, slot, td, tda);
    M HT;
    double FT[D], cT = cur.oc;
#pragma unroll
    for (int p = 0; p < d; ++p) {
      FT[p] = cur.oF[p];
#pragma unroll
      for (int q = 0; q < d; ++q) HT(p, q) = cur.oH[flt::packed_ix(d, p, q)];
    }
    if (cur.kind == 1) {
      const double inv = 1.0 / a.art_eps;
      double vv = 0.0;
#pragma unroll
      for (int p = 0; p < d; ++p) {
        const double v = cur.ov[p];
        HT(p, p) += inv;
        FT[p] += inv * v;
        vv += v * v;
      }
      cT += 0.5 * inv * vv + 0.5 * d * (0x1.d67f1c864beb4p+0 + flt::flt_log(a.art_eps));
    } else if (g < g1) {
      HT = flt::madd(HT, Hc);
#pragma unroll
      for (int p = 0; p < d; ++p) FT[p] += Fc[p];
      cT += cc;
    }
    auto ix = [&](int64_t q, int c, int C) -> int64_t { return ((cur.tq + q) * C + c) * a.tw + cur.rl; };
    auto tat = [&](int i) -> double {
      return a.t_shared ? (double)tt[cur.q0 + i] : (double)tt[(cur.tq + cur.q0 + i) * a.tw + cur.rl];
    };
    T* Ht = (T*)a.H[cur.slot][cur.kind];
    T* Ft = (T*)a.F[cur.slot][cur.kind];
    Hc = HT;
#pragma unroll
    for (int p = 0; p < d; ++p) Fc[p] = FT[p];
    cc = cT;
    auto store = [&](int i, const M& Hs, const double* Fs) {
#pragma unroll
      for (int p = 0; p < d; ++p)
#pragma unroll
        for (int q = p; q < d; ++q) Ht[ix(cur.q0 + i, flt::packed_ix(d, p, q), hp)] = (T)Hs(p, q);
#pragma unroll
      for (int p = 0; p < d; ++p) Ft[ix(cur.q0 + i, p, d)] = (T)Fs[p];
    };
    if (lane == 0) store(cur.np - 1, Hc, Fc);
    const int nch = filt_nchunks(cur.np);
    for (int j = 0; j < nch; ++j) {
      int lo, cnt;
      filt_chunk(cur.np, j, lo, cnt);
      flt::Trans<D> q;
      if (lane < cnt) {
        M Bq = B, Aq = At;
        double bq[D];
#pragma unroll
        for (int p = 0; p < d; ++p) bq[p] = beta[p];
        if (td) {
          constexpr int CA = kAuxCols<D>;
          filt_aux_step<D>((const T*)a.aux[cur.kind],
                           [&](int64_t qq, int c) { return ix(cur.q0 + qq, c, CA); }, lo + lane, Bq,
                           bq, Aq, tda);
        }
        q = flt::step_trans<D>(Bq, bq, Aq, tat(lo + lane + 1) - tat(lo + lane));
      } else {
        q.Phi = flt::meye<D>();
        q.K = flt::mzero<D>();
#pragma unroll
        for (int i = 0; i < D; ++i) q.mu[i] = 0.0;
      }
#pragma unroll
      for (int k = 1; k < flt::kFiltChunk; k *= 2) {
        const flt::Trans<D> o = shfl_down_trans<D>(q, k);
        if (lane + k < cnt) q = flt::compose<D>(q, o);
      }
      M H = Hc;
      double F[D], c = cc;
#pragma unroll
      for (int p = 0; p < d; ++p) F[p] = Fc[p];
      const bool ok = lane >= cnt || flt::filter_combine<D>(q, H, F, c);
      if (__ballot(!ok) != 0) {
        if (lane == 0) *a.fail = 1;
        return;
      }
      if (lane < cnt) store(lo + lane, H, F);
#pragma unroll
      for (int i = 0; i < d * d; ++i) Hc.a[i] = bcast0(H.a[i]);
#pragma unroll
      for (int p = 0; p < d; ++p) Fc[p] = bcast0(F[p]);
      cc = bcast0(c);
    }
    if (lane == 0) a.law[cur.slot][cur.kind][(int64_t)g * DMT_LAW_STRIDE + DMT_LAW_C0] = cc;
  }
}

// set_proposal_law!(bb, θ°, pnames) (src/biblock.jl:334-364): for every segment of the block
// and both law kinds, u°'s record ← u's except c(t0) (equalize_law_params!), the named
// parameters ← θ° (DD.set_parameters!), then the fields derived from θ, in this arithmetic
// order (restated in oracle/oracle.py set_law_params):
//   FHN     θ0 = 1/ϵ; σ = (0, σ); a = σσᵀ (packed, one product each);
//           auxlin: B̃ = ((1 − 3(y·y))/ϵ, −1/ϵ; γ, −1), β̃ = ((s + 2((y·y)·y))/ϵ, β), a − ã = 0
//   Lorenz  auxlin: J = (−s, s, 0; r − x2, −1, −x0; x1, x0, −b),
//           β̃_i = f_i − ((J_i0 x0 + J_i1 x1) + J_i2 x2),  f = (s(x1 − x0), x0(r − x2) − x1,
//           x0 x1 − b x2)
//   OU      Θ, μ only (the auxiliary law is fixed)
// crit[blk] = 1 when a record the backward filter uses for this block (PP, or PPb of a
// non-terminal block's last segment) has a different auxiliary law (B̃, β̃, ã = a − (a − ã))
// afterwards.
// r[DMT_LAW_THETA + p] = v with static indices only (r stays in registers)
__device__ __forceinline__ void put_theta(double* r, int p, double v) {
#pragma unroll
  for (int q = 0; q < 12; ++q)
    if (q == p) r[DMT_LAW_THETA + q] = v;
}

__device__ __forceinline__ void derive_law(int model, double* r);

__device__ __forceinline__ void write_params(const ParamArgs& a, double* r) {
  for (int k = 0; k < a.n; ++k) {
    const int p = a.idx[k];
    const double v = a.val[k];
    if (a.model == DMT_MODEL_FHN) {
      if (p == DMT_PAR_FHN_EPS) { r[DMT_LAW_THETA + 4] = v; r[DMT_LAW_THETA + 0] = 1.0 / v; }
      else if (p == DMT_PAR_FHN_SIGMA) r[DMT_LAW_THETA + 5] = v;
      else put_theta(r, p, v);
    } else if (a.model == DMT_MODEL_LORENZ) {
      put_theta(r, p, v);
    } else {
      const int dd = a.d * a.d;
      put_theta(r, p < dd ? p : 9 + (p - dd), v);
    }
  }
  derive_law(a.model, r);
}

// the fields of a law record derived from θ (and, for a linearised auxiliary law, its anchor)
__device__ __forceinline__ void derive_law(int model, double* r) {
  if (model == DMT_MODEL_FHN) {
    const double sg = r[DMT_LAW_THETA + 5];
    r[DMT_LAW_SIGMA + 0] = 0.0;
    r[DMT_LAW_SIGMA + 1] = sg;
    r[DMT_LAW_A + 0] = 0.0 * 0.0;
    r[DMT_LAW_A + 1] = 0.0 * sg;
    r[DMT_LAW_A + 2] = sg * sg;
    if (r[DMT_LAW_AUXLIN] != 0.0) {
      const double e = r[DMT_LAW_THETA + 4], y = r[DMT_LAW_ANCHOR];
      const double yy = y * y;
      r[DMT_LAW_BT + 0] = (1.0 - 3.0 * yy) / e;
      r[DMT_LAW_BT + 1] = -1.0 / e;
      r[DMT_LAW_BT + 2] = r[DMT_LAW_THETA + 2];
      r[DMT_LAW_BT + 3] = -1.0;
      r[DMT_LAW_BETA + 0] = (r[DMT_LAW_THETA + 1] + 2.0 * (yy * y)) / e;
      r[DMT_LAW_BETA + 1] = r[DMT_LAW_THETA + 3];
      for (int i = 0; i < 3; ++i) r[DMT_LAW_DA + i] = 0.0;
      r[DMT_LAW_TRACE] = 0.0;
    }
  } else if (model == DMT_MODEL_LORENZ && r[DMT_LAW_AUXLIN] != 0.0) {
    const double s = r[DMT_LAW_THETA + 0], rr = r[DMT_LAW_THETA + 1], b = r[DMT_LAW_THETA + 2];
    const double x0 = r[DMT_LAW_ANCHOR + 0], x1 = r[DMT_LAW_ANCHOR + 1],
                 x2 = r[DMT_LAW_ANCHOR + 2];
    const double J[9] = {-s, s, 0.0, rr - x2, -1.0, -x0, x1, x0, -b};
    const double f[3] = {s * (x1 - x0), x0 * (rr - x2) - x1, x0 * x1 - b * x2};
#pragma unroll
    for (int i = 0; i < 9; ++i) r[DMT_LAW_BT + i] = J[i];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      r[DMT_LAW_BETA + i] = f[i] - ((J[3 * i] * x0 + J[3 * i + 1] * x1) + J[3 * i + 2] * x2);
  }
}

// one thread per block, or (wg_per_block, for few blocks with many segments) one workgroup per
// block with its threads over the block's (segment, law kind) records
#if DMT_TU_COMMON
__global__ __launch_bounds__(64) void k_set_prop_law(const ParamArgs a, int wg_per_block) {
  const int64_t blk = wg_per_block ? a.b0 + blockIdx.x : a.b0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= a.b1) return;
  const int g0 = a.gfirst[blk], g1 = a.glast[blk];
  const bool term = a.term[blk] != 0;
  bool changed = false;
  constexpr int kAux0 = DMT_LAW_A, kAux1 = DMT_LAW_TRACE + 1;  // a, B̃, β̃, a − ã, (c0), trace
  const int r0 = wg_per_block ? (int)threadIdx.x : 0, st = wg_per_block ? (int)blockDim.x : 1;
  for (int rr = r0; rr < 2 * (g1 - g0 + 1); rr += st) {
    const int g = g0 + (rr >> 1), kind = rr & 1;
    if (!a.law[0][kind]) continue;
    const int s = kind ? a.selPPB[g] : a.selPP[g];
    const double* __restrict__ src = a.law[s][kind] + (int64_t)g * DMT_LAW_STRIDE;
    double* __restrict__ dst = a.law[s ^ 1][kind] + (int64_t)g * DMT_LAW_STRIDE;
    double old[kAux1 - kAux0], rec[DMT_LAW_STRIDE];
#pragma unroll
    for (int i = kAux0; i < kAux1; ++i) old[i - kAux0] = dst[i];
    const double c0 = dst[DMT_LAW_C0];
    const bool old_stale = dst[DMT_LAW_GSTALE] != 0.0;
#pragma unroll
    for (int i = 0; i < DMT_LAW_STRIDE; ++i) rec[i] = src[i];
    rec[DMT_LAW_C0] = c0;
    // critical_change = false: only GP.equalize_law_params! (u°'s law ← u's) can make the update
    // critical (src/biblock.jl:361-362) — compare u°'s auxiliary law before with u's
    bool eq_changed = false;
    if (a.cc_mode == 0) {
#pragma unroll
      for (int i = kAux0; i < kAux1; ++i)
        if (i != DMT_LAW_C0 && __double_as_longlong(old[i - kAux0]) != __double_as_longlong(rec[i]))
          eq_changed = true;
    }
    write_params(a, rec);
    bool aux_changed = false;  // u°'s auxiliary law, before vs after the update
#pragma unroll
    for (int i = kAux0; i < kAux1; ++i)
      if (i != DMT_LAW_C0 && __double_as_longlong(old[i - kAux0]) != __double_as_longlong(rec[i]))
        aux_changed = true;
    const bool used = kind == ((!term && g == g1) ? 1 : 0);
    // the stale-guiding-term bit of u°'s record: false keeps a guiding term whose
    // auxiliary law changed — marked, so that the default treats the record as critical later;
    // a recomputed (or unchanged) guiding term clears it; a record the block does not use keeps it
    if (used && a.cc_mode == 1) {
      changed = true;
      rec[DMT_LAW_GSTALE] = 0.0;
    } else if (used && a.cc_mode == 0) {
      changed = changed || eq_changed;
      rec[DMT_LAW_GSTALE] = ((old_stale || aux_changed) && !eq_changed) ? 1.0 : 0.0;
    } else if (used) {
      changed = changed || aux_changed || old_stale;
      rec[DMT_LAW_GSTALE] = 0.0;
    } else {
      rec[DMT_LAW_GSTALE] = old_stale ? 1.0 : 0.0;
    }
#pragma unroll
    for (int i = 0; i < DMT_LAW_STRIDE; ++i) dst[i] = rec[i];
  }
  if (wg_per_block) {
    changed = __syncthreads_or(changed ? 1 : 0) != 0;
    if (threadIdx.x != 0) return;
  }
  a.crit[blk] = changed ? 1 : 0;
  if (changed) atomicAdd(a.ncrit, 1u);
}
#endif  // DMT_TU_COMMON

// set_obs!(bb) (src/biblock.jl:273-280): the artificial observation of a non-terminal block's
// P_last is the end point of its accepted path; the P_last laws of b and b° that are
// linearised at an anchor (FHN y_T, Lorenz x_T) are re-anchored there and re-derived
// (set_obs!).
template <class T>
__global__ void k_set_obs(int tw, int pk, int d, const T* X0, const T* X1, const T* X2,
                          const uint8_t* selX,
                          const int64_t* tile_qoff, const int32_t* seg_rec, const int32_t* seg_q,
                          const int32_t* seg_np, const int32_t* glast, const uint8_t* term,
                          int64_t b0, int64_t b1, double* obsv, int model, double* lawb0,
                          double* lawb1) {
  const int64_t blk = b0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= b1 || term[blk]) return;
  const int g = glast[blk];
  const int xb = sel_u(selX[g]);
  const T* X = xb == 0 ? X0 : xb == 1 ? X1 : X2;  // u.XX
  const int64_t r = seg_rec[g];
  const int64_t q = seg_q[g] + seg_np[g] - 1;
  double v[3] = {0.0, 0.0, 0.0};
  for (int p = 0; p < d; ++p) {
    v[p] = (double)X[plane_ix(tile_qoff[r / tw] + q, p, d, tw, (int)(r % tw), pk)];
    obsv[(int64_t)g * d + p] = v[p];
  }
  const int na = model == DMT_MODEL_FHN ? 1 : model == DMT_MODEL_LORENZ ? 3 : 0;
  if (!na || !lawb0) return;
  double* recs[2] = {lawb0 + (int64_t)g * DMT_LAW_STRIDE, lawb1 + (int64_t)g * DMT_LAW_STRIDE};
  for (int u = 0; u < 2; ++u) {
    double* rec = recs[u];
    if (rec[DMT_LAW_AUXLIN] == 0.0) continue;
    for (int i = 0; i < na; ++i) rec[DMT_LAW_ANCHOR + i] = v[i];
    derive_law(model, rec);
  }
}

// ---------------------------------------------------------------- small utility kernels
struct FlipArgs {
  uint8_t* sel[4];
  int only_nonterm[4];
};
// selector flips of blocks [b0, b1): one thread per block, or (wg_per_block, for few blocks
// with many segments) one workgroup per block striding over its segments
#if DMT_TU_COMMON
__global__ void k_flip(const FlipArgs f, const int32_t* gfirst, const int32_t* glast,
                       const uint8_t* term, int64_t b0, int64_t b1, int wg_per_block) {
  const int64_t blk = wg_per_block ? b0 + blockIdx.x : b0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= b1) return;
  const int gs = wg_per_block ? (int)threadIdx.x : 0, st = wg_per_block ? (int)blockDim.x : 1;
  const bool tm = term[blk] != 0;
  for (int g = gfirst[blk] + gs; g <= glast[blk]; g += st)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (f.sel[i] && !(f.only_nonterm[i] && tm))
        f.sel[i][g] = i < 2 ? sel_swap(f.sel[i][g]) : (uint8_t)(f.sel[i][g] ^ 1);  // paths: swap u/u°
}
#endif  // DMT_TU_COMMON

#if DMT_TU_COMMON
__global__ void k_swap_ll(double* ll, double* llp, int64_t b0, int64_t b1) {
  const int64_t blk = b0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= b1) return;
  double v = ll[blk];
  ll[blk] = llp[blk];
  llp[blk] = v;
}
#endif  // DMT_TU_COMMON

#if DMT_TU_COMMON
__global__ void k_save_ll(const double* ll, const double* llp, double* llh, double* llph,
                          int64_t nblocks, int64_t it0, int64_t b0, int64_t b1) {
  const int64_t blk = b0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= b1) return;
  llh[it0 * nblocks + blk] = ll[blk];
  llph[it0 * nblocks + blk] = llp[blk];
}
#endif  // DMT_TU_COMMON

__device__ __forceinline__ int64_t find_seg(const int64_t* pt_off, int64_t G, int64_t p) {
  int64_t lo = 0, hi = G;  // largest g with pt_off[g] <= p
  while (hi - lo > 1) {
    int64_t mid = (lo + hi) >> 1;
    if (pt_off[mid] <= p) lo = mid; else hi = mid;
  }
  return lo;
}

// Physical buffer of segment g: path selectors (enc = 1: sel_buf) or law / 0-1 selectors
// (the other slot implied); no selector: buffer 0.
__device__ __forceinline__ int plane_slot(const uint8_t* sel, int enc, int64_t g, int flip) {
  if (!sel) return 0;
  return enc ? sel_buf(sel[g], flip) : ((sel[g] ^ flip) & 1);
}

// Reference layout -> planes.  incr: the source is a cumulative Wiener path; the planes get
// row 0 = W(t0) and row i+1 = W(t_{i+1}) - W(t_i), computed in the working precision.
template <class T>
__global__ void k_to_planes(const int tw, const double* __restrict__ src, T* dst0, T* dst1,
                            T* dst2, const uint8_t* __restrict__ sel, int enc, int flip, int C,
                            int64_t P,
                            const int64_t* __restrict__ pt_off, int64_t G,
                            const int32_t* __restrict__ seg_rec, const int32_t* __restrict__ seg_q,
                            const int64_t* __restrict__ tile_qoff, int incr, int pk) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P * C) return;
  const int64_t p = e / C;
  const int c = (int)(e % C);
  const int64_t g = find_seg(pt_off, G, p);
  const int64_t r = seg_rec[g];
  const int64_t q = seg_q[g] + (p - pt_off[g]);
  const int64_t o = plane_ix(tile_qoff[r / tw] + q, c, C, tw, (int)(r % tw), pk);
  const int slot = plane_slot(sel, enc, g, flip);
  T v = (T)src[e];
  if (incr && p > pt_off[g]) v = v - (T)src[e - C];
  (slot == 0 ? dst0 : slot == 1 ? dst1 : dst2)[o] = v;
}

// planes (increments) -> cumulative reference layout: one thread per (segment, component)
template <class T>
__global__ void k_from_planes_incr(const int tw, double* __restrict__ dst, const T* src0,
                                   const T* src1, const T* src2, const uint8_t* __restrict__ sel,
                                   int enc, int flip, int C,
                                   int64_t G, const int64_t* __restrict__ pt_off,
                                   const int32_t* __restrict__ seg_np,
                                   const int32_t* __restrict__ seg_rec,
                                   const int32_t* __restrict__ seg_q,
                                   const int64_t* __restrict__ tile_qoff, int pk) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= G * C) return;
  const int64_t g = e / C;
  const int c = (int)(e % C);
  const int64_t r = seg_rec[g];
  const int slot = plane_slot(sel, enc, g, flip);
  const T* src = slot == 0 ? src0 : slot == 1 ? src1 : src2;
  T acc = (T)0;
  for (int i = 0; i < seg_np[g]; ++i) {
    const int64_t o = plane_ix(tile_qoff[r / tw] + seg_q[g] + i, c, C, tw, (int)(r % tw), pk);
    acc = i == 0 ? src[o] : acc + src[o];
    dst[(pt_off[g] + i) * C + c] = (double)acc;
  }
}

template <class T>
__global__ void k_from_planes(const int tw, double* __restrict__ dst, const T* src0, const T* src1,
                              const T* src2, const uint8_t* __restrict__ sel, int enc, int flip,
                              int C, int64_t P,
                              const int64_t* __restrict__ pt_off, int64_t G,
                              const int32_t* __restrict__ seg_rec,
                              const int32_t* __restrict__ seg_q,
                              const int64_t* __restrict__ tile_qoff, int pk) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P * C) return;
  const int64_t p = e / C;
  const int c = (int)(e % C);
  const int64_t g = find_seg(pt_off, G, p);
  const int64_t r = seg_rec[g];
  const int64_t q = seg_q[g] + (p - pt_off[g]);
  const int64_t o = plane_ix(tile_qoff[r / tw] + q, c, C, tw, (int)(r % tw), pk);
  const int slot = plane_slot(sel, enc, g, flip);
  dst[e] = (double)(slot == 0 ? src0 : slot == 1 ? src1 : src2)[o];
}

template <class T>
__global__ void k_cast(const double* __restrict__ src, T* __restrict__ dst, int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) dst[e] = (T)src[e];
}

// Deterministic sum over n leaves: the complete adjacent-pair binary tree over the leaves
// padded with zeros to a power of two.  One level reduces aligned groups of
// 1024 leaves per workgroup (64-lane xor-shuffle trees, then a 16-leaf tree of the wave
// sums); levels repeat until one value is left.  A zero-padded group equals the smaller
// power-of-two tree up to the sign of a zero, which the final "+ 0.0" canonicalises.
template <bool FIRST>
__global__ __launch_bounds__(1024) void k_tree_level(const double* __restrict__ a0,
                                                     const double* __restrict__ a1,
                                                     const uint8_t* __restrict__ acc, int64_t n,
                                                     double* __restrict__ out, int64_t nout) {
  __shared__ double w0[16], w1[16], w2[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t i = (int64_t)blockIdx.x * 1024 + tid;
  double v0 = 0.0, v1 = 0.0, v2 = 0.0;
  if (i < n) {
    if (FIRST) {
      v0 = a0[i];
      v1 = a1[i];
      v2 = acc ? (double)acc[i] : 0.0;
    } else {
      v0 = a0[i];
      v1 = a0[n + i];
      v2 = a0[2 * n + i];
    }
  }
  v0 = wave_tree_sum<double>(v0);
  v1 = wave_tree_sum<double>(v1);
  v2 = wave_tree_sum<double>(v2);
  if (lane == 0) { w0[wv] = v0; w1[wv] = v1; w2[wv] = v2; }
  __syncthreads();
  if (wv == 0) {
    v0 = lane < 16 ? w0[lane] : 0.0;
    v1 = lane < 16 ? w1[lane] : 0.0;
    v2 = lane < 16 ? w2[lane] : 0.0;
    v0 = group_tree_sum<16, double>(v0);
    v1 = group_tree_sum<16, double>(v1);
    v2 = group_tree_sum<16, double>(v2);
    if (lane == 0) {
      out[blockIdx.x] = v0;
      out[nout + blockIdx.x] = v1;
      out[2 * nout + blockIdx.x] = v2;
    }
  }
}

#if DMT_TU_COMMON
__global__ void k_tree_final(const double* __restrict__ in, int64_t nout, double* __restrict__ out3) {
  out3[0] = in[0] + 0.0;
  out3[1] = in[nout] + 0.0;
  out3[2] = in[2 * nout];
}
#endif  // DMT_TU_COMMON

#if DMT_TU_COMMON
__global__ void k_debug_philox(uint64_t seed, const uint32_t* ctr, int64_t n, uint32_t* out,
                               double* normals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  U4 c{ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]};
  U4 o = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  out[4 * i] = o.x; out[4 * i + 1] = o.y; out[4 * i + 2] = o.z; out[4 * i + 3] = o.w;
  double z0, z1;
  normal_pair(o, z0, z1);
  normals[2 * i] = z0;
  normals[2 * i + 1] = z1;
}
#endif  // DMT_TU_COMMON

// ---------------------------------------------------------------- launchers
[[maybe_unused]] static inline unsigned nblk(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }
// block counts up to which the per-block utility kernels run one workgroup per block (the
// segments of a block in parallel) instead of one thread per block
[[maybe_unused]] constexpr int64_t kFewBlocks = 2048;

#if DMT_TU_COMMON
thread_local DispatchEvents g_dispatch_events;
thread_local const void* g_recent_k[kRecentKernels];
thread_local unsigned g_recent_n;
#endif

// Launch; when the runtime has armed dispatch events (timed launch), they are attached to
// the kernel's own dispatch packet (hipExtLaunchKernel), so the measured time is the
// kernel's execution as the profiler sees it, without the stream's event-packet overheads.
template <class... KArgs, class... Args>
static void dlaunch(void (*k)(KArgs...), dim3 grid, dim3 block, hipStream_t s, Args... args) {
  g_recent_k[g_recent_n++ % kRecentKernels] = reinterpret_cast<const void*>(k);
  if (g_dispatch_events.start) {
    const DispatchEvents ev = g_dispatch_events;
    g_dispatch_events = DispatchEvents{};
    hipExtLaunchKernelGGL(k, grid, block, 0, s, ev.start, ev.stop, 0, args...);
  } else {
    hipLaunchKernelGGL(k, grid, block, 0, s, args...);
  }
}

#ifndef DMT_KCHUNK
#define DMT_KCHUNK 4
#endif
constexpr int kChunk = DMT_KCHUNK;  // lane-kernel steps per prefetch chunk
static_assert(2 * kChunk <= kPadPoints, "prefetch reads up to 2 chunks past a segment end");
#ifndef DMT_PK_KCHUNK  // the packet kernels' chunk (their guiding-term prefetch distance)
#define DMT_PK_KCHUNK DMT_KCHUNK
#endif
constexpr int kPkChunk = DMT_PK_KCHUNK;
static_assert(2 * kPkChunk <= kPadPoints, "prefetch reads up to 2 chunks past a segment end");

template <class Mdl, class T>
static hipError_t launch_block_t(int mapping, int mode, const void* args, int64_t nwaves,
                                 hipStream_t s) {
  const BlockArgs<T>& a = *static_cast<const BlockArgs<T>*>(args);
  if (nwaves <= 0) return hipSuccess;
  const dim3 grid((unsigned)nwaves);
  if constexpr (Mdl::kLinear) {  // one wave per block, always
    const bool td = a.aux[0] || a.aux[1];  // time-dependent auxiliary laws: scan kernels only
    if constexpr (Mdl::D <= 2) {
      if (a.resident1 && !td) {  // single-segment blocks of <= kSChunk steps: run-order kernel
        const dim3 rgrid((unsigned)((nwaves + 3) / 4)), rblock(256);
        switch (mode) {
          case MODE_PCN: dlaunch(k_block_resident<Mdl, T, MODE_PCN>, rgrid, rblock, s, a); break;
          case MODE_RECOMPUTE: dlaunch(k_block_resident<Mdl, T, MODE_RECOMPUTE>, rgrid, rblock, s, a); break;
          case MODE_FRESH: dlaunch(k_block_resident<Mdl, T, MODE_FRESH>, rgrid, rblock, s, a); break;
          default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
      }
    }
    constexpr int WPB = ScanCfg<Mdl::D, T>::WPB;
    const dim3 grid((unsigned)((nwaves + WPB - 1) / WPB)), sblock(64 * WPB);
    switch (mode * 2 + (td ? 1 : 0)) {
      case 2 * MODE_PCN: dlaunch(k_block_scan<Mdl, T, MODE_PCN>, grid, sblock, s, a); break;
      case 2 * MODE_RECOMPUTE: dlaunch(k_block_scan<Mdl, T, MODE_RECOMPUTE>, grid, sblock, s, a); break;
      case 2 * MODE_FRESH: dlaunch(k_block_scan<Mdl, T, MODE_FRESH>, grid, sblock, s, a); break;
      case 2 * MODE_PCN + 1: dlaunch(k_block_scan<Mdl, T, MODE_PCN, true>, grid, sblock, s, a); break;
      case 2 * MODE_RECOMPUTE + 1: dlaunch(k_block_scan<Mdl, T, MODE_RECOMPUTE, true>, grid, sblock, s, a); break;
      case 2 * MODE_FRESH + 1: dlaunch(k_block_scan<Mdl, T, MODE_FRESH, true>, grid, sblock, s, a); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  } else {
    if (mapping == MAP_WAVE) {
      const dim3 wblock(128);
      switch (mode) {
        case MODE_PCN: dlaunch(k_block_wave<Mdl, T, MODE_PCN>, grid, wblock, s, a); break;
        case MODE_RECOMPUTE: dlaunch(k_block_wave<Mdl, T, MODE_RECOMPUTE>, grid, wblock, s, a); break;
        case MODE_FRESH: dlaunch(k_block_wave<Mdl, T, MODE_FRESH>, grid, wblock, s, a); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
    const dim3 block(64);
    const bool par = a.Z != nullptr;
    if (a.pk) {  // lane packets (fp32 ensembles): k_block_pk, every mode; lane pairs for draws
      if constexpr (sizeof(T) == 4) {
        const bool td = a.aux[0] || a.aux[1];
        if (!par && a.lane_pair && (mode == MODE_PCN || mode == MODE_FRESH)) {
          const dim3 pgrid((unsigned)(2 * nwaves));
          if (mode == MODE_PCN) {
            if (td) dlaunch(k_block_pk_pair<Mdl, T, MODE_PCN, true>, pgrid, block, s, a);
            else dlaunch(k_block_pk_pair<Mdl, T, MODE_PCN>, pgrid, block, s, a);
          } else {
            if (td) dlaunch(k_block_pk_pair<Mdl, T, MODE_FRESH, true>, pgrid, block, s, a);
            else dlaunch(k_block_pk_pair<Mdl, T, MODE_FRESH>, pgrid, block, s, a);
          }
          return hipGetLastError();
        }
        if (mode == MODE_PCN && !par && !td && a.lane_split) {  // producer/consumer waves
          if (DMT_PK_SDT_TABLE && a.t_shared && a.sdt)
            dlaunch(k_block_ps_pk<Mdl, T, kPkChunk, true>, grid, dim3(128), s, a);
          else
            dlaunch(k_block_ps_pk<Mdl, T, kPkChunk, false>, grid, dim3(128), s, a);
          return hipGetLastError();
        }
        switch (mode) {
          case MODE_PCN:
            if (td) {
              if (par) dlaunch(k_block_pk<Mdl, T, MODE_PCN, true, kPkChunk, true>, grid, block, s, a);
              else dlaunch(k_block_pk<Mdl, T, MODE_PCN, false, kPkChunk, true>, grid, block, s, a);
            } else {
              if (par) dlaunch(k_block_pk<Mdl, T, MODE_PCN, true, kPkChunk>, grid, block, s, a);
              else if (DMT_PK_SDT_TABLE && a.t_shared && a.sdt)  // shared grid: √dt table
                dlaunch(k_block_pk<Mdl, T, MODE_PCN, false, kPkChunk, false, true>, grid, block, s, a);
              else dlaunch(k_block_pk<Mdl, T, MODE_PCN, false, kPkChunk>, grid, block, s, a);
            }
            break;
          case MODE_RECOMPUTE:
            if (td) dlaunch(k_block_pk<Mdl, T, MODE_RECOMPUTE, false, kPkChunk, true>, grid, block, s, a);
            else dlaunch(k_block_pk<Mdl, T, MODE_RECOMPUTE, false, kPkChunk>, grid, block, s, a);
            break;
          case MODE_FRESH:
            if (td) {
              if (par) dlaunch(k_block_pk<Mdl, T, MODE_FRESH, true, kPkChunk, true>, grid, block, s, a);
              else dlaunch(k_block_pk<Mdl, T, MODE_FRESH, false, kPkChunk, true>, grid, block, s, a);
            } else {
              if (par) dlaunch(k_block_pk<Mdl, T, MODE_FRESH, true, kPkChunk>, grid, block, s, a);
              else if (DMT_PK_SDT_TABLE && a.t_shared && a.sdt)
                dlaunch(k_block_pk<Mdl, T, MODE_FRESH, false, kPkChunk, false, true>, grid, block, s, a);
              else dlaunch(k_block_pk<Mdl, T, MODE_FRESH, false, kPkChunk>, grid, block, s, a);
            }
            break;
          default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
      } else {
        return hipErrorInvalidValue;  // lane packets are an fp32 layout (dmt_create)
      }
    }
    if (a.aux[0] || a.aux[1]) {  // time-dependent auxiliary laws: the TD instantiation
      switch (mode) {
        case MODE_PCN:
          if (par) dlaunch(k_block<Mdl, T, MODE_PCN, true, kChunk, true>, grid, block, s, a);
          else dlaunch(k_block<Mdl, T, MODE_PCN, false, kChunk, true>, grid, block, s, a);
          break;
        case MODE_RECOMPUTE:
          dlaunch(k_block<Mdl, T, MODE_RECOMPUTE, false, kChunk, true>, grid, block, s, a);
          break;
        case MODE_FRESH:
          if (par) dlaunch(k_block<Mdl, T, MODE_FRESH, true, kChunk, true>, grid, block, s, a);
          else dlaunch(k_block<Mdl, T, MODE_FRESH, false, kChunk, true>, grid, block, s, a);
          break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
    if (!par && a.lane_pair && (mode == MODE_PCN || mode == MODE_FRESH)) {  // lane pairs
      const dim3 pgrid((unsigned)(2 * nwaves));
      if (mode == MODE_PCN) dlaunch(k_block_pair<Mdl, T, MODE_PCN>, pgrid, block, s, a);
      else dlaunch(k_block_pair<Mdl, T, MODE_FRESH>, pgrid, block, s, a);
      return hipGetLastError();
    }
    if (mode == MODE_PCN && !par && a.lane_split) {  // producer/consumer waves (k_block_ps)
      dlaunch(k_block_ps<Mdl, T>, grid, dim3(128), s, a);
      return hipGetLastError();
    }
    switch (mode) {
      case MODE_PCN:
        if (par) dlaunch(k_block<Mdl, T, MODE_PCN, true, kChunk>, grid, block, s, a);
        else dlaunch(k_block<Mdl, T, MODE_PCN, false, kChunk>, grid, block, s, a);
        break;
      case MODE_RECOMPUTE: dlaunch(k_block<Mdl, T, MODE_RECOMPUTE, false, kChunk>, grid, block, s, a); break;
      case MODE_FRESH:
        if (par) dlaunch(k_block<Mdl, T, MODE_FRESH, true, kChunk>, grid, block, s, a);
        else dlaunch(k_block<Mdl, T, MODE_FRESH, false, kChunk>, grid, block, s, a);
        break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
}

// find_W_for_X! on the lane layout: lane = recording tile slot, steps in order (x carried).
template <class Mdl, class T>
__global__ __launch_bounds__(64) void k_invsolve(const BlockArgs<T> a) {
  constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2;
  int64_t tile, blk;
  if (!map_block(a, tile, blk)) return;
  const int lane = threadIdx.x;
  const int64_t tq = a.tile_qoff[tile];
  auto idx = [&](int64_t q, int c, int C) -> int64_t { return ((tq + q) * C + c) * kLanes + lane; };
  auto pidx = [&](int64_t q, int c, int C) -> int64_t { return plane_ix(tq + q, c, C, kLanes, lane, a.pk); };
  auto tload = [&](int64_t q) -> T { return a.t_shared ? a.t[q] : a.t[idx(q, 0, 1)]; };
  const int g0 = a.gfirst[blk], g1 = a.glast[blk];
  const bool term = a.term[blk] != 0;
  for (int g = g0; g <= g1; ++g) {
    const int kind = (!term && g == g1) ? 1 : 0;
    const int ls = (kind ? a.selPPB[g] : a.selPP[g]) ^ a.law_flip;
    const double* lr = a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE;
    Law<Mdl, T> L;
    L.load(lr);
    T siginv[D * D];
#pragma unroll
    for (int c = 0; c < D * D; ++c) siginv[c] = (T)lr[DMT_LAW_SIGINV + c];
    const T* Ht = a.H[ls][kind];
    const T* Ft = a.F[ls][kind];
    const int Hsh = a.H_shared[ls][kind];
    const T* Xs = a.X[sel_buf(a.selX[g], a.xs_flip)];
    T* Wd = a.W[sel_buf(a.selW[g], a.wd_flip)];
    const int64_t q0 = a.seg_q[g];
    const int nst = a.seg_np[g] - 1;
#pragma unroll
    for (int k = 0; k < M; ++k) Wd[pidx(q0, k, M)] = (T)0;  // W(t0) = 0
    T x[D];
#pragma unroll
    for (int c = 0; c < D; ++c) x[c] = Xs[pidx(q0, c, D)];
    T tcur = tload(q0);
    for (int i = 0; i < nst; ++i) {
      const int64_t q = q0 + i;
      T Hi[HP], Fi[D], xn[D], dW[M];
#pragma unroll
      for (int c = 0; c < HP; ++c) Hi[c] = Hsh ? Ht[q * HP + c] : Ht[idx(q, c, HP)];
#pragma unroll
      for (int c = 0; c < D; ++c) { Fi[c] = Ft[idx(q, c, D)]; xn[c] = Xs[pidx(q + 1, c, D)]; }
      const T tn = tload(q + 1);
      inv_step<Mdl, T>(L, siginv, Hi, Fi, tn - tcur, x, xn, dW);
#pragma unroll
      for (int k = 0; k < M; ++k) Wd[pidx(q + 1, k, M)] = dW[k];
#pragma unroll
      for (int c = 0; c < D; ++c) x[c] = xn[c];
      tcur = tn;
    }
  }
}

// find_W_for_X! on the wave layout: a wave per block, 64 consecutive steps per pass.
template <class Mdl, class T>
__global__ __launch_bounds__(64) void k_invsolve_wave(const BlockArgs<T> a) {
  constexpr int D = Mdl::D, M = Mdl::M, HP = D * (D + 1) / 2;
  const int lane = threadIdx.x;
  const int64_t blk = a.b0 + (int64_t)blockIdx.x;
  if (blk >= a.b1) return;
  const int64_t r = a.blk_rec[blk];
  const int64_t tq = a.tile_qoff[r];
  const int g0 = a.gfirst[blk], g1 = a.glast[blk];
  const bool term = a.term[blk] != 0;
  for (int g = g0; g <= g1; ++g) {
    const int kind = (!term && g == g1) ? 1 : 0;
    const int ls = (kind ? a.selPPB[g] : a.selPP[g]) ^ a.law_flip;
    const double* lr = a.law[ls][kind] + (int64_t)g * DMT_LAW_STRIDE;
    Law<Mdl, T> L;
    L.load(lr);
    T siginv[D * D];
#pragma unroll
    for (int c = 0; c < D * D; ++c) siginv[c] = (T)lr[DMT_LAW_SIGINV + c];
    const int64_t q0 = a.seg_q[g], row = tq + q0;
    const T* tb = a.t_shared ? a.t + q0 : a.t + row;
    const T* Hb = a.H_shared[ls][kind] ? a.H[ls][kind] + q0 * HP : a.H[ls][kind] + row * HP;
    const T* Fb = a.F[ls][kind] + row * D;
    const T* Xb = a.X[sel_buf(a.selX[g], a.xs_flip)] + row * D;
    T* Wb = a.W[sel_buf(a.selW[g], a.wd_flip)] + row * M;
    const int nst = a.seg_np[g] - 1;
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < M; ++k) Wb[k] = (T)0;  // W(t0) = 0
    }
    for (int c0 = 0; c0 < nst; c0 += 64) {
      const int i = c0 + lane;
      if (i < nst) {
        T Hi[HP], Fi[D], x[D], xn[D], dW[M];
#pragma unroll
        for (int c = 0; c < HP; ++c) Hi[c] = Hb[(int64_t)i * HP + c];
#pragma unroll
        for (int c = 0; c < D; ++c) {
          Fi[c] = Fb[(int64_t)i * D + c];
          x[c] = Xb[(int64_t)i * D + c];
          xn[c] = Xb[(int64_t)(i + 1) * D + c];
        }
        inv_step<Mdl, T>(L, siginv, Hi, Fi, tb[i + 1] - tb[i], x, xn, dW);
#pragma unroll
        for (int k = 0; k < M; ++k) Wb[(int64_t)(i + 1) * M + k] = dW[k];
      }
    }
  }
}

template <class Mdl, class T>
static hipError_t launch_invsolve_t(int mapping, const void* args, int64_t nwaves, hipStream_t s) {
  const BlockArgs<T>& a = *static_cast<const BlockArgs<T>*>(args);
  if (nwaves <= 0) return hipSuccess;
  if (Mdl::kLinear || mapping == MAP_WAVE)
    dlaunch(k_invsolve_wave<Mdl, T>, dim3((unsigned)nwaves), dim3(64), s, a);
  else
    dlaunch(k_invsolve<Mdl, T>, dim3((unsigned)nwaves), dim3(64), s, a);
  return hipGetLastError();
}

template <class Mdl, class T>
static hipError_t launch_pathll_t(int mapping, const void* args, int64_t nwaves, hipStream_t s) {
  const BlockArgs<T>& a = *static_cast<const BlockArgs<T>*>(args);
  if (nwaves <= 0) return hipSuccess;
  if (Mdl::kLinear || mapping == MAP_WAVE)
    dlaunch(k_pathll_wave<Mdl, T>, dim3((unsigned)nwaves), dim3(64), s, a);
  else if constexpr (!Mdl::kLinear) {
    if (a.aux[0] || a.aux[1])  // time-dependent auxiliary laws: the TD instantiation
      dlaunch(k_pathll<Mdl, T, kChunk, true>, dim3((unsigned)nwaves), dim3(64), s, a);
    else
      dlaunch(k_pathll<Mdl, T, kChunk>, dim3((unsigned)nwaves), dim3(64), s, a);
  }
  return hipGetLastError();
}

// Model dispatch.  One monolithic translation unit by default; the Makefile's split build
// compiles this file seven times in parallel (DMT_TU_GROUP = 0..5: one (precision, model)
// group's kernels and entry points, named <entry>_g<group>; DMT_TU_GROUP = -1 with
// DMT_SPLIT: the model-independent kernels and launchers plus the dispatchers below), so a
// change to one model's kernels rebuilds in a fraction of the time.  Groups: 3·(precision) +
// model — 0 f64 OU, 1 f64 FHN, 2 f64 Lorenz, 3 f32 OU, 4 f32 FHN, 5 f32 Lorenz.
#define DMT_CAT_(a, b) a##b
#define DMT_CAT(a, b) DMT_CAT_(a, b)
#if DMT_TU_GROUP >= 0
#define DMT_ENTRY(name) DMT_CAT(name, DMT_CAT(_g, DMT_TU_GROUP))
#else
#define DMT_ENTRY(name) name
#endif
#define DMT_GROUP_ON(g) (!DMT_SPLIT || DMT_TU_GROUP == (g))
#if DMT_GROUP_ON(0)
#define DMT_CASE_0(KEY, CALL)                                                          \
  if ((KEY).precision == DMT_F64 && (KEY).model == DMT_MODEL_OU) {                     \
    using T = double;                                                                  \
    if ((KEY).d == 1 && (KEY).m == 1) { using Mdl = OU<T, 1, 1>; return CALL; }        \
    if ((KEY).d == 2 && (KEY).m == 2) { using Mdl = OU<T, 2, 2>; return CALL; }        \
    if ((KEY).d == 2 && (KEY).m == 1) { using Mdl = OU<T, 2, 1>; return CALL; }        \
    if ((KEY).d == 3 && (KEY).m == 3) { using Mdl = OU<T, 3, 3>; return CALL; }        \
  }
#else
#define DMT_CASE_0(KEY, CALL)
#endif
#if DMT_GROUP_ON(1)
#define DMT_CASE_1(KEY, CALL)                                                          \
  if ((KEY).precision == DMT_F64 && (KEY).model == DMT_MODEL_FHN) {                    \
    using T = double; using Mdl = FHN<T>; return CALL;                                 \
  }
#else
#define DMT_CASE_1(KEY, CALL)
#endif
#if DMT_GROUP_ON(2)
#define DMT_CASE_2(KEY, CALL)                                                          \
  if ((KEY).precision == DMT_F64 && (KEY).model == DMT_MODEL_LORENZ) {                 \
    using T = double; using Mdl = Lorenz<T>; return CALL;                              \
  }
#else
#define DMT_CASE_2(KEY, CALL)
#endif
#if DMT_GROUP_ON(3)
#define DMT_CASE_3(KEY, CALL)                                                          \
  if ((KEY).precision != DMT_F64 && (KEY).model == DMT_MODEL_OU) {                     \
    using T = float;                                                                   \
    if ((KEY).d == 1 && (KEY).m == 1) { using Mdl = OU<T, 1, 1>; return CALL; }        \
    if ((KEY).d == 2 && (KEY).m == 2) { using Mdl = OU<T, 2, 2>; return CALL; }        \
    if ((KEY).d == 2 && (KEY).m == 1) { using Mdl = OU<T, 2, 1>; return CALL; }        \
    if ((KEY).d == 3 && (KEY).m == 3) { using Mdl = OU<T, 3, 3>; return CALL; }        \
  }
#else
#define DMT_CASE_3(KEY, CALL)
#endif
#if DMT_GROUP_ON(4)
#define DMT_CASE_4(KEY, CALL)                                                          \
  if ((KEY).precision != DMT_F64 && (KEY).model == DMT_MODEL_FHN) {                    \
    using T = float; using Mdl = FHN<T>; return CALL;                                  \
  }
#else
#define DMT_CASE_4(KEY, CALL)
#endif
#if DMT_GROUP_ON(5)
#define DMT_CASE_5(KEY, CALL)                                                          \
  if ((KEY).precision != DMT_F64 && (KEY).model == DMT_MODEL_LORENZ) {                 \
    using T = float; using Mdl = Lorenz<T>; return CALL;                               \
  }
#else
#define DMT_CASE_5(KEY, CALL)
#endif
#define DMT_DISPATCH(KEY, CALL)                                                        \
  do {                                                                                 \
    DMT_CASE_0(KEY, CALL)                                                              \
    DMT_CASE_1(KEY, CALL)                                                              \
    DMT_CASE_2(KEY, CALL)                                                              \
    DMT_CASE_3(KEY, CALL)                                                              \
    DMT_CASE_4(KEY, CALL)                                                              \
    DMT_CASE_5(KEY, CALL)                                                              \
    return hipErrorInvalidValue;                                                       \
  } while (0)

#if !DMT_SPLIT || DMT_TU_GROUP >= 0
hipError_t DMT_ENTRY(launch_block_kernel)(const ModelKey& k, int mapping, int mode, const void* args,
                               int64_t nwaves, hipStream_t s) {
  DMT_DISPATCH(k, (launch_block_t<Mdl, T>(mapping, mode, args, nwaves, s)));
}

template <class Mdl, class T>
static hipError_t launch_mcmc_t(const void* args, const AcceptArgs& c, int64_t iter0, int64_t n,
                                double* part, int64_t nwaves, int resident, double* out3,
                                unsigned* counter, hipStream_t s) {
  if constexpr (Mdl::kLinear) {
    const BlockArgs<T>& a = *static_cast<const BlockArgs<T>*>(args);
    if (nwaves <= 0) return hipSuccess;
    // part[n][3][nwaves], then the tree nodes [n][3][ceil(nwaves / WPB)] (dmt_mcmc_run sizes it)
    double* nodes = part + 3 * n * nwaves;
    // time-dependent auxiliary laws: k_mcmc_scan's TD instantiation only (the register-resident
    // kernels take the law's own B̃, β̃; dmt_mcmc_run does not pick them while a table is present)
    const bool td = a.aux[0] || a.aux[1];
    if (td && resident) return hipErrorInvalidValue;
    if constexpr (Mdl::D <= 2) {
      if (resident >= 2) {  // producer / consumer waves (k_mcmc_resident_pc), resident - 1 producers
        const SvcArgs none{};
        if (resident == 3)
          dlaunch(k_mcmc_resident_pc<Mdl, T, 2>, dim3((unsigned)((nwaves + 3) / 4)), dim3(768), s,
                  a, c, iter0, n, part, nodes, counter, out3, none);
        else if (resident == 4)  // one block per workgroup
          dlaunch(k_mcmc_resident_pc<Mdl, T, 1, false, 1>, dim3((unsigned)nwaves), dim3(128), s,
                  a, c, iter0, n, part, nodes, counter, out3, none);
        else
          dlaunch(k_mcmc_resident_pc<Mdl, T, 1>, dim3((unsigned)((nwaves + 3) / 4)), dim3(512), s,
                  a, c, iter0, n, part, nodes, counter, out3, none);
        return hipGetLastError();
      }
      if (resident) {
        dlaunch(k_mcmc_resident<Mdl, T>, dim3((unsigned)((nwaves + 3) / 4)), dim3(256), s, a, c,
                iter0, n, part, nodes, counter, out3);
        return hipGetLastError();
      }
    }
    constexpr int WPB = ScanCfg<Mdl::D, T>::WPB;
    if (td)
      dlaunch(k_mcmc_scan<Mdl, T, true>, dim3((unsigned)((nwaves + WPB - 1) / WPB)), dim3(64 * WPB),
              s, a, c, iter0, n, part, nodes, counter, out3);
    else
      dlaunch(k_mcmc_scan<Mdl, T>, dim3((unsigned)((nwaves + WPB - 1) / WPB)), dim3(64 * WPB), s, a,
              c, iter0, n, part, nodes, counter, out3);
    return hipGetLastError();
  } else {
    return hipErrorInvalidValue;
  }
}

// The service's workgroups wait on one another through the host (an iteration is posted once
// every block has finished the previous one): the whole grid must be resident at once.
template <class Mdl, class T>
static bool svc_fits_t(int64_t nwaves, int producers, int n_cu) {
  if constexpr (Mdl::kLinear && Mdl::D <= 2) {
    int per_cu = 0;
    const hipError_t e =
        producers == 2
            ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                  &per_cu, reinterpret_cast<const void*>(k_mcmc_resident_pc<Mdl, T, 2, true>), 768, 0)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                  &per_cu, reinterpret_cast<const void*>(k_mcmc_resident_pc<Mdl, T, 1, true>), 512, 0);
    return e == hipSuccess && (nwaves + 3) / 4 <= (int64_t)per_cu * n_cu;
  } else {
    return false;
  }
}

template <class Mdl, class T>
static hipError_t launch_svc_t(const void* args, const AcceptArgs& c, int64_t iter0, int64_t cap,
                               double* part, int64_t nwaves, int producers, int n_cu,
                               const SvcArgs& sv, hipStream_t s) {
  if constexpr (Mdl::kLinear && Mdl::D <= 2) {
    const BlockArgs<T>& a = *static_cast<const BlockArgs<T>*>(args);
    if (nwaves <= 0) return hipSuccess;
    const dim3 grid((unsigned)((nwaves + 3) / 4));
    if (!svc_fits_t<Mdl, T>(nwaves, producers, n_cu)) return hipErrorCooperativeLaunchTooLarge;
    if (producers == 2)
      dlaunch(k_mcmc_resident_pc<Mdl, T, 2, true>, grid, dim3(768), s, a, c, iter0, cap, part,
              nullptr, nullptr, nullptr, sv);
    else
      dlaunch(k_mcmc_resident_pc<Mdl, T, 1, true>, grid, dim3(512), s, a, c, iter0, cap, part,
              nullptr, nullptr, nullptr, sv);
    return hipGetLastError();
  } else {
    return hipErrorInvalidValue;
  }
}

hipError_t DMT_ENTRY(launch_mcmc_service)(const ModelKey& k, const void* args, const AcceptArgs& c,
                               int64_t iter0, int64_t capacity, double* part, int64_t nwaves,
                               int producers, int n_cu, const SvcArgs& sv, hipStream_t s) {
  DMT_DISPATCH(k, (launch_svc_t<Mdl, T>(args, c, iter0, capacity, part, nwaves, producers, n_cu,
                                        sv, s)));
}

static hipError_t DMT_ENTRY(svc_fits_err)(const ModelKey& k, int64_t nwaves, int producers, int n_cu) {
  DMT_DISPATCH(k, (svc_fits_t<Mdl, T>(nwaves, producers, n_cu) ? hipSuccess
                                                                 : hipErrorCooperativeLaunchTooLarge));
}

bool DMT_ENTRY(mcmc_service_fits)(const ModelKey& k, int64_t nwaves, int producers, int n_cu) {
  return DMT_ENTRY(svc_fits_err)(k, nwaves, producers, n_cu) == hipSuccess;
}

hipError_t DMT_ENTRY(launch_mcmc_persistent)(const ModelKey& k, const void* args, const AcceptArgs& c,
                                  int64_t iter0, int64_t n_iter, double* part, int64_t nwaves,
                                  int resident, double* out3, unsigned* counter, hipStream_t s) {
  DMT_DISPATCH(k, (launch_mcmc_t<Mdl, T>(args, c, iter0, n_iter, part, nwaves, resident, out3,
                                         counter, s)));
}

hipError_t DMT_ENTRY(launch_invsolve_kernel)(const ModelKey& k, int mapping, const void* args,
                                  int64_t nwaves, hipStream_t s) {
  DMT_DISPATCH(k, (launch_invsolve_t<Mdl, T>(mapping, args, nwaves, s)));
}

hipError_t DMT_ENTRY(launch_pathll_kernel)(const ModelKey& k, int mapping, const void* args, int64_t nwaves,
                                hipStream_t s) {
  DMT_DISPATCH(k, (launch_pathll_t<Mdl, T>(mapping, args, nwaves, s)));
}

#endif  // !DMT_SPLIT || DMT_TU_GROUP >= 0

#if DMT_SPLIT && DMT_TU_GROUP < 0
// the split build's dispatchers: the (precision, model) group's translation unit
#define DMT_DECL_GROUP(G)                                                                        \
  hipError_t launch_block_kernel_g##G(const ModelKey&, int, int, const void*, int64_t, hipStream_t); \
  hipError_t launch_mcmc_service_g##G(const ModelKey&, const void*, const AcceptArgs&, int64_t,    \
                                      int64_t, double*, int64_t, int, int, const SvcArgs&,         \
                                      hipStream_t);                                                \
  bool mcmc_service_fits_g##G(const ModelKey&, int64_t, int, int);                                 \
  hipError_t launch_mcmc_persistent_g##G(const ModelKey&, const void*, const AcceptArgs&, int64_t, \
                                         int64_t, double*, int64_t, int, double*, unsigned*,       \
                                         hipStream_t);                                             \
  hipError_t launch_invsolve_kernel_g##G(const ModelKey&, int, const void*, int64_t, hipStream_t); \
  hipError_t launch_pathll_kernel_g##G(const ModelKey&, int, const void*, int64_t, hipStream_t);
DMT_DECL_GROUP(0)
DMT_DECL_GROUP(1)
DMT_DECL_GROUP(2)
DMT_DECL_GROUP(3)
DMT_DECL_GROUP(4)
DMT_DECL_GROUP(5)
static int model_group(const ModelKey& k) {
  if (k.model < DMT_MODEL_OU || k.model > DMT_MODEL_LORENZ) return -1;
  return (k.precision == DMT_F64 ? 0 : 3) + k.model;
}
#define DMT_FORWARD(RET, FN, ...)                      \
  switch (model_group(k)) {                            \
    case 0: return FN##_g0(__VA_ARGS__);               \
    case 1: return FN##_g1(__VA_ARGS__);               \
    case 2: return FN##_g2(__VA_ARGS__);               \
    case 3: return FN##_g3(__VA_ARGS__);               \
    case 4: return FN##_g4(__VA_ARGS__);               \
    case 5: return FN##_g5(__VA_ARGS__);               \
    default: return RET;                               \
  }
hipError_t launch_block_kernel(const ModelKey& k, int mapping, int mode, const void* args,
                               int64_t nwaves, hipStream_t s) {
  DMT_FORWARD(hipErrorInvalidValue, launch_block_kernel, k, mapping, mode, args, nwaves, s);
}
hipError_t launch_mcmc_service(const ModelKey& k, const void* args, const AcceptArgs& c,
                               int64_t iter0, int64_t capacity, double* part, int64_t nwaves,
                               int producers, int n_cu, const SvcArgs& sv, hipStream_t s) {
  DMT_FORWARD(hipErrorInvalidValue, launch_mcmc_service, k, args, c, iter0, capacity, part, nwaves,
              producers, n_cu, sv, s);
}
bool mcmc_service_fits(const ModelKey& k, int64_t nwaves, int producers, int n_cu) {
  DMT_FORWARD(false, mcmc_service_fits, k, nwaves, producers, n_cu);
}
hipError_t launch_mcmc_persistent(const ModelKey& k, const void* args, const AcceptArgs& c,
                                  int64_t iter0, int64_t n_iter, double* part, int64_t nwaves,
                                  int resident, double* out3, unsigned* counter, hipStream_t s) {
  DMT_FORWARD(hipErrorInvalidValue, launch_mcmc_persistent, k, args, c, iter0, n_iter, part, nwaves,
              resident, out3, counter, s);
}
hipError_t launch_invsolve_kernel(const ModelKey& k, int mapping, const void* args,
                                  int64_t nwaves, hipStream_t s) {
  DMT_FORWARD(hipErrorInvalidValue, launch_invsolve_kernel, k, mapping, args, nwaves, s);
}
hipError_t launch_pathll_kernel(const ModelKey& k, int mapping, const void* args, int64_t nwaves,
                                hipStream_t s) {
  DMT_FORWARD(hipErrorInvalidValue, launch_pathll_kernel, k, mapping, args, nwaves, s);
}
#endif  // DMT_SPLIT && DMT_TU_GROUP < 0

#if DMT_TU_COMMON
hipError_t launch_backward_filter(int precision, const FilterArgs& a, hipStream_t s) {
  const int64_t n = a.b1 - a.b0;
  if (n <= 0) return hipSuccess;
  if (!a.fused) hipLaunchKernelGGL(k_filter_mark, dim3(nblk(n, 64)), dim3(64), 0, s, a);
  // the host copies of fchunk_off bound the scan's work items: passed in via qbuf's batch
  const int64_t item0 = a.fchunk_off_h0, item1 = a.fchunk_off_h1;
#define DMT_FILTER_LAUNCH(T, D)                                                                \
  do {                                                                                         \
    if (a.fused) {                                                                             \
      hipLaunchKernelGGL((k_filter_fused<T, D>), dim3(nblk(n, 4)), dim3(256), 0, s, a);        \
      break;                                                                                   \
    }                                                                                          \
    if (item1 > item0)                                                                         \
      hipLaunchKernelGGL((k_filter_scan<T, D>), dim3(nblk(item1 - item0, 4)), dim3(256), 0, s, \
                         a, item0, item1);                                                     \
    hipLaunchKernelGGL((k_filter_chain<T, D>), dim3(n), dim3(64), 0, s, a);                    \
    if (item1 > item0)                                                                         \
      hipLaunchKernelGGL((k_filter_points<T, D>), dim3(nblk(item1 - item0, 4)), dim3(256), 0,  \
                         s, a, item0, item1);                                                  \
  } while (0)
  if (precision == DMT_F64) {
    if (a.d == 1) DMT_FILTER_LAUNCH(double, 1);
    else if (a.d == 2) DMT_FILTER_LAUNCH(double, 2);
    else DMT_FILTER_LAUNCH(double, 3);
  } else {
    if (a.d == 1) DMT_FILTER_LAUNCH(float, 1);
    else if (a.d == 2) DMT_FILTER_LAUNCH(float, 2);
    else DMT_FILTER_LAUNCH(float, 3);
  }
#undef DMT_FILTER_LAUNCH
  return hipGetLastError();
}

hipError_t launch_set_prop_law(const ParamArgs& a, hipStream_t s) {
  const int64_t n = a.b1 - a.b0;
  if (n <= 0) return hipSuccess;
  if (n <= kFewBlocks)
    hipLaunchKernelGGL(k_set_prop_law, dim3((unsigned)n), dim3(64), 0, s, a, 1);
  else
    hipLaunchKernelGGL(k_set_prop_law, dim3(nblk(n, 64)), dim3(64), 0, s, a, 0);
  return hipGetLastError();
}

hipError_t launch_set_obs(int precision, int tw, int pk, int d, const void* X0, const void* X1,
                          const void* X2, const uint8_t* selX, const int64_t* tile_qoff, const int32_t* seg_rec,
                          const int32_t* seg_q, const int32_t* seg_np, const int32_t* glast,
                          const uint8_t* term, int64_t b0, int64_t b1, double* obsv,
                          int model, double* lawb0, double* lawb1, hipStream_t s) {
  const int64_t n = b1 - b0;
  if (n <= 0) return hipSuccess;
  if (precision == DMT_F64)
    k_set_obs<double><<<nblk(n, 256), 256, 0, s>>>(tw, pk, d, (const double*)X0, (const double*)X1,
                                                   (const double*)X2, selX, tile_qoff, seg_rec, seg_q, seg_np, glast,
                                                   term, b0, b1, obsv, model, lawb0, lawb1);
  else
    k_set_obs<float><<<nblk(n, 256), 256, 0, s>>>(tw, pk, d, (const float*)X0, (const float*)X1,
                                                  (const float*)X2, selX,
                                                  tile_qoff, seg_rec, seg_q, seg_np, glast, term,
                                                  b0, b1, obsv, model, lawb0, lawb1);
  return hipGetLastError();
}

hipError_t launch_accept(const AcceptArgs& a, hipStream_t s) {
  const int64_t n = a.b1 - a.b0;
  if (n <= 0) return hipSuccess;
  dlaunch(k_accept, dim3(nblk(n, 256)), dim3(256), s, a);
  return hipGetLastError();
}

hipError_t launch_to_planes(int precision, int tw, const double* src, void* dst0, void* dst1,
                            const uint8_t* sel, int flip, int C, int64_t P, const int64_t* pt_off,
                            int64_t G, const int32_t* seg_rec, const int32_t* seg_q,
                            const int64_t* tile_qoff, hipStream_t s, int incr, void* dst2,
                            int enc, int pk) {
  const int64_t n = P * C;
  if (n <= 0) return hipSuccess;
  if (precision == DMT_F64)
    k_to_planes<double><<<nblk(n, 256), 256, 0, s>>>(tw, src, (double*)dst0, (double*)dst1,
                                                      (double*)dst2, sel, enc, flip, C, P, pt_off,
                                                      G, seg_rec, seg_q, tile_qoff, incr, pk);
  else
    k_to_planes<float><<<nblk(n, 256), 256, 0, s>>>(tw, src, (float*)dst0, (float*)dst1,
                                                     (float*)dst2, sel, enc, flip, C, P, pt_off, G,
                                                     seg_rec, seg_q, tile_qoff, incr, pk);
  return hipGetLastError();
}

hipError_t launch_from_planes_incr(int precision, int tw, double* dst, const void* src0,
                                   const void* src1, const uint8_t* sel, int flip, int C,
                                   int64_t G, const int64_t* pt_off, const int32_t* seg_np,
                                   const int32_t* seg_rec, const int32_t* seg_q,
                                   const int64_t* tile_qoff, hipStream_t s, const void* src2,
                                   int enc, int pk) {
  const int64_t n = G * C;
  if (n <= 0) return hipSuccess;
  if (precision == DMT_F64)
    k_from_planes_incr<double><<<nblk(n, 64), 64, 0, s>>>(tw, dst, (const double*)src0,
                                                          (const double*)src1, (const double*)src2,
                                                          sel, enc, flip, C, G,
                                                          pt_off, seg_np, seg_rec, seg_q, tile_qoff, pk);
  else
    k_from_planes_incr<float><<<nblk(n, 64), 64, 0, s>>>(tw, dst, (const float*)src0,
                                                         (const float*)src1, (const float*)src2,
                                                         sel, enc, flip, C, G,
                                                         pt_off, seg_np, seg_rec, seg_q, tile_qoff, pk);
  return hipGetLastError();
}

hipError_t launch_from_planes(int precision, int tw, double* dst, const void* src0, const void* src1,
                              const uint8_t* sel, int flip, int C, int64_t P,
                              const int64_t* pt_off, int64_t G, const int32_t* seg_rec,
                              const int32_t* seg_q, const int64_t* tile_qoff, hipStream_t s,
                              const void* src2, int enc, int pk) {
  const int64_t n = P * C;
  if (n <= 0) return hipSuccess;
  if (precision == DMT_F64)
    k_from_planes<double><<<nblk(n, 256), 256, 0, s>>>(tw, dst, (const double*)src0,
                                                        (const double*)src1, (const double*)src2,
                                                        sel, enc, flip, C, P,
                                                        pt_off, G, seg_rec, seg_q, tile_qoff, pk);
  else
    k_from_planes<float><<<nblk(n, 256), 256, 0, s>>>(tw, dst, (const float*)src0, (const float*)src1,
                                                       (const float*)src2, sel, enc, flip, C, P,
                                                       pt_off, G, seg_rec, seg_q,
                                                       tile_qoff, pk);
  return hipGetLastError();
}

hipError_t launch_cast(int precision, const double* src, void* dst, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (precision == DMT_F64)
    k_cast<double><<<nblk(n, 256), 256, 0, s>>>(src, (double*)dst, n);
  else
    k_cast<float><<<nblk(n, 256), 256, 0, s>>>(src, (float*)dst, n);
  return hipGetLastError();
}

template <class T>
__global__ void k_cast_back(const T* __restrict__ src, double* __restrict__ dst, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (double)src[i];
}

hipError_t launch_cast_back(int precision, const void* src, double* dst, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (precision == DMT_F64)
    k_cast_back<double><<<nblk(n, 256), 256, 0, s>>>((const double*)src, dst, n);
  else
    k_cast_back<float><<<nblk(n, 256), 256, 0, s>>>((const float*)src, dst, n);
  return hipGetLastError();
}

hipError_t launch_block_sum(const double* ll, const double* llp, const uint8_t* acc, int64_t n,
                            double* work, double* out3, hipStream_t s) {
  // work: 2 × 3 × ceil(n/1024) doubles (ping-pong partials)
  int64_t groups = (n + 1023) / 1024;
  if (groups < 1) groups = 1;
  double* bufs[2] = {work, work + 3 * groups};
  k_tree_level<true><<<(unsigned)groups, 1024, 0, s>>>(ll, llp, acc, n, bufs[0], groups);
  // (a single group still goes through k_tree_final for the canonical "+ 0.0")
  int cur = 0;
  int64_t m = groups;
  while (m > 1) {
    const int64_t g2 = (m + 1023) / 1024;
    k_tree_level<false><<<(unsigned)g2, 1024, 0, s>>>(bufs[cur], nullptr, nullptr, m, bufs[cur ^ 1], g2);
    cur ^= 1;
    m = g2;
  }
  k_tree_final<<<1, 1, 0, s>>>(bufs[cur], m, out3);
  return hipGetLastError();
}

// accept + fetch tree (ll, ll°, accepted of this iteration) over [b0, b1)
hipError_t launch_accept_reduce(const AcceptArgs& a, double* work, double* lb, double* out3,
                                hipStream_t s) {
  const int64_t n = a.b1 - a.b0;
  if (n <= 1024) {  // one 1024-thread workgroup: decisions and the whole tree, no second pass
    dlaunch(k_accept_reduce, dim3(1), dim3(1024), s, a, work, (int64_t)1, out3);
    return hipGetLastError();
  }
  {  // single launch while the group partials fit one workgroup
    const int64_t groups = std::max<int64_t>(1, (n + kAccGroup - 1) / kAccGroup);
    if (groups <= kAccGroup) {
      // work layout: [3 * 256] partials, then the counter
      dlaunch(k_accept_reduce_lb, dim3((unsigned)groups), dim3(kAccGroup), s, a, lb,
              reinterpret_cast<unsigned*>(lb + 3 * kAccGroup), out3);
      return hipGetLastError();
    }
  }
  int64_t groups = (n + 1023) / 1024;
  if (groups < 1) groups = 1;
  double* bufs[2] = {work, work + 3 * groups};
  dlaunch(k_accept_reduce, dim3((unsigned)groups), dim3(1024), s, a, bufs[0], groups, out3);
  if (groups == 1) return hipGetLastError();
  int cur = 0;
  int64_t m = groups;
  while (m > 1) {
    const int64_t g2 = (m + 1023) / 1024;
    k_tree_level<false><<<(unsigned)g2, 1024, 0, s>>>(bufs[cur], nullptr, nullptr, m, bufs[cur ^ 1], g2);
    cur ^= 1;
    m = g2;
  }
  k_tree_final<<<1, 1, 0, s>>>(bufs[cur], m, out3);
  return hipGetLastError();
}

hipError_t launch_flip(uint8_t* sel0, uint8_t* sel1, uint8_t* sel2, uint8_t* sel3,
                       const int32_t* gfirst, const int32_t* glast, const uint8_t* term,
                       int32_t swap_ppb_nonterm_only, int64_t b0, int64_t b1, hipStream_t s) {
  const int64_t n = b1 - b0;
  if (n <= 0) return hipSuccess;
  FlipArgs f{{sel0, sel1, sel2, sel3}, {0, 0, 0, swap_ppb_nonterm_only}};
  if (!sel0 && !sel1 && !sel2 && !sel3) return hipSuccess;
  if (n <= kFewBlocks)
    k_flip<<<(unsigned)n, 64, 0, s>>>(f, gfirst, glast, term, b0, b1, 1);
  else
    k_flip<<<nblk(n, 256), 256, 0, s>>>(f, gfirst, glast, term, b0, b1, 0);
  return hipGetLastError();
}

hipError_t launch_swap_ll(double* ll, double* llp, int64_t b0, int64_t b1, hipStream_t s) {
  const int64_t n = b1 - b0;
  if (n <= 0) return hipSuccess;
  k_swap_ll<<<nblk(n, 256), 256, 0, s>>>(ll, llp, b0, b1);
  return hipGetLastError();
}

hipError_t launch_save_ll(const double* ll, const double* llp, double* llh, double* llph,
                          int64_t nblocks, int64_t it0, int64_t b0, int64_t b1, hipStream_t s) {
  const int64_t n = b1 - b0;
  if (n <= 0) return hipSuccess;
  k_save_ll<<<nblk(n, 256), 256, 0, s>>>(ll, llp, llh, llph, nblocks, it0, b0, b1);
  return hipGetLastError();
}

hipError_t launch_debug_philox(uint64_t seed, const uint32_t* ctr, int64_t n, uint32_t* out,
                               double* normals, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  k_debug_philox<<<nblk(n, 256), 256, 0, s>>>(seed, ctr, n, out, normals);
  return hipGetLastError();
}

#endif  // DMT_TU_COMMON
}  // namespace dmt

#if DMT_AUX_CHECK && !DMT_SPLIT
extern "C" int dmt_debug_aux_check(unsigned long long* out, int n) {
  // out[0] = count of out-of-table aux reads, then up to kAuxDbg records of 8 words
  // (block, segment, kind, row, step, chunk start, chunk count, table present); resets them
  if (n < 1 + 8 * dmt::kAuxDbg) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(dmt::g_aux_dbg), sizeof(dmt::g_aux_dbg)) != hipSuccess) return -3;
  static const unsigned long long zero[1 + 8 * dmt::kAuxDbg] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(dmt::g_aux_dbg), zero, sizeof(zero)) != hipSuccess) return -4;
  return 0;
}
#endif
