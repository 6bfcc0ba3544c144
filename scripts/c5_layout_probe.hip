// c5_layout_probe.hip — timing probe (not product code): the C5 lane draw's memory pattern under
// different path-plane layouts, with the real per-step arithmetic (Philox4x32-10 + Box–Muller
// normals, the Lorenz guided Euler step with σ = I, its Girsanov term) so that issue and memory
// interact as in k_block<Lorenz<float>>.
//
// Per step and lane: read t (shared), H (6) and F (3) rows of a read-only table, u's W increment
// (3) from the lane's u buffer; write X° (3) and W° (3) to the lane's proposal buffer.
// Layouts of the path planes (X, W; H/F keep the row layout):
//   P = 1   row layout of today: ((q·C + c)·64 + lane)            — a wave's row is 256 B
//   P = 8/16/32  lane packets: a lane's P consecutive points of one component contiguous,
//           row q at position q + P − 1 so that chunk rows c0+1 … c0+4 are one aligned float4
// Selectors: uniform (every lane reads buffer 0, writes buffer 1), mixed (lane u ∈ {0,1} at
// random, writes 1 − u), consolidated (row layout only: mixed, the minority copies its u.X/u.W
// to the majority's buffer during the sweep and every proposal goes to the other buffer — what
// path_plan does for C5 today).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/c5_layout_probe.hip \
//          -o scripts/c5_layout_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <random>

#include "../diffusionmcmctools.jl_amd/csrc/dmt_device.h"

using namespace dmt;
typedef float T;
typedef Lorenz<T> Mdl;
constexpr int D = 3, M = 3, HP = 6, K = 4;

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(2);                                                                          \
    }                                                                                   \
  } while (0)

struct Args {
  const T* t;  // shared grid [rows]
  const T* H;  // row layout, per tile [rows][HP][64]
  const T* F;  // [rows][D][64]
  T* X[3];
  T* W[3];
  const uint8_t* u;  // [R] lane's u buffer
  int64_t rows;      // padded point rows per tile (path planes and tables alike)
  int nst;           // steps per segment
  double* ll;        // [R]
  uint32_t iter;
};

template <int P>
__device__ __forceinline__ int64_t ppos(int64_t q, int c, int C, int lane) {
  if constexpr (P == 1) {
    return (q * C + c) * 64 + lane;
  } else {
    const int64_t p = q + P - 1;
    return ((p / P) * C + c) * 64 * P + (int64_t)lane * P + (p % P);
  }
}

// SEL: 0 uniform, 1 mixed, 2 consolidated (P = 1 only), 3 reads mixed (buffer u) / writes
// uniform (buffer 2), 4 reads uniform (buffer 0) / writes mixed (buffer 1 + u)
template <int P, int SEL>
__global__ __launch_bounds__(64) void k_probe(const Args a) {
  const int lane = threadIdx.x;
  const int64_t tile = blockIdx.x;
  const int64_t r = tile * 64 + lane;
  const int64_t tb = tile * a.rows;  // first row of the tile
  const int64_t pbD = tb * D * 64, pbM = tb * M * 64;
  int u = SEL == 0 ? 0 : a.u[r];
  int pbuf = 1 - u;
  bool copy = false;
  if (SEL == 2) {  // consolidate: the majority's buffer m; minority copies, proposals to 1 − m
    const int c1 = __popcll(__ballot(u == 1));
    const int m = c1 > 32 ? 1 : 0;
    copy = u != m;
    pbuf = 1 - m;
  }
  const T* Ws = a.W[SEL == 4 ? 0 : u] + pbM;
  if (SEL == 3) pbuf = 2;
  if (SEL == 4) pbuf = 1 + u;
  T* Wd = a.W[pbuf] + pbM;
  T* Xd = a.X[pbuf] + pbD;
  T* Xcd = a.X[1 - pbuf] + pbD;  // consolidation target (= the majority's buffer)
  const T* Xcs = a.X[u] + pbD;
  T* Wcd = a.W[1 - pbuf] + pbM;
  const T* Hb = a.H + tb * HP * 64 + lane;
  const T* Fb = a.F + tb * D * 64 + lane;

  Law<Mdl, T> L;
  L.th[0] = 10; L.th[1] = 28; L.th[2] = 8.0f / 3;
  for (int i = 0; i < D * D; ++i) L.Bt[i] = (i % 4 == 0) ? -1.0f : 0.1f;
  for (int i = 0; i < D; ++i) L.beta[i] = 0.5f;
  for (int i = 0; i < HP; ++i) L.da[i] = 0;
  L.trace = false;
  L.unit = true;
  L.auxtd = false;

  T x[D] = {1.0f, 1.0f, 20.0f};
  T tcur = a.t[0];
  T ll = 0;
  const T rho = 0.9f, srho = sqrtf(1 - 0.81f);
  const uint32_t seg = (uint32_t)r;
  struct Chunk {
    T t[K], H[K][HP], F[K][D], W[K][M];
  };
  auto load = [&](int c0, Chunk& c) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int64_t i = c0 + j;
      c.t[j] = a.t[i + 1];
#pragma unroll
      for (int e = 0; e < HP; ++e) c.H[j][e] = Hb[(i * HP + e) * 64];
#pragma unroll
      for (int e = 0; e < D; ++e) c.F[j][e] = Fb[(i * D + e) * 64];
    }
    if constexpr (P == 1) {
#pragma unroll
      for (int j = 0; j < K; ++j)
#pragma unroll
        for (int k = 0; k < M; ++k) c.W[j][k] = Ws[ppos<P>(c0 + j + 1, k, M, lane)];
    } else {
#pragma unroll
      for (int k = 0; k < M; ++k) {
        const float4 v = *(const float4*)&Ws[ppos<P>(c0 + 1, k, M, lane)];
        c.W[0][k] = v.x; c.W[1][k] = v.y; c.W[2][k] = v.z; c.W[3][k] = v.w;
      }
    }
  };
  const int nfull = a.nst - a.nst % K;
  Chunk cur, nxt;
  load(0, cur);
  for (int c0 = 0; c0 < nfull; c0 += K) {
    load(c0 + K, nxt);
    T Z[K][M];
#pragma unroll
    for (int bq = 0; bq < K * M / 4; ++bq) {
      T zb[4];
      normal_block(philox4x32_10(U4{(uint32_t)(c0 * M / 4 + bq), seg, a.iter, 0u}, 0x1234u, 0x5678u),
                   zb);
#pragma unroll
      for (int e = 0; e < 4; ++e) Z[(4 * bq + e) / M][(4 * bq + e) % M] = zb[e];
    }
    T ox[K][D], ow[K][M], cx[K][D];
    T g[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const T dt = cur.t[j] - tcur;
      const T sdt = sqrtf(dt);
      T dW[M];
#pragma unroll
      for (int k = 0; k < M; ++k) dW[k] = dfma(rho, cur.W[j][k], srho * (sdt * Z[j][k]));
      T rr[D], b[D], Mg[D * D], cg[D];
      const T G = g_at<Mdl, T>(L, cur.H[j], cur.F[j], x, rr, b);
      guide_coeffs_unit<Mdl, T>(cur.H[j], cur.F[j], Mg, cg);
      euler_step<Mdl, T>(Mg, cg, b, dt, dW, x);
      tcur = cur.t[j];
      g[j] = G * dt;
#pragma unroll
      for (int p = 0; p < D; ++p) ox[j][p] = x[p];
#pragma unroll
      for (int k = 0; k < M; ++k) ow[j][k] = dW[k];
    }
    ll += (g[0] + g[1]) + (g[2] + g[3]);
    if constexpr (SEL == 2) {  // the minority's u.X of these rows (read before overwritten)
      if (copy) {
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
          for (int p = 0; p < D; ++p) cx[j][p] = Xcs[ppos<P>(c0 + j + 1, p, D, lane)];
#pragma unroll
        for (int j = 0; j < K; ++j) {
#pragma unroll
          for (int p = 0; p < D; ++p) Xcd[ppos<P>(c0 + j + 1, p, D, lane)] = cx[j][p];
#pragma unroll
          for (int k = 0; k < M; ++k) Wcd[ppos<P>(c0 + j + 1, k, M, lane)] = cur.W[j][k];
        }
      }
    }
    if constexpr (P == 1) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
#pragma unroll
        for (int p = 0; p < D; ++p) Xd[ppos<P>(c0 + j + 1, p, D, lane)] = ox[j][p];
#pragma unroll
        for (int k = 0; k < M; ++k) Wd[ppos<P>(c0 + j + 1, k, M, lane)] = ow[j][k];
      }
    } else {
#pragma unroll
      for (int p = 0; p < D; ++p)
        *(float4*)&Xd[ppos<P>(c0 + 1, p, D, lane)] = make_float4(ox[0][p], ox[1][p], ox[2][p], ox[3][p]);
#pragma unroll
      for (int k = 0; k < M; ++k)
        *(float4*)&Wd[ppos<P>(c0 + 1, k, M, lane)] = make_float4(ow[0][k], ow[1][k], ow[2][k], ow[3][k]);
    }
    cur = nxt;
  }
  a.ll[r] = (double)ll + (double)x[0];
}

// Full lane packets: the path planes' row q at position q + P − 1 of the lane's P-point packets
// (P·4 B each: 32 B for P = 8, 64 B for P = 16); per packet of P steps, the lane loads its u.W
// packet (P/4 float4 per component, back to back, one packet ahead) and stores its X°/W°
// packets whole at the packet's end — every access a whole 32/64-byte piece of ONE lane, so a
// lane's buffer never shares a piece with another lane's.  SEL: 0 uniform, 1 mixed.
template <int P, int SEL>
__global__ __launch_bounds__(64) void k_probe_pk(const Args a) {
  const int lane = threadIdx.x;
  const int64_t tile = blockIdx.x;
  const int64_t r = tile * 64 + lane;
  const int64_t tb = tile * a.rows;
  const int64_t pbD = tb * D * 64, pbM = tb * M * 64;
  const int u = SEL == 0 ? 0 : a.u[r];
  const int pbuf = 1 - u;
  const T* Ws = a.W[u] + pbM;
  T* Wd = a.W[pbuf] + pbM;
  T* Xd = a.X[pbuf] + pbD;
  const T* Hb = a.H + tb * HP * 64 + lane;
  const T* Fb = a.F + tb * D * 64 + lane;
  Law<Mdl, T> L;
  L.th[0] = 10; L.th[1] = 28; L.th[2] = 8.0f / 3;
  for (int i = 0; i < D * D; ++i) L.Bt[i] = (i % 4 == 0) ? -1.0f : 0.1f;
  for (int i = 0; i < D; ++i) L.beta[i] = 0.5f;
  for (int i = 0; i < HP; ++i) L.da[i] = 0;
  L.trace = false;
  L.unit = true;
  L.auxtd = false;
  T x[D] = {1.0f, 1.0f, 20.0f};
  T tcur = a.t[0];
  T ll = 0;
  const T rho = 0.9f, srho = sqrtf(1 - 0.81f);
  const uint32_t seg = (uint32_t)r;
  constexpr int NV = P / 4;
  // packet j (rows jP+1 … jP+P) of component c: lane's float4 pieces
  auto pk = [&](const T* base, int64_t j, int c, int C) -> const float4* {
    return (const float4*)&base[(((j + 1) * C + c) * 64 + lane) * P];
  };
  auto pkw = [&](T* base, int64_t j, int c, int C) -> float4* {
    return (float4*)&base[(((j + 1) * C + c) * 64 + lane) * P];
  };
  float4 wcur[M][NV], wnxt[M][NV];
  auto loadw = [&](int64_t j, float4 (&w)[M][NV]) {
#pragma unroll
    for (int k = 0; k < M; ++k)
#pragma unroll
      for (int v = 0; v < NV; ++v) w[k][v] = pk(Ws, j, k, M)[v];
  };
  struct Chunk {
    T t[K], H[K][HP], F[K][D];
  };
  auto load = [&](int c0, Chunk& c) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int64_t i = c0 + j;
      c.t[j] = a.t[i + 1];
#pragma unroll
      for (int e = 0; e < HP; ++e) c.H[j][e] = Hb[(i * HP + e) * 64];
#pragma unroll
      for (int e = 0; e < D; ++e) c.F[j][e] = Fb[(i * D + e) * 64];
    }
  };
  const int npk = a.nst / P;
  Chunk cur, nxt;
  load(0, cur);
  loadw(0, wcur);
  for (int j = 0; j < npk; ++j) {
    loadw(j + 1, wnxt);  // padded rows keep the last packet's prefetch in bounds
    float4 ox[D][NV], ow[M][NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c0 = j * P + 4 * v;
      load(c0 + K, nxt);
      T Z[K][M];
#pragma unroll
      for (int bq = 0; bq < K * M / 4; ++bq) {
        T zb[4];
        normal_block(philox4x32_10(U4{(uint32_t)(c0 * M / 4 + bq), seg, a.iter, 0u}, 0x1234u, 0x5678u),
                     zb);
#pragma unroll
        for (int e = 0; e < 4; ++e) Z[(4 * bq + e) / M][(4 * bq + e) % M] = zb[e];
      }
      T g[K], oxs[K][D], ows[K][M];
#pragma unroll
      for (int q = 0; q < K; ++q) {
        const T dt = cur.t[q] - tcur;
        const T sdt = sqrtf(dt);
        T dW[M];
#pragma unroll
        for (int k = 0; k < M; ++k) {
          const float4 w4 = wcur[k][v];
          const T wu = q == 0 ? w4.x : q == 1 ? w4.y : q == 2 ? w4.z : w4.w;
          dW[k] = dfma(rho, wu, srho * (sdt * Z[q][k]));
        }
        T rr[D], b[D], Mg[D * D], cg[D];
        const T G = g_at<Mdl, T>(L, cur.H[q], cur.F[q], x, rr, b);
        guide_coeffs_unit<Mdl, T>(cur.H[q], cur.F[q], Mg, cg);
        euler_step<Mdl, T>(Mg, cg, b, dt, dW, x);
        tcur = cur.t[q];
        g[q] = G * dt;
#pragma unroll
        for (int p = 0; p < D; ++p) oxs[q][p] = x[p];
#pragma unroll
        for (int k = 0; k < M; ++k) ows[q][k] = dW[k];
      }
      ll += (g[0] + g[1]) + (g[2] + g[3]);
#pragma unroll
      for (int p = 0; p < D; ++p) ox[p][v] = make_float4(oxs[0][p], oxs[1][p], oxs[2][p], oxs[3][p]);
#pragma unroll
      for (int k = 0; k < M; ++k) ow[k][v] = make_float4(ows[0][k], ows[1][k], ows[2][k], ows[3][k]);
      cur = nxt;
    }
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int v = 0; v < NV; ++v) pkw(Xd, j, p, D)[v] = ox[p][v];
#pragma unroll
    for (int k = 0; k < M; ++k)
#pragma unroll
      for (int v = 0; v < NV; ++v) pkw(Wd, j, k, M)[v] = ow[k][v];
#pragma unroll
    for (int k = 0; k < M; ++k)
#pragma unroll
      for (int v = 0; v < NV; ++v) wcur[k][v] = wnxt[k][v];
  }
  a.ll[r] = (double)ll + (double)x[0];
}

// Full lane packets with the outputs staged in LDS (k_probe_lds): per packet of P steps each
// lane writes its X°/W° values to its own LDS rows step by step and, at the packet's end, reads
// them back as 16-byte pieces and stores whole packets (P·4 B per component: 128 B for P = 32,
// one lane per 128-byte line); u.W's next packet is loaded piece by piece into the registers
// just consumed (one packet ahead).  SEL: 0 uniform, 1 mixed.
template <int P, int SEL>
__global__ __launch_bounds__(64) void k_probe_lds(const Args a) {
  constexpr int NV = P / 4, C6 = D + M;
  __shared__ float stage[C6][P][65];  // [component][step][lane] (+1: conflict-free)
  const int lane = threadIdx.x;
  const int64_t tile = blockIdx.x;
  const int64_t r = tile * 64 + lane;
  const int64_t tb = tile * a.rows;
  const int64_t pbD = tb * D * 64, pbM = tb * M * 64;
  const int u = SEL == 0 ? 0 : a.u[r];
  const int pbuf = 1 - u;
  const T* Ws = a.W[u] + pbM;
  T* Wd = a.W[pbuf] + pbM;
  T* Xd = a.X[pbuf] + pbD;
  const T* Hb = a.H + tb * HP * 64 + lane;
  const T* Fb = a.F + tb * D * 64 + lane;
  Law<Mdl, T> L;
  L.th[0] = 10; L.th[1] = 28; L.th[2] = 8.0f / 3;
  for (int i = 0; i < D * D; ++i) L.Bt[i] = (i % 4 == 0) ? -1.0f : 0.1f;
  for (int i = 0; i < D; ++i) L.beta[i] = 0.5f;
  for (int i = 0; i < HP; ++i) L.da[i] = 0;
  L.trace = false;
  L.unit = true;
  L.auxtd = false;
  T x[D] = {1.0f, 1.0f, 20.0f};
  T tcur = a.t[0];
  T ll = 0;
  const T rho = 0.9f, srho = sqrtf(1 - 0.81f);
  const uint32_t seg = (uint32_t)r;
  auto pk = [&](const T* base, int64_t j, int c, int C) -> const float4* {
    return (const float4*)&base[(((j + 1) * C + c) * 64 + lane) * P];
  };
  auto pkw = [&](T* base, int64_t j, int c, int C) -> float4* {
    return (float4*)&base[(((j + 1) * C + c) * 64 + lane) * P];
  };
  float4 wc[M][NV];
#pragma unroll
  for (int k = 0; k < M; ++k)
#pragma unroll
    for (int v = 0; v < NV; ++v) wc[k][v] = pk(Ws, 0, k, M)[v];
  struct Chunk {
    T t[K], H[K][HP], F[K][D];
  };
  auto load = [&](int c0, Chunk& c) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int64_t i = c0 + j;
      c.t[j] = a.t[i + 1];
#pragma unroll
      for (int e = 0; e < HP; ++e) c.H[j][e] = Hb[(i * HP + e) * 64];
#pragma unroll
      for (int e = 0; e < D; ++e) c.F[j][e] = Fb[(i * D + e) * 64];
    }
  };
  const int npk = a.nst / P;
  Chunk cur, nxt;
  load(0, cur);
  for (int j = 0; j < npk; ++j) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c0 = j * P + 4 * v;
      load(c0 + K, nxt);
      T Z[K][M];
#pragma unroll
      for (int bq = 0; bq < K * M / 4; ++bq) {
        T zb[4];
        normal_block(philox4x32_10(U4{(uint32_t)(c0 * M / 4 + bq), seg, a.iter, 0u}, 0x1234u, 0x5678u),
                     zb);
#pragma unroll
        for (int e = 0; e < 4; ++e) Z[(4 * bq + e) / M][(4 * bq + e) % M] = zb[e];
      }
      T g[K];
#pragma unroll
      for (int q = 0; q < K; ++q) {
        const T dt = cur.t[q] - tcur;
        const T sdt = sqrtf(dt);
        T dW[M];
#pragma unroll
        for (int k = 0; k < M; ++k) {
          const float4 w4 = wc[k][v];
          const T wu = q == 0 ? w4.x : q == 1 ? w4.y : q == 2 ? w4.z : w4.w;
          dW[k] = dfma(rho, wu, srho * (sdt * Z[q][k]));
        }
        T rr[D], b[D], Mg[D * D], cg[D];
        const T G = g_at<Mdl, T>(L, cur.H[q], cur.F[q], x, rr, b);
        guide_coeffs_unit<Mdl, T>(cur.H[q], cur.F[q], Mg, cg);
        euler_step<Mdl, T>(Mg, cg, b, dt, dW, x);
        tcur = cur.t[q];
        g[q] = G * dt;
#pragma unroll
        for (int p = 0; p < D; ++p) stage[p][4 * v + q][lane] = x[p];
#pragma unroll
        for (int k = 0; k < M; ++k) stage[D + k][4 * v + q][lane] = dW[k];
      }
      ll += (g[0] + g[1]) + (g[2] + g[3]);
#pragma unroll
      for (int k = 0; k < M; ++k) wc[k][v] = pk(Ws, j + 1, k, M)[v];  // next packet's piece
      cur = nxt;
    }
#pragma unroll
    for (int c = 0; c < C6; ++c) {
      float4* dst = c < D ? pkw(Xd, j, c, D) : pkw(Wd, j, c - D, M);
#pragma unroll
      for (int v = 0; v < NV; ++v)
        dst[v] = make_float4(stage[c][4 * v][lane], stage[c][4 * v + 1][lane],
                             stage[c][4 * v + 2][lane], stage[c][4 * v + 3][lane]);
    }
  }
  a.ll[r] = (double)ll + (double)x[0];
}

template <int P, int SEL>
static double run_lds(const Args& a, int ntiles, int reps, const char* name) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  k_probe_lds<P, SEL><<<ntiles, 64>>>(a);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) k_probe_lds<P, SEL><<<ntiles, 64>>>(a);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double steps = (double)ntiles * 64 * (a.nst / P) * P;
  printf("{\"variant\": \"%s\", \"P\": %d, \"sel\": %d, \"us_per_draw\": %.1f, \"frac_72B\": %.3f}\n",
         name, P, SEL, us, steps * 72 / (us * 1e-6) / 8e12);
  fflush(stdout);
  return us;
}

template <int P, int SEL>
static double run_pk(const Args& a, int ntiles, int reps, const char* name) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  k_probe_pk<P, SEL><<<ntiles, 64>>>(a);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) k_probe_pk<P, SEL><<<ntiles, 64>>>(a);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double steps = (double)ntiles * 64 * (a.nst / P) * P;
  printf("{\"variant\": \"%s\", \"P\": %d, \"sel\": %d, \"us_per_draw\": %.1f, \"frac_72B\": %.3f}\n",
         name, P, SEL, us, steps * 72 / (us * 1e-6) / 8e12);
  fflush(stdout);
  return us;
}

template <int P, int SEL>
static double run(const Args& a, int ntiles, int reps, const char* name) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  k_probe<P, SEL><<<ntiles, 64>>>(a);  // warm-up
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) k_probe<P, SEL><<<ntiles, 64>>>(a);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double steps = (double)ntiles * 64 * a.nst;
  printf("{\"variant\": \"%s\", \"P\": %d, \"sel\": %d, \"us_per_draw\": %.1f, \"frac_72B\": %.3f}\n",
         name, P, SEL, us, steps * 72 / (us * 1e-6) / 8e12);
  fflush(stdout);
  return us;
}

int main(int argc, char** argv) {
  const int ntiles = argc > 1 ? atoi(argv[1]) : 512;
  const int nst = 2000;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const char* only = argc > 3 ? argv[3] : nullptr;
  const int64_t rows = ((nst + 1 + 2 * K + 32 + 31) / 32) * 32 + 96;  // room for prefetch + packet shift
  const int64_t R = (int64_t)ntiles * 64;
  Args a{};
  a.rows = rows;
  a.nst = nst;
  a.iter = 1;
  std::vector<T> th(rows);
  for (int64_t i = 0; i < rows; ++i) th[i] = (T)i * 1e-3f;
  T* dt;
  CHECK(hipMalloc(&dt, rows * sizeof(T)));
  CHECK(hipMemcpy(dt, th.data(), rows * sizeof(T), hipMemcpyHostToDevice));
  a.t = dt;
  auto alloc = [&](int C, float v) {
    T* p;
    const size_t n = (size_t)ntiles * rows * C * 64;
    CHECK(hipMalloc(&p, n * sizeof(T)));
    std::vector<T> h(n, v);
    CHECK(hipMemcpy(p, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
    return p;
  };
  a.H = alloc(HP, 0.01f);
  a.F = alloc(D, 0.02f);
  for (int b = 0; b < 3; ++b) {
    a.X[b] = alloc(D, 0.0f);
    a.W[b] = alloc(M, 0.001f);
  }
  std::vector<uint8_t> hu(R);
  std::mt19937 g(7);
  for (auto& v : hu) v = (uint8_t)(g() & 1);
  uint8_t* du;
  CHECK(hipMalloc(&du, R));
  CHECK(hipMemcpy(du, hu.data(), R, hipMemcpyHostToDevice));
  a.u = du;
  CHECK(hipMalloc(&a.ll, R * sizeof(double)));
  auto want = [&](const char* n) { return !only || strstr(n, only) != nullptr; };
  for (int rep = 0; rep < 2; ++rep) {  // two interleaved passes
    if (want("row_uniform")) run<1, 0>(a, ntiles, reps, "row_uniform");
    if (want("row_mixed")) run<1, 1>(a, ntiles, reps, "row_mixed");
    if (want("row_consolidated")) run<1, 2>(a, ntiles, reps, "row_consolidated");
    if (want("row_mixread")) run<1, 3>(a, ntiles, reps, "row_mixread");
    if (want("row_mixwrite")) run<1, 4>(a, ntiles, reps, "row_mixwrite");
    if (want("pk8f_uniform")) run_pk<8, 0>(a, ntiles, reps, "pk8f_uniform");
    if (want("pk8f_mixed")) run_pk<8, 1>(a, ntiles, reps, "pk8f_mixed");
    if (want("pk16f_uniform")) run_pk<16, 0>(a, ntiles, reps, "pk16f_uniform");
    if (want("pk16f_mixed")) run_pk<16, 1>(a, ntiles, reps, "pk16f_mixed");
    if (want("pk16l_uniform")) run_lds<16, 0>(a, ntiles, reps, "pk16l_uniform");
    if (want("pk16l_mixed")) run_lds<16, 1>(a, ntiles, reps, "pk16l_mixed");
    if (want("pk32l_uniform")) run_lds<32, 0>(a, ntiles, reps, "pk32l_uniform");
    if (want("pk32l_mixed")) run_lds<32, 1>(a, ntiles, reps, "pk32l_mixed");
  }
  return 0;
}
