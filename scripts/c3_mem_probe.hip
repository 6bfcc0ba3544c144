// C3's memory pattern without its arithmetic: how fast can 1 024 waves (one per SIMD) stream the
// lane kernel's row layout — per step and lane, reads H (3 rows), F (2), u.W (1),
// writes X° (2), W° (1), fp64, 512-byte rows of 64 lanes, 1 000 steps per tile — as a function of
// how many K = 4-step chunks are loaded ahead (k_block ships two).  A grid-stride copy of the same
// bytes (6 read streams, 3 write streams, no per-wave order) is the pattern-free ceiling.
// Measurement helper only: not part of libdmt.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/c3_mem_probe scripts/c3_mem_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int kLanes = 64, kK = 4, kTiles = 1024, kSteps = 1000, kPad = 40;
constexpr int kRows = kSteps + kPad;  // spare rows keep the prefetch past the end in bounds

struct Chunk {
  double h[kK][3], f[kK][2], w[kK];
};

template <int A>
__global__ __launch_bounds__(64) void k_probe(const double* __restrict__ H,
                                              const double* __restrict__ F,
                                              const double* __restrict__ W, double* X, double* Wo) {
  const int64_t tile = blockIdx.x;
  const int lane = threadIdx.x;
  const double* Hb = H + tile * kRows * 3 * kLanes + lane;
  const double* Fb = F + tile * kRows * 2 * kLanes + lane;
  const double* Wb = W + tile * kRows * kLanes + lane;
  double* Xb = X + tile * kRows * 2 * kLanes + lane;
  double* Wob = Wo + tile * kRows * kLanes + lane;
  auto load = [&](int c0, Chunk& c) {
#pragma unroll
    for (int j = 0; j < kK; ++j) {
      const int64_t i = c0 + j;
#pragma unroll
      for (int e = 0; e < 3; ++e) c.h[j][e] = __builtin_nontemporal_load(&Hb[(i * 3 + e) * kLanes]);
#pragma unroll
      for (int e = 0; e < 2; ++e) c.f[j][e] = __builtin_nontemporal_load(&Fb[(i * 2 + e) * kLanes]);
      c.w[j] = __builtin_nontemporal_load(&Wb[(i + 1) * kLanes]);
    }
  };
  double x0 = 0.5, x1 = 0.25;
  auto run = [&](int c0, const Chunk& c) {
#pragma unroll
    for (int j = 0; j < kK; ++j) {
      const int64_t i = c0 + j;
      const double wo = 0.9 * c.w[j];
      x0 = fma(x0, c.h[j][0], c.f[j][0]);
      x1 = fma(x1, c.h[j][1], fma(c.h[j][2], wo, c.f[j][1]));
      __builtin_nontemporal_store(wo, &Wob[(i + 1) * kLanes]);
      __builtin_nontemporal_store(x0, &Xb[((i + 1) * 2) * kLanes]);
      __builtin_nontemporal_store(x1, &Xb[((i + 1) * 2 + 1) * kLanes]);
    }
  };
  Chunk ring[A + 1];
#pragma unroll
  for (int s = 0; s < A; ++s) load(s * kK, ring[s]);
  for (int c0 = 0; c0 < kSteps; c0 += (A + 1) * kK) {
#pragma unroll
    for (int s = 0; s <= A; ++s) {
      const int cc = c0 + s * kK;
      if (cc < kSteps) {
        load(cc + A * kK, ring[(s + A) % (A + 1)]);
        run(cc, ring[s]);
      }
    }
  }
}

// pattern-free ceiling: the same bytes as a flat grid-stride stream
__global__ __launch_bounds__(256) void k_flat(const double* __restrict__ H,
                                              const double* __restrict__ F,
                                              const double* __restrict__ W, double* X, double* Wo,
                                              size_t n) {  // n = rows of W (= points × lanes)
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const double h0 = __builtin_nontemporal_load(&H[3 * i]), h1 = __builtin_nontemporal_load(&H[3 * i + 1]),
                 h2 = __builtin_nontemporal_load(&H[3 * i + 2]);
    const double f0 = __builtin_nontemporal_load(&F[2 * i]), f1 = __builtin_nontemporal_load(&F[2 * i + 1]);
    const double w = __builtin_nontemporal_load(&W[i]);
    __builtin_nontemporal_store(0.9 * w, &Wo[i]);
    __builtin_nontemporal_store(h0 * f0, &X[2 * i]);
    __builtin_nontemporal_store(h1 * f1 + h2, &X[2 * i + 1]);
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <class L>
static float time_it(L launch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  std::vector<float> v;
  launch();
  for (int r = 0; r < reps; ++r) {
    (void)hipEventRecord(a);
    launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    v.push_back(ms * 1000.f);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const size_t n1 = (size_t)kTiles * kRows * kLanes;  // one plane
  double *H, *F, *W, *X, *Wo;
  CK(hipMalloc(&H, 3 * n1 * 8));
  CK(hipMalloc(&F, 2 * n1 * 8));
  CK(hipMalloc(&W, n1 * 8));
  CK(hipMalloc(&X, 2 * n1 * 8));
  CK(hipMalloc(&Wo, n1 * 8));
  CK(hipMemset(H, 0, 3 * n1 * 8));
  CK(hipMemset(F, 0, 2 * n1 * 8));
  CK(hipMemset(W, 0, n1 * 8));
  const double bytes = 9.0 * 8 * kTiles * kLanes * kSteps;  // 72 B per step and lane (§8(d))
  auto report = [&](const char* name, float us) {
    std::printf("{\"probe\": \"%s\", \"us\": %.1f, \"GBps\": %.0f, \"frac\": %.3f}\n", name, us,
                bytes / us / 1e3, bytes / us / 1e3 / 8000.0);
  };
  report("ahead1", time_it([&] { k_probe<1><<<kTiles, 64>>>(H, F, W, X, Wo); }, 7));
  report("ahead2", time_it([&] { k_probe<2><<<kTiles, 64>>>(H, F, W, X, Wo); }, 7));
  report("ahead3", time_it([&] { k_probe<3><<<kTiles, 64>>>(H, F, W, X, Wo); }, 7));
  report("ahead4", time_it([&] { k_probe<4><<<kTiles, 64>>>(H, F, W, X, Wo); }, 7));
  report("ahead6", time_it([&] { k_probe<6><<<kTiles, 64>>>(H, F, W, X, Wo); }, 7));
  const size_t nf = (size_t)kTiles * kSteps * kLanes;
  report("flat", time_it([&] { k_flat<<<8192, 256>>>(H, F, W, X, Wo, nf); }, 7));
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
