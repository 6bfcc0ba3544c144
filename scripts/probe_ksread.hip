// Checks the cross-lane fetches of the Kogge–Stone scans (ks_read_b32 in dmt_kernels.hip, copied
// here) against lane − o for every lane >= o and o = 1, 2, …, 32; prints OK or the first mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ int ks_read_b32(int v, int o, int lane) {
  if (o == 1) return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false);
  if (o == 32) return (int)__builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false)[0];
  if (o == 16) {
    const auto a = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    const unsigned r2 = __builtin_amdgcn_permlane32_swap(a[1], a[1], false, false)[0];
    return (int)(((lane >> 4) & 1) ? a[0] : r2);
  }
  return __builtin_amdgcn_ds_bpermute(4 * (lane - o), v);
}
__global__ void k(int* out) {
  const int lane = threadIdx.x;
  const int v = 1000 + lane;
#pragma unroll
  for (int i = 0, o = 1; o < 64; o <<= 1, ++i) out[i * 64 + lane] = ks_read_b32(v, o, lane);
}
int main() {
  int* d;
  if (hipMalloc(&d, 6 * 64 * sizeof(int)) != hipSuccess) return 2;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[6 * 64];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int bad = 0;
  for (int i = 0, o = 1; o < 64; o <<= 1, ++i)
    for (int l = o; l < 64; ++l)
      if (h[i * 64 + l] != 1000 + l - o) {
        if (bad++ < 8) std::printf("mismatch o=%d lane=%d got %d want %d\n", o, l, h[i * 64 + l] - 1000, l - o);
      }
  std::printf(bad ? "FAIL %d\n" : "OK\n", bad);
  (void)hipFree(d);
  return bad ? 1 : 0;
}
