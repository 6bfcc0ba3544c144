// PMC calibration for FETCH_SIZE / WRITE_SIZE on gfx950 with the access widths the dmt
// kernels use (8 B/lane fp64 and 4 B/lane fp32 coalesced loads and stores; MI355X_MICROARCH.md:
// "other access widths are uncalibrated: calibrate on a known byte count").
// Each kernel reads N elements and writes N elements once (1 GiB per array, past the 256 MiB
// Infinity Cache).  Measurement helper only: not part of libdmt.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/calib_stream scripts/calib_stream.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <class T>
__global__ __launch_bounds__(256) void k_stream(const T* __restrict__ in, T* __restrict__ out,
                                                size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[i] * (T)2;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const size_t bytes = (size_t)1 << 30;
  void *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  for (int rep = 0; rep < 3; ++rep) {
    k_stream<double><<<8192, 256>>>((const double*)a, (double*)b, bytes / 8);
    CK(hipGetLastError());
    k_stream<float><<<8192, 256>>>((const float*)a, (float*)b, bytes / 4);
    CK(hipGetLastError());
  }
  CK(hipDeviceSynchronize());
  std::printf("{\"bytes_read_per_launch\": %zu, \"bytes_written_per_launch\": %zu}\n", bytes, bytes);
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
