/* dmt_callbench.c — the reference's unchanged caller loop issued as separate C-ABI calls, timed
 * in C: what a Julia caller's ccalls do for
 *   draw_proposal_path!(be); accept_reject_proposal_path!(be, i); fetch_ll(be); fetch_ll°(be)
 * (docs/src/tutorials/biblock/smoothing.md:40-44).  Measurement helper of bench.py (loaded with
 * ctypes), not part of the drop-in ABI; it calls nothing but include/dmt.h. */
#include <stdint.h>
#include <time.h>

#include "../../include/dmt.h"

int dmt_callbench_loop(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int64_t iter0,
                       int64_t n, int32_t global, double* out, double* seconds) {
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t it = iter0 + i;
    double ll = 0, llp = 0, ll2 = 0, llp2 = 0;
    int64_t na = 0, na2 = 0;
    if (dmt_draw_proposal(h, layout, b0, b1, 0, 0, DMT_RNG_AUTO, 0)) return 1;
    if (dmt_accept_reject(h, layout, b0, b1, 0, it, DMT_RNG_AUTO, 0)) return 2;
    /* fetch_ll(be) then fetch_ll°(be): two calls, as the reference's two functions */
    if ((global ? dmt_fetch_ll : dmt_fetch_ll_local)(h, layout, b0, b1, it, &ll, &llp, &na)) return 3;
    if ((global ? dmt_fetch_ll : dmt_fetch_ll_local)(h, layout, b0, b1, 0, &ll2, &llp2, &na2)) return 4;
    out[3 * i] = ll;
    out[3 * i + 1] = llp2;
    out[3 * i + 2] = (double)na;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  return 0;
}

/* The same loop, the duration of every iteration in lat[i] (seconds): the latency spread. */
int dmt_callbench_lat(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int64_t iter0,
                      int64_t n, double* lat) {
  for (int64_t i = 0; i < n; ++i) {
    struct timespec t0, t1;
    const int64_t it = iter0 + i;
    double ll = 0, llp = 0;
    int64_t na = 0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    if (dmt_draw_proposal(h, layout, b0, b1, 0, 0, DMT_RNG_AUTO, 0)) return 1;
    if (dmt_accept_reject(h, layout, b0, b1, 0, it, DMT_RNG_AUTO, 0)) return 2;
    if (dmt_fetch_ll_local(h, layout, b0, b1, it, &ll, &llp, &na)) return 3;
    if (dmt_fetch_ll_local(h, layout, b0, b1, 0, &ll, &llp, &na)) return 4;
    clock_gettime(CLOCK_MONOTONIC, &t1);
    lat[i] = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  }
  return 0;
}
