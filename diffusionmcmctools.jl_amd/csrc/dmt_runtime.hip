// dmt_runtime.hip — host side of libdmt: the C-ABI of include/dmt.h.
//
// The handle owns every device buffer of a SamplingEnsemble (u and u°) and of its block
// layouts.  Swaps are selector flips (one byte per segment per container kind), never
// copies: the reference swaps container *pointers* element by element
// (src/biblock.jl:148-199), and views from different block layouts alias the same
// SamplingPair vectors (src/block.jl:66-72), so selectors live per segment.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <cxxabi.h>
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dmt.h"
#include "dmt_internal.h"
#include "dmt_filter.h"

using namespace dmt;

namespace {

thread_local std::string g_err;

dmt_status fail(dmt_status code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_OK(expr)                                                                      \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      return fail(DMT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));        \
  } while (0)

template <class T>
hipError_t dalloc(T** p, int64_t n) {
  *p = nullptr;
  if (n <= 0) n = 1;
  return hipMalloc((void**)p, (size_t)n * sizeof(T));
}

struct Layout {
  int64_t nblocks = 0;
  int32_t MB = 0;
  int64_t hist_len = 0;
  std::vector<int64_t> blk_off;  // [R + 1]
  std::vector<int32_t> gfirst, glast, blk_rec;
  std::vector<uint8_t> term;
  bool single_seg = false;  // every block is one segment (the lane kernels' producer/consumer split)
  int32_t max_steps = 0;    // longest segment of any block (single-segment layouts)
  bool all_term = false;    // every block is terminal (no PPb law needed: law_ready)
  int64_t* d_blk_off = nullptr;
  BlkInfo* d_binfo = nullptr;
  int32_t* d_blk_rec = nullptr;
  int32_t* d_gfirst = nullptr;
  int32_t* d_glast = nullptr;
  uint8_t* d_term = nullptr;
  double* d_rho = nullptr;
  double* d_srho = nullptr;
  double* d_ll = nullptr;
  double* d_llp = nullptr;
  double* d_llh = nullptr;
  double* d_llph = nullptr;
  uint8_t* d_acch = nullptr;
  uint8_t* d_success = nullptr;
  uint8_t* d_acc = nullptr;
  uint8_t* d_crit = nullptr;    // [nblocks] set_proposal_law!'s critical-change flags
  uint32_t* d_ncrit = nullptr;  // their count
  void release() {
    void* ps[] = {d_blk_off, d_binfo, d_blk_rec, d_gfirst, d_glast, d_term,  d_rho,
                  d_srho,    d_ll,    d_llp,     d_llh,    d_llph,  d_acch,  d_success,
                  d_acc,     d_crit,  d_ncrit};
    for (void* p : ps)
      if (p) (void)hipFree(p);
  }
};

}  // namespace

struct dmt_ens {
  ModelKey key{};
  int d = 0, m = 0, hp = 0;
  size_t esz = 8;
  int device = 0;
  uint64_t seed = 0;
  uint32_t seg_base = 0;  // dmt_set_shard
  // DMT_RNG_AUTO stream counter (include/dmt.h): next key, the key of the last auto draw and
  // whether an auto accept may still take it
  uint64_t rng_ctr = 0, rng_last_draw = 0;
  bool rng_pending = false;
  bool spin_wait = true;  // wait for the stream by polling it (DMT_SPIN_WAIT=0: block in HIP)
  // Deferred draws (include/dmt.h): a device-RNG dmt_draw_proposal over a range the
  // register-resident kernel serves is not launched at once; the dmt_accept_reject that follows
  // on the same range runs draw + decision + fetch_ll tree as ONE launch of that kernel, whose
  // fetch_ll values (pinned h_run[0..2]) the next dmt_fetch_ll of the range returns without a
  // launch.  Any other call launches the deferred draw first (flush_deferred), so every call
  // sees exactly the state the launch-per-call order gives.  DMT_DEFER=0: off.
  struct {
    bool on = false;
    int32_t layout = 0;
    int64_t b0 = 0, b1 = 0;
    uint32_t iter = 0, salt = 0;
  } def;
  struct {
    bool on = false;
    int32_t layout = 0;
    int64_t b0 = 0, b1 = 0, mcmciter = 0;
    int64_t slot = -1;  // >= 0: the values are the service's iteration `slot` (its records)
    double vals[3];     // slot -1: h_run; -2: these (folded when the service stopped)
  } fused;
  bool defer = true;
  // The resident MCMC service (SvcArgs, dmt_kernels.hip): the fused draw + accept iterations
  // of consecutive stream keys and mcmciters on one range run in ONE launch of the resident
  // producer/consumer kernel, which keeps the blocks' state in registers and waits for the
  // host to post each iteration; fetch_ll reads the iteration's tree from pinned memory.  The
  // launch stops (the host asks, and waits) before any other call touches the stream, and
  // leaves on its own after DMT_SVC_IDLE_MS (2 ms) without a command.  DMT_SERVICE=0: off.
  struct {
    bool on = false;
    int32_t layout = 0;
    int64_t b0 = 0, b1 = 0, iter0 = 0, cap = 0;
    uint32_t key0 = 0, salt = 0;
    uint64_t posted = 0;
    uint64_t done = 0;    // iterations whose records the host has seen complete
    int64_t nwg = 0;      // workgroups of the launch (records per iteration)
    std::chrono::steady_clock::time_point t_last;
  } svc;
  bool service = true;
  double svc_idle_ms = 2.0;   // DMT_SVC_IDLE_MS: a launch idles this long for a post, then leaves
  int64_t svc_fit_nb = -1;    // the range size whose co-residency svc_fit holds
  bool svc_fit = false;
  // DMT_SVC_STATS; posts0 / relaunches0: the counts when the service was last enabled (the
  // self-disable rule looks at the counts since then)
  struct { uint64_t starts = 0, relaunches = 0, posts = 0, waits = 0, off = 0, posts0 = 0,
           relaunches0 = 0; } svc_stats;
  char* svc_host = nullptr;     // pinned: posted @0, stop @64 (separate lines)
  uint64_t* svc_rec = nullptr;  // pinned: [2][svc_rec_nwg][8] records (SvcArgs::rec)
  int64_t svc_rec_nwg = 0;
  uint64_t* d_svc_words = nullptr;  // device: go @0, quit @128 bytes
  uint64_t* d_svc_probe = nullptr;  // DMT_SVC_PROBE builds
  std::vector<double> svc_host_seen, svc_host_post, svc_host_code;  // DMT_SVC_PROBE: host stamps (µs)
  uint64_t wall_khz = 100000;   // device wall clock (hipDeviceAttributeWallClockRate)
  int grid_shared = 0;
  // path snapshots (dmt_snapshot_*): [slots][P][C] doubles in reference layout per kind
  int snap_mask = 0;
  int64_t snap_slots = 0;
  int64_t run_snap_every = 0;  // dmt_mcmc_run: snapshot u after every iteration k with k % every == 0
  int64_t run_snap_next = 0;   // ... into this slot next (ring over snap_slots)
  double* d_snap[2] = {nullptr, nullptr};
  std::vector<int64_t> snap_iter, snap_unit;
  int mapping = MAP_LANE;  // thread mapping of the recursion kernels
  int tw = kLanes;         // tile width of the device layout (64 lane-mapped, 1 wave-mapped)
  hipStream_t stream = nullptr;
  // structure
  int64_t R = 0, G = 0, P = 0, S = 0, ntiles = 0, Ptile = 0, Q0 = 0;
  std::vector<int64_t> rec_seg0;  // [R + 1]
  std::vector<int32_t> seg_rec, seg_q, seg_np;
  std::vector<int64_t> pt_off, st_off, tile_qoff;
  int64_t* d_pt_off = nullptr;
  int64_t* d_st_off = nullptr;
  int64_t* d_tile_qoff = nullptr;
  int32_t* d_seg_rec = nullptr;
  int32_t* d_seg_q = nullptr;
  int32_t* d_seg_np = nullptr;
  uint8_t* d_sel[4] = {nullptr, nullptr, nullptr, nullptr};  // X, W, PP, PPB
  std::vector<uint8_t> h_selPP, h_selPPB;                     // host mirrors (laws swap only by dmt_swap)
  void* d_X[3] = {nullptr, nullptr, nullptr};  // path buffers; [2]: MAP_LANE only (nbuf = 3)
  void* d_W[3] = {nullptr, nullptr, nullptr};
  int full_copy = 0;  // DMT_FULL_COPY
  int nbuf = 2;  // path buffers per container (DESIGN.md §2 "path buffers"; DMT_PATH_BUFS)
  int pk = 0;    // path planes in lane packets of pk points (fp32 MAP_LANE; DMT_PATH_PACKETS)
  void* d_t = nullptr;
  void* d_sdt = nullptr;  // shared grid: √dt per point in the working precision (lane kernels)
  bool have_t = false;
  void* d_H[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};  // [slot][kind]
  int H_shared[2] = {0, 0};                                     // per kind
  void* d_F[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  void* d_aux[2] = {nullptr, nullptr};  // [kind] per-point B̃(t_i), β̃(t_i) (dmt_upload_aux)
  double* d_law[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  bool have_law[2][2] = {{false, false}, {false, false}};  // [unit][kind] uploaded at least once
  // [unit][kind]: an uploaded law record asks for ã(t) from the table (DMT_LAW_AUXTD = 2) /
  // [kind]: the aux table holds ã columns (dmt_upload_aux_a with d·d + d + d(d+1)/2 columns)
  bool law_auxtd2[2][2] = {{false, false}, {false, false}};
  bool aux_has_a[2] = {false, false};
  // observation information for the device backward filter (dmt_upload_obs / dmt_set_obs)
  double* d_obsH = nullptr;  // [G][hp]
  double* d_obsF = nullptr;  // [G][d]
  double* d_obsc = nullptr;  // [G]
  double* d_obsv = nullptr;  // [G][d] artificial observations of P_last segments
  int* d_fail = nullptr;
  // chunked device filter (k_filter_*): chunk prefix per segment, segment law marks, scratch
  std::vector<int64_t> fchunk_off;  // [G + 1]
  int64_t* d_fchunk_off = nullptr;
  uint8_t* d_segsel = nullptr;      // [G]
  double* d_qbuf = nullptr;         // [kFiltNQ(d)][qbuf_cap]
  int64_t qbuf_cap = 0;
  double* d_tbuf = nullptr;         // [tbuf_cap][hp + d + 1] guiding term at chunk ends
  int64_t tbuf_cap = 0;
  double art_eps = 1e-11;    // artificial_noise (src/sampling_unit.jl:57)
  // staging
  double* d_stage = nullptr;
  int64_t stage_n = 0;
  double* d_Z = nullptr;
  int64_t Z_n = 0;
  double* d_red = nullptr;  // [3] reduction output, [3 * nranks] gather
  double* d_red_work = nullptr;
  double* d_red_lb = nullptr;
  int64_t red_work_n = 0;
  double* h_red = nullptr;  // pinned host copy of the 3 reduction results
  double* d_gather = nullptr;
  double* d_run = nullptr;         // dmt_mcmc_run: [n][3] per-iteration reductions
  double* h_run_dev = nullptr;     // h_run's device address (hipHostGetDevicePointer, once)
  double* h_run = nullptr;         // pinned host [run_cap][3]: one rank's results, written by
                                   // the kernels directly (no device-to-host copy)
  double* d_run_gather = nullptr;  // [n][nranks][3] (persistent path: [nranks][n][3])
  int64_t run_cap = 0;
  double* d_part = nullptr;  // k_mcmc_scan per-iteration block partials [n][3][nb]
  int64_t part_cap = 0;
  bool persist = true;       // dmt_mcmc_run of a linear drift in one launch (DMT_MCMC_PERSIST=0: off)
  bool resident = true;      // ... with register-resident block state when eligible (DMT_MCMC_RESIDENT=0: off)
  // ... also with a time-dependent aux table, through k_mcmc_scan<…, TD> (DMT_MCMC_SCAN_TD=1:
  // opt-in; off by default since the round-4/5 fault of that kernel was not root-caused,
  // DESIGN.md §7 — the per-iteration kernels run such ensembles)
  bool persist_td = false;
  // timing events recorded on the stream around the timed launch (default), or attached to its
  // dispatch packet (DMT_DISPATCH_EVENTS=1: hipExtLaunchKernel with events — the kernel's own
  // execution interval, but ≈ 10 µs more host time in the launch call, profiles/r02zo)
  bool dispatch_events = false;
  // flags of the timing events (DMT_EVENT_FLAGS): they only measure, so a system-scope fence
  // (cache writeback and invalidation when the event is recorded) buys nothing
  unsigned event_flags = hipEventDefault;
  int resident_pc = 1;       // ... split over a consumer and this many producer waves per block
  bool pc_bpw1 = false;      // ... one block per workgroup (DMT_PC_BPW=1)
                             // (DMT_MCMC_PC=0: one wave; 1 or 2 producers)
  int lane_split = -1;       // MAP_LANE draws on producer/consumer waves: 1 on, 0 off, -1 auto
  int lane_pair = -1;        // MAP_LANE device-RNG draws on lane pairs: 1 on, 0 off, -1 auto
                             // (when the draw has fewer waves than the device has SIMDs)
  int64_t n_simd = 1024;
  int repair_div = 1;        // MAP_LANE path consolidation threshold (DMT_REPAIR_DIV; path_plan)
  int repair_min = 1;        // … and minimum minority (DMT_REPAIR_MIN)
  bool scan_resident = true; // one-shot OU draws on k_block_resident when eligible (DMT_SCAN_RESIDENT=0: off)
  std::vector<std::unique_ptr<Layout>> layouts;  // layouts[0] = internal "unit" layout
  // timing
  uint32_t timing = 0;  // bit k: time kernel class k (dmt_set_timing)
  struct PendingTime {
    hipEvent_t first, second;
    int64_t units;  // kernel invocations the interval stands for (k_mcmc_scan: iterations)
  };
  std::vector<PendingTime> pending[DMT_K_COUNT];
  double t_ms[DMT_K_COUNT] = {0, 0, 0, 0, 0};
  int64_t t_cnt[DMT_K_COUNT] = {0, 0, 0, 0, 0};
  std::vector<hipEvent_t> free_events;
  // comm
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  int64_t bytes = 0;
};

namespace {

hipError_t stream_wait(dmt_ens* h);

template <class T>
dmt_status ens_alloc(dmt_ens* h, T** p, int64_t n) {
  hipError_t e = dalloc(p, n);
  if (e != hipSuccess)
    return fail(DMT_ERR_OOM, std::string("hipMalloc of ") + std::to_string(n * sizeof(T)) +
                                 " bytes failed: " + hipGetErrorString(e));
  h->bytes += std::max<int64_t>(n, 1) * (int64_t)sizeof(T);
  return DMT_OK;
}
dmt_status ens_alloc_bytes(dmt_ens* h, void** p, int64_t nbytes) {
  return ens_alloc(h, (uint8_t**)p, nbytes);
}

#define DMT_TRY(expr)            \
  do {                           \
    dmt_status _s = (expr);      \
    if (_s != DMT_OK) return _s; \
  } while (0)

hipEvent_t get_event(dmt_ens* h) {
  if (!h->free_events.empty()) {
    hipEvent_t e = h->free_events.back();
    h->free_events.pop_back();
    return e;
  }
  hipEvent_t e;
  (void)hipEventCreateWithFlags(&e, h->event_flags);
  return e;
}

void drain_timing(dmt_ens* h) {
  for (int k = 0; k < DMT_K_COUNT; ++k) {
    for (auto& pr : h->pending[k]) {
      float ms = 0.f;
      if (hipEventSynchronize(pr.second) == hipSuccess &&
          hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
        h->t_ms[k] += ms;
        h->t_cnt[k] += pr.units;
      }
      h->free_events.push_back(pr.first);
      h->free_events.push_back(pr.second);
    }
    h->pending[k].clear();
  }
}

// Times the kernel launched inside the scope.  dispatch = true (DMT_DISPATCH_EVENTS=1): the
// events ride on that kernel's dispatch packet (the launcher uses hipExtLaunchKernel; the time is
// the kernel's execution, as rocprofv3 reports it); otherwise (default) they are recorded on the
// stream around it: the interval also holds the dispatch itself (≈ 2 µs on a 138 µs C2 launch
// against rocprofv3's 138.2), and the launch call stays ≈ 10 µs cheaper on the host.
struct TimedScope {
  dmt_ens* h;
  int k;
  bool dispatch;
  int64_t units;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  TimedScope(dmt_ens* h_, int k_, bool dispatch_ = true, int64_t units_ = 1)
      : h(h_), k(k_), dispatch(dispatch_ && h_->dispatch_events), units(units_) {
    if (h->timing >> k & 1u) {
      e0 = get_event(h);
      e1 = get_event(h);
      if (dispatch) {
        g_dispatch_events.start = e0;
        g_dispatch_events.stop = e1;
      } else {
        (void)hipEventRecord(e0, h->stream);
      }
    }
  }
  ~TimedScope() {
    if (e0) {
      if (dispatch && g_dispatch_events.start) {  // no kernel consumed them (empty range)
        g_dispatch_events = DispatchEvents{};
        (void)hipEventRecord(e0, h->stream);
        (void)hipEventRecord(e1, h->stream);
      } else if (!dispatch) {
        (void)hipEventRecord(e1, h->stream);
      }
      h->pending[k].push_back({e0, e1, units});
      if (h->pending[k].size() > 512) drain_timing(h);
    }
  }
};

dmt_status ensure_stage(dmt_ens* h, int64_t n) {
  if (n <= h->stage_n) return DMT_OK;
  if (h->d_stage) {
    (void)hipFree(h->d_stage);
    h->bytes -= h->stage_n * 8;
  }
  h->d_stage = nullptr;
  h->stage_n = 0;
  DMT_TRY(ens_alloc(h, &h->d_stage, n));
  h->stage_n = n;
  return DMT_OK;
}

dmt_status ensure_Z(dmt_ens* h, int64_t n) {
  if (n <= h->Z_n) return DMT_OK;
  if (h->d_Z) {
    (void)hipFree(h->d_Z);
    h->bytes -= h->Z_n * 8;
  }
  h->d_Z = nullptr;
  h->Z_n = 0;
  DMT_TRY(ens_alloc(h, &h->d_Z, n));
  h->Z_n = n;
  return DMT_OK;
}

int64_t plane_elems(const dmt_ens* h, int C) { return h->Ptile * C * h->tw; }

dmt_status check_h(dmt_ens* h) {
  if (!h) return fail(DMT_ERR_INVALID, "null handle");
  if (hipSetDevice(h->device) != hipSuccess) return fail(DMT_ERR_HIP, "hipSetDevice failed");
  return DMT_OK;
}

// Wait for everything queued on the handle's stream by polling it from this thread
// (DMT_SPIN_WAIT=0: block in hipStreamSynchronize).  On the driver's 20-iteration C2 run the two
// measured within noise of each other (profiles/r02j); polling keeps the wake-up off the
// scheduler for short calls.
hipError_t stream_wait(dmt_ens* h) {
  if (!h->spin_wait) return hipStreamSynchronize(h->stream);
  // poll for at most kSpinUs, then block in HIP: short waits (the hot path's per-call results)
  // stay off the scheduler, long ones (filters, snapshot writes, destroy) do not burn a core
  constexpr double kSpinUs = 200.0;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(h->stream);
    if (e != hipErrorNotReady) return e;
    if (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() >
        kSpinUs)
      return hipStreamSynchronize(h->stream);
  }
}

// ---- stream keys (include/dmt.h, "device random streams")
struct RngKey {
  uint32_t iter, salt;
};
RngKey auto_key(uint64_t k) {
  return {(uint32_t)k, DMT_SALT_LIMIT + (uint32_t)((k >> 32) & (DMT_SALT_LIMIT - 1))};
}
dmt_status check_salt(uint32_t salt) {
  if (salt != DMT_RNG_AUTO && salt >= DMT_SALT_LIMIT)
    return fail(DMT_ERR_INVALID, "salt must be < DMT_SALT_LIMIT (larger keys belong to DMT_RNG_AUTO)");
  return DMT_OK;
}
// key of a draw call (draw_proposal: arm = true, the next auto accept reuses it)
dmt_status draw_key(dmt_ens* h, int64_t iter, uint32_t salt, bool arm, RngKey* k) {
  DMT_TRY(check_salt(salt));
  if (salt != DMT_RNG_AUTO) {
    *k = {(uint32_t)iter, salt};
    return DMT_OK;
  }
  const uint64_t c = h->rng_ctr++;
  h->rng_last_draw = c;
  h->rng_pending = arm;
  *k = auto_key(c);
  return DMT_OK;
}
dmt_status accept_key(dmt_ens* h, int64_t mcmciter, uint32_t salt, RngKey* k) {
  DMT_TRY(check_salt(salt));
  if (salt != DMT_RNG_AUTO) {
    *k = {(uint32_t)mcmciter, salt};
    return DMT_OK;
  }
  const uint64_t c = h->rng_pending ? h->rng_last_draw : h->rng_ctr++;
  h->rng_pending = false;
  *k = auto_key(c);
  return DMT_OK;
}

dmt_status get_layout(dmt_ens* h, int32_t id, Layout** L) {
  if (id < 0 || id >= (int32_t)h->layouts.size() || !h->layouts[id])
    return fail(DMT_ERR_INVALID, "bad layout id " + std::to_string(id));
  *L = h->layouts[id].get();
  return DMT_OK;
}

dmt_status check_range(const Layout* L, int64_t b0, int64_t b1) {
  if (b0 < 0 || b1 > L->nblocks || b0 > b1)
    return fail(DMT_ERR_INVALID, "block range [" + std::to_string(b0) + "," + std::to_string(b1) +
                                     ") outside layout of " + std::to_string(L->nblocks) + " blocks");
  return DMT_OK;
}

// recording of a flat block id (largest r with blk_off[r] <= blk)
int64_t rec_of_block(const Layout* L, int64_t blk) {
  auto it = std::upper_bound(L->blk_off.begin(), L->blk_off.end(), blk);
  return (int64_t)(it - L->blk_off.begin()) - 1;
}

dmt_status law_ready(dmt_ens* h, int unit_needed_flip, const Layout* L, int64_t b0, int64_t b1) {
  // the PP law is always needed; PPB only for non-terminal blocks
  bool need_ppb = false;  // (per call: a host loop over the range unless the layout says)
  for (int64_t b = b0; b < b1 && !need_ppb && !L->all_term; ++b) need_ppb = !L->term[b];
  if (!h->have_t) return fail(DMT_ERR_STATE, "time grid not uploaded (dmt_upload_grid)");
  if (!h->d_law[0][0] || !h->d_law[1][0] || !h->d_H[0][0] || !h->d_F[0][0])
    return fail(DMT_ERR_STATE, "PP law not uploaded (dmt_upload_law)");
  if (need_ppb && (!h->d_law[0][1] || !h->d_H[0][1] || !h->d_F[0][1]))
    return fail(DMT_ERR_STATE, "PPb (blocking) law not uploaded but a non-terminal block is used");
  for (int k = 0; k < 2; ++k)
    if ((h->law_auxtd2[0][k] || h->law_auxtd2[1][k]) && !(h->d_aux[k] && h->aux_has_a[k]))
      return fail(DMT_ERR_STATE, "a law record with DMT_LAW_AUXTD = 2 needs an aux table with ã "
                                 "columns (dmt_upload_aux_a)");
  (void)unit_needed_flip;
  return DMT_OK;
}

template <class T>
void fill_common(dmt_ens* h, const Layout* L, BlockArgs<T>& a) {
  a.R = h->R;
  a.tile_qoff = h->d_tile_qoff;
  a.seg_q = h->d_seg_q;
  a.seg_np = h->d_seg_np;
  a.st_off = h->d_st_off;
  a.selX = h->d_sel[0];
  a.selW = h->d_sel[1];
  a.selPP = h->d_sel[2];
  a.selPPB = h->d_sel[3];
  a.nbuf = h->nbuf;
  a.pk = h->pk;
  a.full_copy = h->full_copy;
  for (int s = 0; s < 3; ++s) {
    a.X[s] = (T*)h->d_X[s];
    a.W[s] = (T*)h->d_W[s];
  }
  for (int s = 0; s < 2; ++s) {
    for (int k = 0; k < 2; ++k) {
      a.H[s][k] = (const T*)h->d_H[s][k];
      a.H_shared[s][k] = h->H_shared[k];
      a.F[s][k] = (const T*)h->d_F[s][k];
      a.law[s][k] = h->d_law[s][k];
    }
  }
  a.t = (const T*)h->d_t;
  a.sdt = h->grid_shared ? (const T*)h->d_sdt : nullptr;
  a.t_shared = h->grid_shared;
  a.aux[0] = (const T*)h->d_aux[0];
  a.aux[1] = (const T*)h->d_aux[1];
  a.aux_n = plane_elems(h, (int)(h->d * h->d + h->d + h->hp));
  a.blk_off = L->d_blk_off;
  a.blk_rec = L->d_blk_rec;
  a.binfo = L->d_binfo;
  a.gfirst = L->d_gfirst;
  a.glast = L->d_glast;
  a.term = L->d_term;
  a.rho = L->d_rho;
  a.srho = L->d_srho;
  a.MB = L->MB;
  a.seed = h->seed;
  a.seg_base = h->seg_base;
  a.Z = nullptr;
  a.success = nullptr;
  a.repair_div = h->repair_div;
  a.repair_min = h->repair_min;
  a.lane_split = 0;
  a.lane_pair = 0;
  a.resident1 = 0;
}

// A time-dependent auxiliary law's table is present: linear drifts then run on the scan
// kernels only (the register-resident ones take the law's own B̃, β̃)
static bool has_aux_table(const dmt_ens* h) { return h->d_aux[0] || h->d_aux[1]; }

dmt_status run_block_kernel(dmt_ens* h, const Layout* L, int mode, int kind_timer, int64_t b0,
                            int64_t b1, int law_flip, int xs, int xd, int ws, int wd,
                            const double* dZ, int64_t iter, uint32_t salt, double* ll_out,
                            uint8_t* success, int op /* 0 draw/solve, 1 loglikhd, 2 invsolve */,
                            int ll_skip = 0 /* MODE_RECOMPUTE: recompute_path!(…; skip) */) {
  if (b1 <= b0) return DMT_OK;
  const int64_t r0 = rec_of_block(L, b0), r1 = rec_of_block(L, b1 - 1);
  const int64_t tile0 = r0 / kLanes, tile1 = r1 / kLanes + 1;
  // MAP_LANE: one wave per (recording tile, block index); MAP_WAVE: one wave per block
  const int64_t nwaves = h->mapping == MAP_WAVE ? (b1 - b0) : (tile1 - tile0) * (int64_t)L->MB;
  TimedScope ts(h, kind_timer);
  hipError_t e;
  auto fill = [&](auto& a) {
    fill_common(h, L, a);
    a.tile0 = tile0;
    a.tile1 = tile1;
    a.b0 = b0;
    a.b1 = b1;
    a.law_flip = law_flip;
    a.xs_flip = xs;
    a.xd_flip = xd;
    a.ws_flip = ws;
    a.wd_flip = wd;
    a.Z = dZ;
    a.iter = (uint32_t)iter;
    a.salt = salt;
    a.ll_out = ll_out;
    a.success = success;
    a.ll_skip = ll_skip;
    a.resident1 = h->scan_resident && h->key.model == DMT_MODEL_OU && h->key.d <= 2 &&
                  !has_aux_table(h) && L->single_seg && L->max_steps <= kResidentMaxSteps;
    // auto: fp64 only — with fp32's four normals per Philox block the single wave is faster
    // (C5: 1773 vs 1934 µs per draw, profiles/r02m)
    // lane pairs (k_block_pair): on request only — bit-identical, but measured no faster on C5
    // (1 862 / 1 925 vs 1 829 µs per draw) and slower on C3 (1 821 vs 1 301 µs):
    // profiles/r03d, DESIGN.md §6
    // lane pairs: on request only (DMT_LANE_PAIR=1) — bit-identical, but no faster on the row
    // layout (profiles/r03d) and slower on the packet layout: C5 1 753–1 789 vs 1 455–1 463 µs
    // per draw with register-staged packets (profiles/r04g)
    a.lane_pair = h->lane_pair == 1;
    // the packet layout's split (k_block_ps_pk; fp32 lane packets): C5 1 343-1 355 vs
    // 1 445-1 461 µs per draw (profiles/r05j)
    a.lane_split = !a.lane_pair && L->single_seg &&
                   (h->lane_split == 1 || (h->lane_split < 0 && nwaves < h->n_simd &&
                                           (h->key.precision == DMT_F64 || h->pk)));
  };
  if (h->key.precision == DMT_F64) {
    BlockArgs<double> a{};
    fill(a);
    e = op == 1 ? launch_pathll_kernel(h->key, h->mapping, &a, nwaves, h->stream)
        : op == 2 ? launch_invsolve_kernel(h->key, h->mapping, &a, nwaves, h->stream)
                  : launch_block_kernel(h->key, h->mapping, mode, &a, nwaves, h->stream);
  } else {
    BlockArgs<float> a{};
    fill(a);
    e = op == 1 ? launch_pathll_kernel(h->key, h->mapping, &a, nwaves, h->stream)
        : op == 2 ? launch_invsolve_kernel(h->key, h->mapping, &a, nwaves, h->stream)
                  : launch_block_kernel(h->key, h->mapping, mode, &a, nwaves, h->stream);
  }
  if (e != hipSuccess) return fail(DMT_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
  return DMT_OK;
}

// ---- the resident MCMC service
constexpr int64_t kSvcCap = 4096;       // iterations per service launch
dmt_status svc_relaunch(dmt_ens* h, uint64_t base);  // svc_launch (below)
inline volatile uint64_t* svc_posted(dmt_ens* h) { return (volatile uint64_t*)(h->svc_host); }
inline volatile uint32_t* svc_stopw(dmt_ens* h) { return (volatile uint32_t*)(h->svc_host + 64); }

// Iteration `slot`'s records are all in: every workgroup's three 16-byte (sum, check) records
// agree for tag slot + 1 (check = sum bits ^ svc_mix(slot + 1), dmt_internal.h).  The two words
// are read separately, and nothing promises that the device's 16-byte store reaches host memory
// as one piece; a record read half old, half new fails the check and is read again.  A check
// reads the value word last, so the value that passed is the one svc_fold reads (records of
// `slot` are not rewritten before the host has posted slot + 2).
bool svc_slot_ready(const dmt_ens* h, uint64_t slot) {
  const volatile uint64_t* r = h->svc_rec + (slot & 1) * h->svc.nwg * 8;
  const uint64_t mix = svc_mix(slot + 1);
  for (int64_t w = h->svc.nwg - 1; w >= 0; --w)
    for (int c = 0; c < 3; ++c) {
      const uint64_t chk = r[8 * w + 2 * c + 1];
      std::atomic_thread_fence(std::memory_order_acquire);
      if (chk != (r[8 * w + 2 * c] ^ mix)) return false;
    }
  return true;
}

// fetch_ll, fetch_ll° and the accepted count of iteration `slot` from its records: the
// workgroups' 4-block sums folded by the canonical adjacent-pair tree (padded with zeros to a
// power of two >= 64 leaves, + 0.0 on the two sums — the tree of dmt_fetch_ll)
void svc_fold(const dmt_ens* h, uint64_t slot, double* out3) {
  const volatile uint64_t* r = h->svc_rec + (slot & 1) * h->svc.nwg * 8;
  const int64_t n = h->svc.nwg;
  int64_t P = 64;
  while (P < n) P <<= 1;
  std::vector<double> v(P);
  for (int c = 0; c < 3; ++c) {
    for (int64_t w = 0; w < P; ++w) {
      uint64_t bits = w < n ? r[8 * w + 2 * c] : 0;
      double x;
      std::memcpy(&x, &bits, 8);
      v[w] = w < n ? x : 0.0;
    }
    for (int64_t m = P; m > 1; m >>= 1)
      for (int64_t k = 0; k < m / 2; ++k) v[k] = v[2 * k] + v[2 * k + 1];
    out3[c] = c == 2 ? v[0] : v[0] + 0.0;
  }
}

// A service whose launches keep leaving idle before their iteration is posted is turned off for
// the handle; the fused iterations then run one launch each.  Two causes, both counted: other
// work holding the CUs the grid needs (the non-resident workgroups start only after workgroup
// 0's idle exit: found in svc_wait_done), and a host that is away longer than half the idle
// window between its iterations (relaunched at the post) — then every iteration pays a launch
// anyway and the resident launch buys nothing.  The rule looks at the posts and relaunches
// since the service was last enabled (dmt_set_service), so re-enabling it starts afresh.
void svc_check_degraded(dmt_ens* h) {
  const auto& st = h->svc_stats;
  const uint64_t posts = st.posts - st.posts0, rel = st.relaunches - st.relaunches0;
  if (h->service && posts >= 16 && 4 * rel > posts) {
    h->service = false;
    h->svc_stats.off = 1;
  }
}

// Wait until the service has finished n iterations (spin: the caller waits for this very
// result).  A launch that left idle before an iteration was posted to it (the host was away
// longer than the idle window) is launched again from the first iteration it did not run; a
// launch that failed is an error, never a hang.
dmt_status svc_wait_done(dmt_ens* h, uint64_t n) {
  auto& v = h->svc;
  auto t0 = std::chrono::steady_clock::now();
  bool waited = false;
  while (v.done < n) {
    if (svc_slot_ready(h, v.done)) {
      ++v.done;
      continue;
    }
    waited = true;
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (us > 100.0) {
      const hipError_t e = hipStreamQuery(h->stream);
      if (e == hipSuccess) {  // the launch has ended: everything it wrote is visible
        if (svc_slot_ready(h, v.done)) continue;
        ++h->svc_stats.relaunches;
        svc_check_degraded(h);
        DMT_TRY(svc_relaunch(h, v.done));
        t0 = std::chrono::steady_clock::now();
      } else if (e != hipErrorNotReady) {
        return fail(DMT_ERR_HIP, std::string("resident service: ") + hipGetErrorString(e));
      } else if (us > 10e6) {
        return fail(DMT_ERR_HIP, "resident service: no result in 10 s");
      }
    }
  }
  if (waited) ++h->svc_stats.waits;
  return DMT_OK;
}

// Stop a running service: every posted iteration finished, then the stop word, then the launch
// drains (its waves leave at their next gate); the words are re-armed for the next launch.  The
// values of a fused iteration of the service are folded first (they stay fetch_ll's answer).
dmt_status svc_stop(dmt_ens* h) {
  if (!h->svc.on) return DMT_OK;
  h->svc.on = false;
  dmt_status st = svc_wait_done(h, h->svc.posted);
  if (st == DMT_OK && h->fused.on && h->fused.slot >= 0) {
    svc_fold(h, (uint64_t)h->fused.slot, h->fused.vals);
    h->fused.slot = -2;
  }
  __atomic_store_n(svc_stopw(h), 1u, __ATOMIC_RELEASE);
  const hipError_t e = stream_wait(h);
  __atomic_store_n(svc_stopw(h), 0u, __ATOMIC_RELEASE);
  __atomic_store_n(svc_posted(h), (uint64_t)0, __ATOMIC_RELEASE);
  h->svc.posted = 0;
  h->svc.done = 0;
  if (st != DMT_OK) return st;
  if (e != hipSuccess) return fail(DMT_ERR_HIP, std::string("resident service: ") + hipGetErrorString(e));
  return DMT_OK;
}

// Launch a deferred draw (if any): the kernel launch dmt_draw_proposal would have made, with
// the stream key it took.  The fused results stay valid (the draw is ordered after them).
dmt_status flush_deferred(dmt_ens* h) {
  if (!h->def.on) return DMT_OK;
  DMT_TRY(svc_stop(h));
  h->def.on = false;
  Layout* L;
  DMT_TRY(get_layout(h, h->def.layout, &L));
  return run_block_kernel(h, L, MODE_PCN, DMT_K_DRAW, h->def.b0, h->def.b1, 0, 0, 1, 0, 1,
                          nullptr, h->def.iter, h->def.salt, L->d_llp, L->d_success, false);
}

// Entry of every call that reads or changes state: the deferred draw is launched first and the
// fused fetch_ll values are dropped.
dmt_status enter(dmt_ens* h) {
  DMT_TRY(check_h(h));
  DMT_TRY(svc_stop(h));
  DMT_TRY(flush_deferred(h));
  h->fused.on = false;
  return DMT_OK;
}

// The register-resident MCMC kernel serves the range: single-segment blocks of <= 512 steps of
// a linear drift with d <= 2 (dmt_mcmc_run's own condition, layout-wide)
bool resident_range(const dmt_ens* h, const Layout* L) {
  return h->persist && h->resident && h->key.model == DMT_MODEL_OU && h->key.d <= 2 &&
         !has_aux_table(h) && L->single_seg && L->max_steps <= kResidentMaxSteps;
}

dmt_status upload_Z(dmt_ens* h, const double* Z, const double** dZ) {
  *dZ = nullptr;
  if (!Z) return DMT_OK;
  const int64_t n = h->S * h->m;
  DMT_TRY(ensure_Z(h, n + 2 * kPadPoints * h->m));  // chunk prefetch may read past the end
  HIP_OK(hipMemcpyAsync(h->d_Z, Z, (size_t)n * 8, hipMemcpyHostToDevice, h->stream));
  *dZ = h->d_Z;
  return DMT_OK;
}

dmt_status build_layout(dmt_ens* h, const int32_t* n_blocks, const int32_t* seg_first,
                        const int32_t* seg_last, const uint8_t* last, const double* rho,
                        int64_t hist_len, int32_t* id) {
  auto L = std::make_unique<Layout>();
  L->blk_off.assign(h->R + 1, 0);
  for (int64_t r = 0; r < h->R; ++r) {
    if (n_blocks[r] < 0) return fail(DMT_ERR_INVALID, "negative block count");
    L->blk_off[r + 1] = L->blk_off[r] + n_blocks[r];
    L->MB = std::max<int32_t>(L->MB, n_blocks[r]);
  }
  L->nblocks = L->blk_off[h->R];
  L->hist_len = hist_len < 0 ? 0 : hist_len;
  L->gfirst.resize(L->nblocks);
  L->glast.resize(L->nblocks);
  L->blk_rec.resize(L->nblocks);
  L->term.resize(L->nblocks);
  std::vector<double> srho(L->nblocks), rr(L->nblocks);
  for (int64_t r = 0; r < h->R; ++r) {
    const int64_t nseg = h->rec_seg0[r + 1] - h->rec_seg0[r];
    for (int64_t b = L->blk_off[r]; b < L->blk_off[r + 1]; ++b) {
      if (seg_first[b] < 0 || seg_last[b] >= nseg || seg_first[b] > seg_last[b])
        return fail(DMT_ERR_INVALID, "block " + std::to_string(b) + " has an invalid segment range");
      if (!last[b] && seg_first[b] == seg_last[b])
        return fail(DMT_ERR_INVALID, "non-terminal block " + std::to_string(b) +
                                         " needs >= 2 segments (reference indexes PP[1], src/block.jl:66,178)");
      L->gfirst[b] = (int32_t)(h->rec_seg0[r] + seg_first[b]);
      L->glast[b] = (int32_t)(h->rec_seg0[r] + seg_last[b]);
      L->term[b] = last[b] ? 1 : 0;
      L->blk_rec[b] = (int32_t)r;
      rr[b] = rho[b];
      if (!(rho[b] >= 0.0 && rho[b] <= 1.0)) return fail(DMT_ERR_INVALID, "rho outside [0,1]");
      srho[b] = std::sqrt(1.0 - rho[b] * rho[b]);
    }
  }
  L->single_seg = true;
  for (int64_t b = 0; b < L->nblocks && L->single_seg; ++b) L->single_seg = L->gfirst[b] == L->glast[b];
  L->max_steps = 0;
  for (int64_t b = 0; b < L->nblocks && L->single_seg; ++b)
    L->max_steps = std::max(L->max_steps, h->seg_np[L->gfirst[b]] - 1);
  L->all_term = true;
  for (int64_t b = 0; b < L->nblocks && L->all_term; ++b) L->all_term = L->term[b] != 0;
  const int64_t nb = L->nblocks;
  DMT_TRY(ens_alloc(h, &L->d_blk_off, h->R + 1));
  DMT_TRY(ens_alloc(h, &L->d_gfirst, nb));
  DMT_TRY(ens_alloc(h, &L->d_blk_rec, nb));
  DMT_TRY(ens_alloc_bytes(h, (void**)&L->d_binfo, std::max<int64_t>(nb, 1) * (int64_t)sizeof(BlkInfo)));
  DMT_TRY(ens_alloc(h, &L->d_glast, nb));
  DMT_TRY(ens_alloc(h, &L->d_term, nb));
  DMT_TRY(ens_alloc(h, &L->d_rho, nb));
  DMT_TRY(ens_alloc(h, &L->d_srho, nb));
  DMT_TRY(ens_alloc(h, &L->d_ll, nb));
  DMT_TRY(ens_alloc(h, &L->d_llp, nb));
  DMT_TRY(ens_alloc(h, &L->d_success, nb));
  DMT_TRY(ens_alloc(h, &L->d_crit, nb));
  DMT_TRY(ens_alloc(h, &L->d_ncrit, 1));
  DMT_TRY(ens_alloc(h, &L->d_acc, nb));
  if (L->hist_len > 0) {
    DMT_TRY(ens_alloc(h, &L->d_llh, L->hist_len * nb));
    DMT_TRY(ens_alloc(h, &L->d_llph, L->hist_len * nb));
    DMT_TRY(ens_alloc(h, &L->d_acch, L->hist_len * nb));
    HIP_OK(hipMemsetAsync(L->d_llh, 0, (size_t)(L->hist_len * nb) * 8, h->stream));
    HIP_OK(hipMemsetAsync(L->d_llph, 0, (size_t)(L->hist_len * nb) * 8, h->stream));
    HIP_OK(hipMemsetAsync(L->d_acch, 0, (size_t)(L->hist_len * nb), h->stream));
  }
  HIP_OK(hipMemcpy(L->d_blk_off, L->blk_off.data(), (h->R + 1) * 8, hipMemcpyHostToDevice));
  if (nb > 0) {
    HIP_OK(hipMemcpy(L->d_gfirst, L->gfirst.data(), nb * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(L->d_blk_rec, L->blk_rec.data(), nb * 4, hipMemcpyHostToDevice));
    std::vector<BlkInfo> bi(nb);
    for (int64_t b = 0; b < nb; ++b) {
      const int64_t r = L->blk_rec[b];
      bi[b].tq = h->tile_qoff[r / h->tw];
      bi[b].g0 = L->gfirst[b];
      bi[b].g1 = L->glast[b];
      int32_t kt = 0;
      for (int32_t g = L->gfirst[b]; g <= L->glast[b]; ++g) kt += (h->seg_np[g] - 1 + 63) / 64;
      bi[b].ktot = kt;
      bi[b].term = L->term[b];
      bi[b].np0 = h->seg_np[L->gfirst[b]];
      bi[b].q0 = h->seg_q[L->gfirst[b]];
      bi[b].kfirst = (bi[b].np0 - 1 + 63) / 64;
      bi[b].pad_ = 0;
      bi[b].rho = rr[b];
      bi[b].srho = srho[b];
    }
    HIP_OK(hipMemcpy(L->d_binfo, bi.data(), nb * sizeof(BlkInfo), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(L->d_glast, L->glast.data(), nb * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(L->d_term, L->term.data(), nb, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(L->d_rho, rr.data(), nb * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(L->d_srho, srho.data(), nb * 8, hipMemcpyHostToDevice));
    std::vector<double> ninf(nb, -INFINITY);  // ll = -Inf initially (src/block.jl:75)
    HIP_OK(hipMemcpy(L->d_ll, ninf.data(), nb * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(L->d_llp, ninf.data(), nb * 8, hipMemcpyHostToDevice));
  }
  h->layouts.push_back(std::move(L));
  *id = (int32_t)h->layouts.size() - 1;
  return DMT_OK;
}

inline int dmt_packed(int d, int a, int b) {
  if (a > b) std::swap(a, b);
  return a * d - (a * (a - 1)) / 2 + (b - a);
}

bool supported(const dmt_model* m) {
  if (m->precision != DMT_F64 && m->precision != DMT_F32) return false;
  switch (m->model) {
    case DMT_MODEL_OU:
      return (m->d == 1 && m->m == 1) || (m->d == 2 && m->m == 2) || (m->d == 2 && m->m == 1) ||
             (m->d == 3 && m->m == 3);
    case DMT_MODEL_FHN: return m->d == 2 && m->m == 1;
    case DMT_MODEL_LORENZ: return m->d == 3 && m->m == 3;
  }
  return false;
}

// ------------------------------------------------------------ backward filter
// (dmt_filter.h: shared with the device kernel k_backward_filter)

}  // namespace

// =====================================================================================
extern "C" {

const char* dmt_last_error(void) { return g_err.c_str(); }
const char* dmt_version(void) { return "dmt-mi355x 0.1.0 (gfx950)"; }

dmt_status dmt_create(dmt_ens** out, const dmt_model* model, const dmt_structure* st,
                      const dmt_config* cfg) {
  if (!out || !model || !st || !cfg) return fail(DMT_ERR_INVALID, "null argument");
  *out = nullptr;
  if (!supported(model)) return fail(DMT_ERR_INVALID, "unsupported model/dimension/precision combination");
  if (st->n_recordings <= 0 || !st->n_segments || !st->n_points)
    return fail(DMT_ERR_INVALID, "empty structure");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(DMT_ERR_HIP, "no HIP device available: libdmt has no CPU fallback");
  if (cfg->device < 0 || cfg->device >= ndev) return fail(DMT_ERR_INVALID, "bad device ordinal");
  HIP_OK(hipSetDevice(cfg->device));
  auto h = std::make_unique<dmt_ens>();
  h->spin_wait = !(std::getenv("DMT_SPIN_WAIT") && std::getenv("DMT_SPIN_WAIT")[0] == '0');
  h->key = ModelKey{model->model, model->precision, model->d, model->m};
  h->d = model->d;
  h->m = model->m;
  h->hp = model->d * (model->d + 1) / 2;
  h->esz = model->precision == DMT_F64 ? 8 : 4;
  h->device = cfg->device;
  h->seed = cfg->seed;
  h->grid_shared = cfg->grid_shared ? 1 : 0;
  h->R = st->n_recordings;
  h->rec_seg0.assign(h->R + 1, 0);
  for (int64_t r = 0; r < h->R; ++r) {
    if (st->n_segments[r] <= 0) return fail(DMT_ERR_INVALID, "recording without segments");
    h->rec_seg0[r + 1] = h->rec_seg0[r] + st->n_segments[r];
  }
  h->G = h->rec_seg0[h->R];
  if (h->G > INT32_MAX) return fail(DMT_ERR_INVALID, "too many segments");
  h->seg_rec.resize(h->G);
  h->seg_q.resize(h->G);
  h->seg_np.resize(h->G);
  h->pt_off.resize(h->G);
  h->st_off.resize(h->G);
  std::vector<int64_t> recQ(h->R);
  int64_t P = 0, S = 0;
  for (int64_t r = 0; r < h->R; ++r) {
    int64_t q = 0;
    for (int64_t g = h->rec_seg0[r]; g < h->rec_seg0[r + 1]; ++g) {
      const int32_t np = st->n_points[g];
      if (np < 2) return fail(DMT_ERR_INVALID, "segment with fewer than 2 grid points");
      h->seg_rec[g] = (int32_t)r;
      h->seg_q[g] = (int32_t)q;
      h->seg_np[g] = np;
      h->pt_off[g] = P;
      h->st_off[g] = S;
      q += np;
      P += np;
      S += np - 1;
    }
    recQ[r] = q;
  }
  h->P = P;
  h->S = S;
  h->Q0 = recQ[0];
  if (h->grid_shared) {
    for (int64_t r = 1; r < h->R; ++r) {
      if (h->rec_seg0[r + 1] - h->rec_seg0[r] != h->rec_seg0[1] - h->rec_seg0[0])
        return fail(DMT_ERR_INVALID, "grid_shared requires identical segment structure");
      for (int64_t k = 0; k < h->rec_seg0[1]; ++k)
        if (h->seg_np[h->rec_seg0[r] + k] != h->seg_np[k])
          return fail(DMT_ERR_INVALID, "grid_shared requires identical segment structure");
    }
  }
  // Mapping: MAP_WAVE (one wavefront per block) while the ensemble is too small to give every
  // SIMD several 64-recording lane tiles; MAP_LANE (one lane per block) beyond that.
  if (cfg->mapping == MAP_LANE || cfg->mapping == MAP_WAVE) h->mapping = cfg->mapping;
  else if (cfg->mapping == MAP_AUTO) h->mapping = h->R <= kAutoWaveMaxRecordings ? MAP_WAVE : MAP_LANE;
  else return fail(DMT_ERR_INVALID, "bad mapping");
  // linear drift (OU): the recursion is an affine scan, always one workgroup per block
  if (model->model == DMT_MODEL_OU) h->mapping = MAP_WAVE;
  if (const char* e = std::getenv("DMT_MCMC_PERSIST")) h->persist = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("DMT_MCMC_RESIDENT")) h->resident = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("DMT_MCMC_SCAN_TD")) h->persist_td = std::strcmp(e, "1") == 0;
  if (const char* e = std::getenv("DMT_MCMC_PC")) h->resident_pc = std::max(0, std::min(2, std::atoi(e)));
  if (const char* e = std::getenv("DMT_PC_BPW")) h->pc_bpw1 = std::atoi(e) == 1;
  if (const char* e = std::getenv("DMT_DISPATCH_EVENTS")) h->dispatch_events = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("DMT_EVENT_FLAGS")) h->event_flags = (unsigned)std::strtoul(e, nullptr, 0);
  if (const char* e = std::getenv("DMT_LANE_SPLIT")) h->lane_split = std::atoi(e);
  if (const char* e = std::getenv("DMT_LANE_PAIR")) h->lane_pair = std::atoi(e);
  if (const char* e = std::getenv("DMT_DEFER")) h->defer = std::atoi(e) != 0;
  if (const char* e = std::getenv("DMT_SERVICE")) h->service = std::atoi(e) != 0;
  if (const char* e = std::getenv("DMT_SVC_IDLE_MS")) h->svc_idle_ms = std::max(0.1, std::atof(e));
  {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, cfg->device) == hipSuccess &&
        khz > 0)
      h->wall_khz = (uint64_t)khz;
  }
  if (const char* e = std::getenv("DMT_REPAIR_DIV")) h->repair_div = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("DMT_REPAIR_MIN")) h->repair_min = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("DMT_SCAN_RESIDENT")) h->scan_resident = std::strcmp(e, "0") != 0;
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, h->device) != hipSuccess)
      return fail(DMT_ERR_HIP, "hipGetDeviceProperties failed");
    // The kernels are built for gfx950 only, and the in-kernel fetch_ll hand-offs rely on its
    // write-through (sc1) agent-scope stores being performed at vmcnt(0): refuse
    // any other architecture rather than run unvalidated ordering assumptions.
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
      const std::string arch = prop.gcnArchName;
      return fail(DMT_ERR_HIP, "libdmt is built and validated for gfx950 (MI355X) only; device " +
                                   std::to_string(cfg->device) + " is " + arch);
    }
    h->n_simd = 4 * (int64_t)prop.multiProcessorCount;
  }
  h->tw = h->mapping == MAP_WAVE ? 1 : kLanes;
  // lane packets: the path planes of an fp32 lane-mapped ensemble (non-linear
  // drift; OU ensembles are wave-mapped) in 16-point pieces per lane; DMT_PATH_PACKETS=0: rows
  h->pk = (h->mapping == MAP_LANE && model->precision == DMT_F32) ? kPathPacket : 0;
  if (const char* e = std::getenv("DMT_PATH_PACKETS")) h->pk = std::atoi(e) == 0 ? 0 : h->pk;
  h->ntiles = (h->R + h->tw - 1) / h->tw;
  h->tile_qoff.assign(h->ntiles + 1, 0);
  {
    // with packets every tile starts at row ≡ pk − 1 (mod pk): a recording's first segment then
    // starts one point before a packet boundary, so its steps' points fill whole packets
    // (run_segment_pk's fast path); the planes end on a packet boundary
    const int64_t pk = h->pk;
    auto up = [&](int64_t v) { return pk ? (v + pk - 1) / pk * pk : v; };
    int64_t end = 0;
    for (int64_t t = 0; t < h->ntiles; ++t) {
      int64_t mx = 0;
      for (int64_t r = t * h->tw; r < std::min<int64_t>(h->R, (t + 1) * h->tw); ++r) mx = std::max(mx, recQ[r]);
      h->tile_qoff[t] = pk ? up(end) + pk - 1 : end;
      end = h->tile_qoff[t] + mx + kPadPoints;
    }
    h->tile_qoff[h->ntiles] = up(end);
  }
  h->Ptile = h->tile_qoff[h->ntiles];
  HIP_OK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  dmt_ens* hp = h.get();
  DMT_TRY(ens_alloc(hp, &hp->d_pt_off, hp->G));
  DMT_TRY(ens_alloc(hp, &hp->d_st_off, hp->G));
  DMT_TRY(ens_alloc(hp, &hp->d_tile_qoff, hp->ntiles + 1));
  DMT_TRY(ens_alloc(hp, &hp->d_seg_rec, hp->G));
  DMT_TRY(ens_alloc(hp, &hp->d_seg_q, hp->G));
  DMT_TRY(ens_alloc(hp, &hp->d_seg_np, hp->G));
  HIP_OK(hipMemcpy(hp->d_pt_off, hp->pt_off.data(), hp->G * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(hp->d_st_off, hp->st_off.data(), hp->G * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(hp->d_tile_qoff, hp->tile_qoff.data(), (hp->ntiles + 1) * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(hp->d_seg_rec, hp->seg_rec.data(), hp->G * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(hp->d_seg_q, hp->seg_q.data(), hp->G * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(hp->d_seg_np, hp->seg_np.data(), hp->G * 4, hipMemcpyHostToDevice));
  for (int i = 0; i < 4; ++i) {  // paths: u in buffer 0, u° in 1 (kSelInit); laws: slot 0
    DMT_TRY(ens_alloc(hp, &hp->d_sel[i], hp->G));
    HIP_OK(hipMemset(hp->d_sel[i], i < 2 ? kSelInit : 0, hp->G));
  }
  hp->h_selPP.assign(hp->G, 0);
  hp->h_selPPB.assign(hp->G, 0);
  // MAP_LANE: a third path buffer per container, so that a wave's proposals can go to a buffer
  // none of its lanes' u occupies (DESIGN.md §2 "path buffers"; DMT_PATH_BUFS=2: two)
  hp->nbuf = hp->mapping == MAP_LANE ? 3 : 2;
  if (const char* e = std::getenv("DMT_PATH_BUFS")) hp->nbuf = std::atoi(e) == 2 ? 2 : hp->nbuf;
  if (hp->pk) hp->nbuf = 2;  // lane packets: per-lane buffers cost nothing
  if (const char* e = std::getenv("DMT_FULL_COPY")) hp->full_copy = std::atoi(e) != 0;
  for (int s = 0; s < hp->nbuf; ++s) {
    DMT_TRY(ens_alloc_bytes(hp, &hp->d_X[s], plane_elems(hp, hp->d) * hp->esz));
    DMT_TRY(ens_alloc_bytes(hp, &hp->d_W[s], plane_elems(hp, hp->m) * hp->esz));
    HIP_OK(hipMemset(hp->d_X[s], 0, plane_elems(hp, hp->d) * hp->esz));
    HIP_OK(hipMemset(hp->d_W[s], 0, plane_elems(hp, hp->m) * hp->esz));
  }
  DMT_TRY(ens_alloc(hp, &hp->d_red, 3));
  HIP_OK(hipHostMalloc((void**)&hp->h_red, 3 * sizeof(double), hipHostMallocDefault));
  // internal layout 0: one terminal block per recording over all its segments, ρ = 0
  // (the view draw_proposal_path!(u::SamplingUnit) acts on, src/sampling_unit.jl:118-120)
  {
    std::vector<int32_t> nb(hp->R, 1), sf(hp->R, 0), sl(hp->R);
    std::vector<uint8_t> lt(hp->R, 1);
    std::vector<double> rz(hp->R, 0.0);
    for (int64_t r = 0; r < hp->R; ++r) sl[r] = (int32_t)(hp->rec_seg0[r + 1] - hp->rec_seg0[r] - 1);
    int32_t id;
    DMT_TRY(build_layout(hp, nb.data(), sf.data(), sl.data(), lt.data(), rz.data(), 0, &id));
  }
  HIP_OK(hipStreamSynchronize(hp->stream));
  *out = h.release();
  return DMT_OK;
}

dmt_status dmt_destroy(dmt_ens* h) {
  if (!h) return DMT_OK;
  (void)hipSetDevice(h->device);
  (void)svc_stop(h);
#ifdef DMT_SVC_PROBE
  if (h->d_svc_probe) {  // median stage durations (µs) of the first service's iterations
    std::vector<uint64_t> pr(8 * kSvcCap);
    (void)hipMemcpy(pr.data(), h->d_svc_probe, pr.size() * 8, hipMemcpyDeviceToHost);
    const double tick_us = 1e3 / (double)h->wall_khz;
    std::vector<double> d[3];
    for (int64_t r = 1; r + 1 < kSvcCap && pr[8 * (r + 1)]; ++r) {
      const uint64_t* p = &pr[8 * r];
      d[0].push_back((p[1] - p[0]) * tick_us);   // poller saw the post -> last workgroup's gate
      d[1].push_back((p[2] - p[1]) * tick_us);   // -> last workgroup's records sent (publish, B2)
      d[2].push_back((pr[8 * (r + 1)] - p[2]) * tick_us);  // -> the next post seen (PCIe, host)
    }
    for (int64_t r = 1; r < (int64_t)std::min(h->svc_host_post.size(), h->svc_host_seen.size()); ++r)
      if (h->svc_host_post[r] > 0 && h->svc_host_seen[r - 1] > 0)
        h->svc_host_code.push_back(h->svc_host_post[r] - h->svc_host_seen[r - 1]);
    if (!h->svc_host_code.empty()) {
      auto& v = h->svc_host_code;
      std::sort(v.begin(), v.end());
      std::fprintf(stderr, "svc probe host code (result seen -> next post) median %.2f us  p10 %.2f  p90 %.2f\n",
                   v[v.size() / 2], v[v.size() / 10], v[v.size() * 9 / 10]);
    }
    const char* nm[3] = {"gate", "publish", "return"};
    for (int k = 0; k < 3; ++k) {
      if (d[k].empty()) continue;
      std::sort(d[k].begin(), d[k].end());
      std::fprintf(stderr, "svc probe %-9s median %.2f us  p10 %.2f  p90 %.2f  (n=%zu)\n", nm[k],
                   d[k][d[k].size() / 2], d[k][d[k].size() / 10], d[k][d[k].size() * 9 / 10],
                   d[k].size());
    }
  }
#endif
  if (std::getenv("DMT_SVC_STATS"))
    std::fprintf(stderr, "dmt service: %llu starts, %llu relaunches, %llu posts, %llu waits\n",
                 (unsigned long long)h->svc_stats.starts, (unsigned long long)h->svc_stats.relaunches,
                 (unsigned long long)h->svc_stats.posts, (unsigned long long)h->svc_stats.waits);
  (void)stream_wait(h);
  drain_timing(h);
  for (auto e : h->free_events) (void)hipEventDestroy(e);
  for (auto& L : h->layouts)
    if (L) L->release();
  void* ps[] = {h->d_pt_off, h->d_st_off, h->d_tile_qoff, h->d_seg_rec, h->d_seg_q, h->d_seg_np,
                h->d_sel[0], h->d_sel[1], h->d_sel[2], h->d_sel[3], h->d_X[0], h->d_X[1],
                h->d_X[2], h->d_W[0], h->d_W[1], h->d_W[2], h->d_t, h->d_sdt, h->d_stage, h->d_Z, h->d_red, h->d_gather,
                h->d_red_work, h->d_run, h->d_run_gather, h->d_part, h->d_red_lb, h->d_obsH,
                h->d_obsF, h->d_obsc, h->d_obsv, h->d_fail, h->d_fchunk_off, h->d_segsel,
                h->d_qbuf, h->d_tbuf};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  for (int s = 0; s < 2; ++s)
    for (int k = 0; k < 2; ++k) {
      if (h->d_H[s][k] && !(s == 1 && h->d_H[1][k] == h->d_H[0][k])) (void)hipFree(h->d_H[s][k]);
      if (h->d_F[s][k]) (void)hipFree(h->d_F[s][k]);
      if (s == 0 && h->d_aux[k]) (void)hipFree(h->d_aux[k]);
      if (h->d_law[s][k]) (void)hipFree(h->d_law[s][k]);
    }
  for (int k = 0; k < 2; ++k)
    if (h->d_snap[k]) (void)hipFree(h->d_snap[k]);
  if (h->comm) (void)ncclCommDestroy(h->comm);
  if (h->h_red) (void)hipHostFree(h->h_red);
  if (h->h_run) (void)hipHostFree(h->h_run);
  if (h->svc_host) (void)hipHostFree(h->svc_host);
  if (h->svc_rec) (void)hipHostFree(h->svc_rec);
  if (h->d_svc_words) (void)hipFree(h->d_svc_words);
  if (h->d_svc_probe) (void)hipFree(h->d_svc_probe);
  (void)hipStreamDestroy(h->stream);
  delete h;
  return DMT_OK;
}

dmt_status dmt_upload_grid(dmt_ens* h, const double* t) {
  DMT_TRY(enter(h));
  if (!t) return fail(DMT_ERR_INVALID, "null grid");
  if (h->grid_shared) {
    if (!h->d_t) {
      DMT_TRY(ens_alloc_bytes(h, &h->d_t, (h->Q0 + kPadPoints) * h->esz));
      HIP_OK(hipMemsetAsync(h->d_t, 0, (h->Q0 + kPadPoints) * h->esz, h->stream));
    }
    DMT_TRY(ensure_stage(h, h->Q0));
    HIP_OK(hipMemcpyAsync(h->d_stage, t, h->Q0 * 8, hipMemcpyHostToDevice, h->stream));
    HIP_OK(launch_cast(h->key.precision, h->d_stage, h->d_t, h->Q0, h->stream));
    // √dt per point for the lane kernels' draws: the value their step computes, sqrt(t[q+1] −
    // t[q]) in the working precision (IEEE subtraction and correctly rounded square root on
    // both sides), so a table read replaces a per-step square root bit for bit
    if (!h->d_sdt) DMT_TRY(ens_alloc_bytes(h, &h->d_sdt, (h->Q0 + kPadPoints) * h->esz));
    const int64_t ns = h->Q0 + kPadPoints;
    if (h->key.precision == DMT_F64) {
      std::vector<double> v(ns, 0.0);
      for (int64_t q = 0; q + 1 < h->Q0; ++q) v[q] = std::sqrt(t[q + 1] - t[q]);
      HIP_OK(hipMemcpyAsync(h->d_sdt, v.data(), ns * 8, hipMemcpyHostToDevice, h->stream));
      HIP_OK(stream_wait(h));
    } else {
      std::vector<float> v(ns, 0.0f);
      for (int64_t q = 0; q + 1 < h->Q0; ++q) v[q] = std::sqrt((float)t[q + 1] - (float)t[q]);
      HIP_OK(hipMemcpyAsync(h->d_sdt, v.data(), ns * 4, hipMemcpyHostToDevice, h->stream));
      HIP_OK(stream_wait(h));
    }
  } else {
    if (!h->d_t) {
      DMT_TRY(ens_alloc_bytes(h, &h->d_t, plane_elems(h, 1) * h->esz));
      HIP_OK(hipMemsetAsync(h->d_t, 0, plane_elems(h, 1) * h->esz, h->stream));
    }
    DMT_TRY(ensure_stage(h, h->P));
    HIP_OK(hipMemcpyAsync(h->d_stage, t, h->P * 8, hipMemcpyHostToDevice, h->stream));
    HIP_OK(launch_to_planes(h->key.precision, h->tw, h->d_stage, h->d_t, h->d_t, nullptr, 0, 1, h->P,
                            h->d_pt_off, h->G, h->d_seg_rec, h->d_seg_q, h->d_tile_qoff, h->stream));
  }
  HIP_OK(stream_wait(h));
  h->have_t = true;
  return DMT_OK;
}

}  // extern "C"

namespace {
__global__ void k_scatter_rows(const double* src, double* dst0, double* dst1, const uint8_t* sel,
                               int flip, int64_t G, int stride) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= G * stride) return;
  const int64_t g = e / stride;
  ((sel[g] ^ flip) & 1 ? dst1 : dst0)[e] = src[e];
}
}  // namespace

extern "C" {

dmt_status dmt_upload_law(dmt_ens* h, int32_t unit, int32_t kind, const double* H,
                          int32_t H_shared, const double* F, const double* laws) {
  DMT_TRY(enter(h));
  if ((unit != DMT_U && unit != DMT_UPROP) || (kind != DMT_LAW_PP && kind != DMT_LAW_PPB))
    return fail(DMT_ERR_INVALID, "bad unit/kind");
  uint8_t* sel = h->d_sel[2 + kind];
  const std::vector<uint8_t>& hsel = kind == 0 ? h->h_selPP : h->h_selPPB;
  const int esz = (int)h->esz;
  // The very first upload of a law kind also fills the other unit: u° = deepcopy(u)
  // (src/sampling_pair.jl:51).  Later uploads touch only the named unit, as
  // recompute_guiding_term!(bb.b) leaves bb.b°'s laws alone (src/block.jl:102-110).
  const bool seeded = h->have_law[0][kind] || h->have_law[1][kind];
  if (H) {
    if (H_shared) {
      // a shared table serves every segment of the unit: the unit's laws must sit in one
      // physical slot for all segments (selectors uniform)
      for (int64_t g = 1; g < h->G; ++g)
        if (hsel[g] != hsel[0])
          return fail(DMT_ERR_STATE, "shared H upload needs uniform PP selectors (laws swapped on a subset)");
      if (h->d_H[0][kind] && !h->H_shared[kind])
        return fail(DMT_ERR_STATE, "cannot switch an uploaded per-segment H table to shared");
      const int slot = hsel[0] ^ unit;
      for (int s = 0; s < 2; ++s)
        if (!h->d_H[s][kind]) {
          DMT_TRY(ens_alloc_bytes(h, &h->d_H[s][kind], (h->Q0 + kPadPoints) * h->hp * esz));
          HIP_OK(hipMemsetAsync(h->d_H[s][kind], 0, (h->Q0 + kPadPoints) * h->hp * esz, h->stream));
        }
      h->H_shared[kind] = 1;
      DMT_TRY(ensure_stage(h, h->Q0 * h->hp));
      HIP_OK(hipMemcpyAsync(h->d_stage, H, h->Q0 * h->hp * 8, hipMemcpyHostToDevice, h->stream));
      HIP_OK(launch_cast(h->key.precision, h->d_stage, h->d_H[slot][kind], h->Q0 * h->hp, h->stream));
      if (!seeded) {  // first upload of this kind also seeds the other unit
        HIP_OK(launch_cast(h->key.precision, h->d_stage, h->d_H[slot ^ 1][kind], h->Q0 * h->hp, h->stream));
      }
    } else {
      if (h->d_H[0][kind] && h->H_shared[kind])
        return fail(DMT_ERR_STATE, "cannot switch an uploaded shared H table to per-segment");
      for (int s = 0; s < 2; ++s)
        if (!h->d_H[s][kind]) {
          DMT_TRY(ens_alloc_bytes(h, &h->d_H[s][kind], plane_elems(h, h->hp) * esz));
          HIP_OK(hipMemsetAsync(h->d_H[s][kind], 0, plane_elems(h, h->hp) * esz, h->stream));
        }
      h->H_shared[kind] = 0;
      DMT_TRY(ensure_stage(h, h->P * h->hp));
      HIP_OK(hipMemcpyAsync(h->d_stage, H, h->P * h->hp * 8, hipMemcpyHostToDevice, h->stream));
      for (int pass = 0; pass < (seeded ? 1 : 2); ++pass)
        HIP_OK(launch_to_planes(h->key.precision, h->tw, h->d_stage, h->d_H[0][kind], h->d_H[1][kind], sel,
                                unit ^ pass, h->hp, h->P, h->d_pt_off, h->G, h->d_seg_rec, h->d_seg_q,
                                h->d_tile_qoff, h->stream));
    }
  }
  if (F) {
    for (int s = 0; s < 2; ++s)
      if (!h->d_F[s][kind]) {
        DMT_TRY(ens_alloc_bytes(h, &h->d_F[s][kind], plane_elems(h, h->d) * esz));
        HIP_OK(hipMemsetAsync(h->d_F[s][kind], 0, plane_elems(h, h->d) * esz, h->stream));
      }
    DMT_TRY(ensure_stage(h, h->P * h->d));
    HIP_OK(hipMemcpyAsync(h->d_stage, F, h->P * h->d * 8, hipMemcpyHostToDevice, h->stream));
    for (int pass = 0; pass < (seeded ? 1 : 2); ++pass)
      HIP_OK(launch_to_planes(h->key.precision, h->tw, h->d_stage, h->d_F[0][kind], h->d_F[1][kind], sel,
                              unit ^ pass, h->d, h->P, h->d_pt_off, h->G, h->d_seg_rec, h->d_seg_q,
                              h->d_tile_qoff, h->stream));
  }
  if (laws) {
    bool td2 = false;
    for (int64_t g = 0; g < h->G && !td2; ++g) td2 = laws[g * DMT_LAW_STRIDE + DMT_LAW_AUXTD] == 2.0;
    if (td2 && h->d_aux[kind] && !h->aux_has_a[kind])
      return fail(DMT_ERR_INVALID, "a law record with DMT_LAW_AUXTD = 2 needs the aux table's ã "
                                   "columns (dmt_upload_aux_a with d*d + d + d(d+1)/2 columns)");
    h->law_auxtd2[unit][kind] = td2;
    if (!seeded) h->law_auxtd2[unit ^ 1][kind] = td2;
    for (int s = 0; s < 2; ++s)
      if (!h->d_law[s][kind]) {
        DMT_TRY(ens_alloc(h, &h->d_law[s][kind], h->G * DMT_LAW_STRIDE));
        HIP_OK(hipMemsetAsync(h->d_law[s][kind], 0, h->G * DMT_LAW_STRIDE * 8, h->stream));
      }
    DMT_TRY(ensure_stage(h, h->G * DMT_LAW_STRIDE));
    HIP_OK(hipMemcpyAsync(h->d_stage, laws, h->G * DMT_LAW_STRIDE * 8, hipMemcpyHostToDevice, h->stream));
    const int64_t n = h->G * DMT_LAW_STRIDE;
    for (int pass = 0; pass < (seeded ? 1 : 2); ++pass) {
      k_scatter_rows<<<(unsigned)((n + 255) / 256), 256, 0, h->stream>>>(
          h->d_stage, h->d_law[0][kind], h->d_law[1][kind], sel, unit ^ pass, h->G, DMT_LAW_STRIDE);
      HIP_OK(hipGetLastError());
    }
  }
  HIP_OK(stream_wait(h));
  if (H || F || laws) h->have_law[unit][kind] = true;
  return DMT_OK;
}

dmt_status dmt_upload_aux(dmt_ens* h, int32_t kind, const double* aux) {
  return dmt_upload_aux_a(h, kind, aux, (int32_t)(h ? h->d * h->d + h->d : 0));
}

dmt_status dmt_upload_aux_a(dmt_ens* h, int32_t kind, const double* aux, int32_t ncols) {
  DMT_TRY(enter(h));
  if (kind != DMT_LAW_PP && kind != DMT_LAW_PPB) return fail(DMT_ERR_INVALID, "bad kind");
  const int nb = (int)(h->d * h->d + h->d), na = nb + (int)h->hp;  // table columns (kAuxCols)
  if (aux && ncols != nb && ncols != na)
    return fail(DMT_ERR_INVALID, "aux table: d*d + d or d*d + d + d(d+1)/2 columns per point");
  if (!aux) {
    if (h->d_aux[kind]) {
      HIP_OK(stream_wait(h));
      (void)hipFree(h->d_aux[kind]);
      h->bytes -= plane_elems(h, na) * (int64_t)h->esz;
      h->d_aux[kind] = nullptr;
    }
    h->aux_has_a[kind] = false;
    return DMT_OK;
  }
  if (ncols == nb && (h->law_auxtd2[0][kind] || h->law_auxtd2[1][kind]))
    return fail(DMT_ERR_INVALID, "a law record with DMT_LAW_AUXTD = 2 needs the aux table's ã "
                                 "columns (d*d + d + d(d+1)/2 per point)");
  h->aux_has_a[kind] = ncols == na;
  const int C = na;  // the device table always holds the ã columns (zero when not given)
  if (!h->d_aux[kind]) {
    DMT_TRY(ens_alloc_bytes(h, &h->d_aux[kind], plane_elems(h, C) * h->esz));
    HIP_OK(hipMemsetAsync(h->d_aux[kind], 0, plane_elems(h, C) * h->esz, h->stream));
  }
  DMT_TRY(ensure_stage(h, h->P * C));
  if (ncols == na) {
    HIP_OK(hipMemcpyAsync(h->d_stage, aux, h->P * C * 8, hipMemcpyHostToDevice, h->stream));
  } else {  // B̃, β̃ only: pad each row with zero ã columns
    std::vector<double> full((size_t)h->P * C, 0.0);
    for (int64_t p = 0; p < h->P; ++p)
      std::memcpy(&full[(size_t)p * C], aux + (size_t)p * nb, nb * 8);
    HIP_OK(hipMemcpyAsync(h->d_stage, full.data(), h->P * C * 8, hipMemcpyHostToDevice, h->stream));
    HIP_OK(stream_wait(h));
  }
  // one table for u and u°: both destinations of the per-segment copy are the table itself
  HIP_OK(launch_to_planes(h->key.precision, h->tw, h->d_stage, h->d_aux[kind], h->d_aux[kind],
                          h->d_sel[2 + kind], 0, C, h->P, h->d_pt_off, h->G, h->d_seg_rec,
                          h->d_seg_q, h->d_tile_qoff, h->stream));
  HIP_OK(stream_wait(h));  // the host buffer is the caller's
  return DMT_OK;
}

dmt_status dmt_set_paths(dmt_ens* h, int32_t unit, const double* X, const double* W) {
  DMT_TRY(enter(h));
  if (unit != DMT_U && unit != DMT_UPROP) return fail(DMT_ERR_INVALID, "bad unit");
  const double* src[2] = {X, W};
  const int C[2] = {h->d, h->m};
  for (int w = 0; w < 2; ++w) {
    if (!src[w]) continue;
    DMT_TRY(ensure_stage(h, h->P * C[w]));
    HIP_OK(hipMemcpyAsync(h->d_stage, src[w], h->P * C[w] * 8, hipMemcpyHostToDevice, h->stream));
    void** dst = w == 0 ? h->d_X : h->d_W;
    // Wiener paths are held as increments on the device
    HIP_OK(launch_to_planes(h->key.precision, h->tw, h->d_stage, dst[0], dst[1], h->d_sel[w], unit, C[w],
                            h->P, h->d_pt_off, h->G, h->d_seg_rec, h->d_seg_q, h->d_tile_qoff,
                            h->stream, w == 1 ? 1 : 0, dst[2], 1, h->pk));
  }
  HIP_OK(stream_wait(h));
  return DMT_OK;
}

dmt_status dmt_download_paths(dmt_ens* h, int32_t unit, int32_t what, double* out) {
  DMT_TRY(enter(h));
  if ((unit != DMT_U && unit != DMT_UPROP) || what < 0 || what > 2 || !out)
    return fail(DMT_ERR_INVALID, "bad unit/what/out");
  const int C = what == 0 ? h->d : h->m;
  DMT_TRY(ensure_stage(h, h->P * C));
  void** src = what == 0 ? h->d_X : h->d_W;
  const int sk = what == 0 ? 0 : 1;  // selector kind
  if (what != 1)  // XX, or the Wiener increments exactly as held (DMT_PATH_DW)
    HIP_OK(launch_from_planes(h->key.precision, h->tw, h->d_stage, src[0], src[1], h->d_sel[sk], unit,
                              C, h->P, h->d_pt_off, h->G, h->d_seg_rec, h->d_seg_q, h->d_tile_qoff,
                              h->stream, src[2], 1, h->pk));
  else  // increments -> cumulative Wiener path
    HIP_OK(launch_from_planes_incr(h->key.precision, h->tw, h->d_stage, src[0], src[1], h->d_sel[what],
                                   unit, C, h->G, h->d_pt_off, h->d_seg_np, h->d_seg_rec, h->d_seg_q,
                                   h->d_tile_qoff, h->stream, src[2], 1, h->pk));
  HIP_OK(hipMemcpyAsync(out, h->d_stage, h->P * C * 8, hipMemcpyDeviceToHost, h->stream));
  HIP_OK(stream_wait(h));
  return DMT_OK;
}

dmt_status dmt_download_law(dmt_ens* h, int32_t unit, int32_t kind, double* H, double* F,
                            double* laws) {
  DMT_TRY(enter(h));
  if ((unit != DMT_U && unit != DMT_UPROP) || (kind != DMT_LAW_PP && kind != DMT_LAW_PPB))
    return fail(DMT_ERR_INVALID, "bad unit/kind");
  if (!h->have_law[0][kind] && !h->have_law[1][kind]) return fail(DMT_ERR_STATE, "law not uploaded");
  const uint8_t* sel = h->d_sel[2 + kind];
  if (H) {
    if (h->H_shared[kind]) {
      const std::vector<uint8_t>& hsel = kind == 0 ? h->h_selPP : h->h_selPPB;
      DMT_TRY(ensure_stage(h, h->Q0 * h->hp));
      HIP_OK(launch_cast_back(h->key.precision, h->d_H[hsel[0] ^ unit][kind], h->d_stage,
                              h->Q0 * h->hp, h->stream));
      HIP_OK(hipMemcpyAsync(H, h->d_stage, h->Q0 * h->hp * 8, hipMemcpyDeviceToHost, h->stream));
    } else {
      DMT_TRY(ensure_stage(h, h->P * h->hp));
      HIP_OK(launch_from_planes(h->key.precision, h->tw, h->d_stage, h->d_H[0][kind], h->d_H[1][kind],
                                sel, unit, h->hp, h->P, h->d_pt_off, h->G, h->d_seg_rec, h->d_seg_q,
                                h->d_tile_qoff, h->stream));
      HIP_OK(hipMemcpyAsync(H, h->d_stage, h->P * h->hp * 8, hipMemcpyDeviceToHost, h->stream));
    }
    HIP_OK(stream_wait(h));
  }
  if (F) {
    DMT_TRY(ensure_stage(h, h->P * h->d));
    HIP_OK(launch_from_planes(h->key.precision, h->tw, h->d_stage, h->d_F[0][kind], h->d_F[1][kind],
                              sel, unit, h->d, h->P, h->d_pt_off, h->G, h->d_seg_rec, h->d_seg_q,
                              h->d_tile_qoff, h->stream));
    HIP_OK(hipMemcpyAsync(F, h->d_stage, h->P * h->d * 8, hipMemcpyDeviceToHost, h->stream));
    HIP_OK(stream_wait(h));
  }
  if (laws) {
    std::vector<double> l0(h->G * DMT_LAW_STRIDE), l1(h->G * DMT_LAW_STRIDE);
    std::vector<uint8_t> hs(h->G);
    HIP_OK(hipMemcpyAsync(l0.data(), h->d_law[0][kind], l0.size() * 8, hipMemcpyDeviceToHost, h->stream));
    HIP_OK(hipMemcpyAsync(l1.data(), h->d_law[1][kind], l1.size() * 8, hipMemcpyDeviceToHost, h->stream));
    HIP_OK(hipMemcpyAsync(hs.data(), sel, h->G, hipMemcpyDeviceToHost, h->stream));
    HIP_OK(stream_wait(h));
    for (int64_t g = 0; g < h->G; ++g) {
      const std::vector<double>& src = (hs[g] ^ unit) ? l1 : l0;
      std::memcpy(laws + g * DMT_LAW_STRIDE, src.data() + g * DMT_LAW_STRIDE, DMT_LAW_STRIDE * 8);
    }
  }
  return DMT_OK;
}

dmt_status dmt_create_layout(dmt_ens* h, const int32_t* n_blocks, const int32_t* seg_first,
                             const int32_t* seg_last, const uint8_t* last, const double* rho,
                             int64_t hist_len, int32_t* layout_id) {
  DMT_TRY(enter(h));
  if (!n_blocks || !seg_first || !seg_last || !last || !rho || !layout_id)
    return fail(DMT_ERR_INVALID, "null argument");
  DMT_TRY(build_layout(h, n_blocks, seg_first, seg_last, last, rho, hist_len, layout_id));
  HIP_OK(stream_wait(h));
  return DMT_OK;
}

dmt_status dmt_layout_size(dmt_ens* h, int32_t layout, int64_t* n) {
  DMT_TRY(enter(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  *n = L->nblocks;
  return DMT_OK;
}

dmt_status dmt_draw_unit(dmt_ens* h, int32_t unit, int64_t r0, int64_t r1, const double* Z,
                         int64_t iter, uint32_t salt, double* ll_out, uint8_t* success_out) {
  DMT_TRY(enter(h));
  if (unit != DMT_U && unit != DMT_UPROP) return fail(DMT_ERR_INVALID, "bad unit");
  Layout* L;
  DMT_TRY(get_layout(h, 0, &L));
  DMT_TRY(check_range(L, r0, r1));
  DMT_TRY(law_ready(h, unit, L, r0, r1));
  RngKey key;
  DMT_TRY(draw_key(h, iter, salt, false, &key));
  const double* dZ;
  DMT_TRY(upload_Z(h, Z, &dZ));
  DMT_TRY(run_block_kernel(h, L, MODE_FRESH, DMT_K_DRAW, r0, r1, unit, unit, unit, unit, unit, dZ,
                           key.iter, key.salt, L->d_llp, L->d_success, false));
  if (ll_out) HIP_OK(hipMemcpyAsync(ll_out, L->d_llp + r0, (r1 - r0) * 8, hipMemcpyDeviceToHost, h->stream));
  if (success_out) HIP_OK(hipMemcpyAsync(success_out, L->d_success + r0, r1 - r0, hipMemcpyDeviceToHost, h->stream));
  HIP_OK(stream_wait(h));
  return DMT_OK;
}

dmt_status dmt_draw_proposal(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, const double* Z,
                             int64_t iter, uint32_t salt, uint8_t* success_out) {
  DMT_TRY(check_h(h));
  {  // a draw the next accept may fuse with leaves a running service alone
    Layout* Lq;
    DMT_TRY(get_layout(h, layout, &Lq));
    if (!(!Z && !success_out && h->defer && resident_range(h, Lq))) DMT_TRY(enter(h));
    DMT_TRY(flush_deferred(h));  // an earlier deferred draw: launched first
    h->fused.on = false;         // fetch_ll° now sees this proposal
  }
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  DMT_TRY(law_ready(h, 0, L, b0, b1));
  RngKey key;
  DMT_TRY(draw_key(h, iter, salt, true, &key));
  if (!Z && !success_out && h->defer && resident_range(h, L)) {
    // deferred: launched with the accept_reject that follows (one fused launch), or by the
    // next call that needs it (flush_deferred)
    h->def.on = true;
    h->def.layout = layout;
    h->def.b0 = b0;
    h->def.b1 = b1;
    h->def.iter = key.iter;
    h->def.salt = key.salt;
    return DMT_OK;
  }
  const double* dZ;
  DMT_TRY(upload_Z(h, Z, &dZ));
  // law: accepted u.PP (flip 0); start from u.XX; write u°.XX/u°.WW; read u.WW
  DMT_TRY(run_block_kernel(h, L, MODE_PCN, DMT_K_DRAW, b0, b1, 0, 0, 1, 0, 1, dZ, key.iter,
                           key.salt, L->d_llp, L->d_success, false));
  if (success_out) {
    HIP_OK(hipMemcpyAsync(success_out, L->d_success + b0, b1 - b0, hipMemcpyDeviceToHost, h->stream));
    HIP_OK(stream_wait(h));
  } else if (Z) {
    HIP_OK(stream_wait(h));  // host Z buffer must stay valid until copied
  }
  return DMT_OK;
}

static AcceptArgs accept_args(dmt_ens* h, Layout* L, int64_t b0, int64_t b1, const double* dE,
                              int64_t mcmciter, RngKey key, uint8_t* acc_dev) {
  AcceptArgs a{};
  a.b0 = b0;
  a.b1 = b1;
  a.nblocks = L->nblocks;
  a.gfirst = L->d_gfirst;
  a.glast = L->d_glast;
  a.selX = h->d_sel[0];
  a.selW = h->d_sel[1];
  a.ll = L->d_ll;
  a.llp = L->d_llp;
  a.ll_hist = L->d_llh;
  a.llp_hist = L->d_llph;
  a.acc_hist = L->d_acch;
  a.hist_len = L->hist_len;
  a.mcmciter = mcmciter;
  a.E = dE;
  a.seed = h->seed;
  a.seg_base = h->seg_base;
  a.salt = key.salt;
  a.key_iter = key.iter;
  a.key_delta = 0;
  a.acc_out = acc_dev;
  return a;
}

static dmt_status ensure_red_work(dmt_ens* h, int64_t n) {
  const int64_t groups = std::max<int64_t>(1, (n + 1023) / 1024);
  // multi-level tree: 2 x 3 doubles per group; single-launch form (k_accept_reduce_lb):
  // 3 x 256 partials + a zeroed counter
  if (!h->d_red_lb) {
    DMT_TRY(ens_alloc(h, &h->d_red_lb, 3 * 256 + 2));
    HIP_OK(hipMemsetAsync(h->d_red_lb, 0, (3 * 256 + 2) * 8, h->stream));
  }
  const int64_t need = groups * 6;
  if (need > h->red_work_n) {
    if (h->d_red_work) { (void)hipFree(h->d_red_work); h->bytes -= h->red_work_n * 8; }
    h->d_red_work = nullptr;
    h->red_work_n = 0;
    DMT_TRY(ens_alloc(h, &h->d_red_work, need));
    h->red_work_n = need;
  }
  return DMT_OK;
}

// The rank-order combination of all-gathered partials (dmt_combine_rank_partials):
// all[(r·n_iter + i)·3 + c] → out[i·3 + c], complete adjacent-pair tree over ranks padded with
// zeros to a power of two, + 0.0.
static void combine_rank_partials(const double* all, int nranks, int64_t n_iter, double* out) {
  int n2 = 1;
  while (n2 < nranks) n2 <<= 1;
  std::vector<double> lv(n2);
  for (int64_t i = 0; i < n_iter; ++i)
    for (int c = 0; c < 3; ++c) {
      std::fill(lv.begin(), lv.end(), 0.0);
      for (int r = 0; r < nranks; ++r) lv[r] = all[(r * n_iter + i) * 3 + c];
      for (int w = n2; w > 1; w >>= 1)
        for (int j = 0; j < w / 2; ++j) lv[j] = lv[2 * j] + lv[2 * j + 1];
      out[3 * i + c] = lv[0] + 0.0;
    }
}

// d_red (3 partials of this rank) -> host values, combined over ranks with RCCL
static dmt_status finish_reduction(dmt_ens* h, double* v, bool global = true) {
  if (h->comm && global) {
    if (!h->d_gather) DMT_TRY(ens_alloc(h, &h->d_gather, 3 * h->nranks));
    if (ncclAllGather(h->d_red, h->d_gather, 3, ncclDouble, h->comm, h->stream) != ncclSuccess)
      return fail(DMT_ERR_COMM, "ncclAllGather failed");
    std::vector<double> all(3 * h->nranks);
    HIP_OK(hipMemcpyAsync(all.data(), h->d_gather, 3 * h->nranks * 8, hipMemcpyDeviceToHost, h->stream));
    HIP_OK(stream_wait(h));
    combine_rank_partials(all.data(), h->nranks, 1, v);  // fixed rank-order tree
  } else {
    HIP_OK(hipMemcpyAsync(h->h_red, h->d_red, 24, hipMemcpyDeviceToHost, h->stream));
    HIP_OK(stream_wait(h));
    v[0] = h->h_red[0];
    v[1] = h->h_red[1];
    v[2] = h->h_red[2];
  }
  return DMT_OK;
}

static dmt_status mcmc_step_impl(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                                 int64_t mcmciter, uint32_t salt, double* ll, double* ll_prop,
                                 int64_t* n_acc, bool global) {
  DMT_TRY(enter(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  DMT_TRY(law_ready(h, 0, L, b0, b1));
  if (L->hist_len > 0 && (mcmciter < 1 || mcmciter > L->hist_len))
    return fail(DMT_ERR_INVALID, "mcmciter outside 1:ll_hist_len");
  RngKey key;  // one key for the draw and its decision (disjoint normal / Exp(1) streams)
  DMT_TRY(draw_key(h, mcmciter, salt, false, &key));
  DMT_TRY(run_block_kernel(h, L, MODE_PCN, DMT_K_DRAW, b0, b1, 0, 0, 1, 0, 1, nullptr, key.iter,
                           key.salt, L->d_llp, nullptr, false));
  DMT_TRY(ensure_red_work(h, b1 - b0));
  {
    TimedScope ts(h, DMT_K_ACCEPT);
    HIP_OK(launch_accept_reduce(accept_args(h, L, b0, b1, nullptr, mcmciter, key, nullptr),
                                h->d_red_work, h->d_red_lb, h->d_red, h->stream));
  }
  double v[3];
  DMT_TRY(finish_reduction(h, v, global));
  if (ll) *ll = v[0];
  if (ll_prop) *ll_prop = v[1];
  if (n_acc) *n_acc = (int64_t)v[2];
  return DMT_OK;
}

dmt_status dmt_mcmc_step(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int64_t mcmciter,
                         uint32_t salt, double* ll, double* ll_prop, int64_t* n_acc) {
  return mcmc_step_impl(h, layout, b0, b1, mcmciter, salt, ll, ll_prop, n_acc, true);
}

dmt_status dmt_mcmc_step_local(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                               int64_t mcmciter, uint32_t salt, double* ll, double* ll_prop,
                               int64_t* n_acc) {
  return mcmc_step_impl(h, layout, b0, b1, mcmciter, salt, ll, ll_prop, n_acc, false);
}

// Capacity of dmt_mcmc_run's buffers: grown geometrically with a floor, so that a run of a
// different length (e.g. a benchmark's warm-up and timed runs) does not free and re-allocate
// device memory — hipFree synchronises the device.
static int64_t grown_cap(int64_t need, int64_t cap, int64_t floor_) {
  return std::max({need, 2 * cap, floor_});
}

dmt_status dmt_set_run_snapshots(dmt_ens* h, int64_t every, int64_t slot0) {
  DMT_TRY(enter(h));
  if (every < 0) return fail(DMT_ERR_INVALID, "every must be >= 0");
  if (every > 0 && !h->snap_mask) return fail(DMT_ERR_STATE, "no snapshot slots (dmt_snapshot_reserve)");
  if (every > 0 && (slot0 < 0 || slot0 >= h->snap_slots)) return fail(DMT_ERR_INVALID, "slot out of range");
  h->run_snap_every = every;
  h->run_snap_next = slot0;
  return DMT_OK;
}

static double hp_now() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
static const bool g_host_prof = std::getenv("DMT_HOST_PROFILE") != nullptr;
static double g_hp[6];
static dmt_status mcmc_run_launch(dmt_ens* h, Layout* L, int64_t b0, int64_t b1, int64_t iter0,
                                  int64_t n_iter, uint32_t salt, int64_t key_delta, bool multi);
static dmt_status mcmc_run_collect(dmt_ens* h, int64_t n_iter, double* out, bool multi);

static dmt_status mcmc_run_impl(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                                int64_t iter0, int64_t n_iter, uint32_t salt, double* out,
                                bool global) {
  if (g_host_prof) g_hp[0] = hp_now();
  DMT_TRY(enter(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  DMT_TRY(law_ready(h, 0, L, b0, b1));
  DMT_TRY(check_salt(salt));
  if (n_iter < 0 || iter0 < 1) return fail(DMT_ERR_INVALID, "bad iteration range");
  if (n_iter == 0) return DMT_OK;
  if (L->hist_len > 0 && iter0 + n_iter - 1 > L->hist_len)
    return fail(DMT_ERR_INVALID, "iterations outside 1:ll_hist_len");
  if (h->run_snap_every > 0) {
    // snapshots inside the run (the smoothing loop's `deepcopy(sp.u.XX)` every k iterations,
    // docs/src/tutorials/biblock/smoothing.md:40-44): the run is cut after every iteration
    // k ≡ 0 mod every and u is snapshotted there, stream-ordered (no host round trip); the
    // pieces take the same stream keys as one run (auto keys: consecutive counter values)
    const int64_t every = h->run_snap_every;
    h->run_snap_every = 0;
    dmt_status st = DMT_OK;
    for (int64_t done = 0; done < n_iter && st == DMT_OK;) {
      const int64_t it = iter0 + done;
      const int64_t k = ((it + every - 1) / every) * every;  // next snapshot iteration >= it
      const int64_t n = std::min(n_iter - done, k - it + 1);
      st = mcmc_run_impl(h, layout, b0, b1, it, n, salt, out ? out + 3 * done : nullptr, global);
      done += n;
      if (st == DMT_OK && (iter0 + done - 1) % every == 0) {
        st = dmt_snapshot_take(h, DMT_U, h->run_snap_next, iter0 + done - 1);
        h->run_snap_next = (h->run_snap_next + 1) % h->snap_slots;
      }
    }
    h->run_snap_every = every;
    return st;
  }
  // stream keys: iteration it draws its normals and its Exp(1) variables with key word
  // it + key_delta (explicit: the iteration itself; auto: n_iter consecutive counter values,
  // never straddling a 2^32 boundary so that the salt word is constant over the run)
  int64_t key_delta = 0;
  if (salt == DMT_RNG_AUTO) {
    uint64_t base = h->rng_ctr;
    if ((base & 0xFFFFFFFFull) + (uint64_t)n_iter > 0x100000000ull)
      base = (base | 0xFFFFFFFFull) + 1;
    h->rng_ctr = base + (uint64_t)n_iter;
    h->rng_pending = false;
    salt = auto_key(base).salt;
    key_delta = (int64_t)(uint32_t)base - iter0;
  }
  // BlockEnsemble level (global): the partials of every rank; BiBlock / BlockCollection
  // level: this rank's blocks only, no collective (src/block_collection.jl:144,156)
  const bool multi = h->comm != nullptr && global;
  DMT_TRY(mcmc_run_launch(h, L, b0, b1, iter0, n_iter, salt, key_delta, multi));
  return mcmc_run_collect(h, n_iter, out, multi);
}

// Queue n_iter MCMC iterations (iteration it keyed by it + key_delta, salt) on the stream; the
// per-iteration (fetch_ll, fetch_ll°, accepted count) go to pinned h_run (one rank) or d_run
// (multi: for the all-gather, which is queued too).  No host synchronisation.
static dmt_status mcmc_run_launch(dmt_ens* h, Layout* L, int64_t b0, int64_t b1, int64_t iter0,
                                  int64_t n_iter, uint32_t salt, int64_t key_delta, bool multi) {
  if (n_iter > h->run_cap) {
    if (h->d_run) { (void)hipFree(h->d_run); h->bytes -= h->run_cap * 24; h->d_run = nullptr; }
    if (h->h_run) { (void)hipHostFree(h->h_run); h->h_run = nullptr; h->h_run_dev = nullptr; }
    if (h->d_run_gather) {
      (void)hipFree(h->d_run_gather);
      h->bytes -= h->run_cap * 24 * h->nranks;
      h->d_run_gather = nullptr;
    }
    const int64_t cap = grown_cap(n_iter, h->run_cap, 4096);
    h->run_cap = 0;
    DMT_TRY(ens_alloc(h, &h->d_run, 3 * cap));
    // coherent and mapped: the kernels write the per-iteration results straight into it
    HIP_OK(hipHostMalloc((void**)&h->h_run, 3 * cap * sizeof(double),
                         hipHostMallocMapped | hipHostMallocCoherent));
    void* dp = nullptr;
    HIP_OK(hipHostGetDevicePointer(&dp, h->h_run, 0));
    h->h_run_dev = static_cast<double*>(dp);
    if (multi) DMT_TRY(ens_alloc(h, &h->d_run_gather, 3 * cap * h->nranks));
    h->run_cap = cap;
  } else if (multi && !h->d_run_gather) {
    DMT_TRY(ens_alloc(h, &h->d_run_gather, 3 * h->run_cap * h->nranks));
  }
  DMT_TRY(ensure_red_work(h, b1 - b0));
  // per-iteration results: one rank → straight into pinned host memory; several → device
  // memory for the all-gather
  double* run_out = multi ? h->d_run : h->h_run_dev;
  const int64_t nb = b1 - b0;
  // kernel eligibility of the range: from the layout's flags when they decide it (no host
  // loop over the blocks per call), else block by block
  const bool lay_res = L->single_seg && L->max_steps <= kResidentMaxSteps;
  // (an ensemble with a time-dependent auxiliary table runs the per-iteration kernels, or with
  // DMT_MCMC_SCAN_TD=1 k_mcmc_scan's TD instantiation; the register-resident kernels take the
  // law's own B̃, β̃ and are not eligible)
  bool persist = h->persist && h->key.model == DMT_MODEL_OU &&
                 (h->persist_td || !has_aux_table(h));
  for (int64_t b = b0; b < b1 && persist && !L->single_seg; ++b)
    persist = L->glast[b] - L->gfirst[b] + 1 <= kPersistMaxSegments;
  bool resident = persist && h->key.d <= 2 && h->resident && !has_aux_table(h);
  for (int64_t b = b0; b < b1 && resident && !lay_res; ++b)
    resident = L->glast[b] == L->gfirst[b] && h->seg_np[L->gfirst[b]] - 1 <= kResidentMaxSteps;
  if (persist) {
    // the whole run in one launch per chunk of iterations (k_mcmc_scan / k_mcmc_resident),
    // every iteration's fetch_ll tree formed inside the launch
    const int64_t chunk_max = std::max<int64_t>(1, (int64_t(64) << 20) / (24 * nb));
    const int64_t chunk = std::min<int64_t>(n_iter, chunk_max);
    // part [chunk][3][nb], then the tree nodes (node1 [3 chunk][≤ nb], node2 [3 chunk][≤ nb/16 + 1]),
    // then the arrival counters (≤ nb/16 + 2 uint32) at the end of the buffer
    const int64_t cnt_words = nb / 2 + 8;  // doubles
    auto need_for = [&](int64_t it) { return 3 * it * (2 * nb + nb / 16 + 1) + cnt_words; };
    const int64_t need = need_for(chunk);
    if (need > h->part_cap) {
      if (h->d_part) { (void)hipFree(h->d_part); h->bytes -= h->part_cap * 8; h->d_part = nullptr; }
      const int64_t cap_it = std::min(chunk_max, std::max<int64_t>(chunk, 256));
      const int64_t cap = std::max(need, need_for(cap_it));
      h->part_cap = 0;
      DMT_TRY(ens_alloc(h, &h->d_part, cap));
      HIP_OK(hipMemsetAsync(h->d_part, 0, cap * 8, h->stream));  // zero the arrival counter
      h->part_cap = cap;
    }
    for (int64_t i0 = 0; i0 < n_iter; i0 += chunk) {
      const int64_t n = std::min(chunk, n_iter - i0);
      AcceptArgs c = accept_args(h, L, b0, b1, nullptr, iter0 + i0, RngKey{0, salt}, nullptr);
      c.key_delta = key_delta;
      hipError_t e;
      {
        TimedScope ts(h, DMT_K_DRAW, true, n);
        auto fill = [&](auto& a) {
          fill_common(h, L, a);
          a.success = L->d_success;  // the last iteration's draw flags (dmt_draw_success)
          a.b0 = b0;
          a.b1 = b1;
          a.tile0 = 0;
          a.tile1 = 0;
          a.xd_flip = 1;  // MODE_PCN: start u, write u°, read u.W, write u°.W
          a.wd_flip = 1;
          a.salt = salt;
        };
        // the arrival counters of the in-kernel trees: the last cnt_words doubles of d_part
        double* counter = h->d_part + h->part_cap - cnt_words;
        if (g_host_prof) g_hp[1] = hp_now();
        if (h->key.precision == DMT_F64) {
          BlockArgs<double> a{};
          fill(a);
          e = launch_mcmc_persistent(h->key, &a, c, iter0 + i0, n, h->d_part, nb,
                                     !resident ? 0 : (h->pc_bpw1 && h->resident_pc == 1) ? 4 : 1 + h->resident_pc,
                                     run_out + 3 * i0, (unsigned*)counter, h->stream);
        } else {
          BlockArgs<float> a{};
          fill(a);
          e = launch_mcmc_persistent(h->key, &a, c, iter0 + i0, n, h->d_part, nb,
                                     !resident ? 0 : (h->pc_bpw1 && h->resident_pc == 1) ? 4 : 1 + h->resident_pc,
                                     run_out + 3 * i0, (unsigned*)counter, h->stream);
        }
      }
      if (g_host_prof) g_hp[2] = hp_now();
      if (e != hipSuccess) return fail(DMT_ERR_HIP, std::string("k_mcmc_scan: ") + hipGetErrorString(e));
    }
  } else {
    // every iteration is stream-ordered: no host synchronisation until the end
    for (int64_t i = 0; i < n_iter; ++i) {
      const int64_t it = iter0 + i;
      const RngKey key{(uint32_t)(it + key_delta), salt};
      DMT_TRY(run_block_kernel(h, L, MODE_PCN, DMT_K_DRAW, b0, b1, 0, 0, 1, 0, 1, nullptr,
                               key.iter, key.salt, L->d_llp, L->d_success, false));
      {
        TimedScope ts(h, DMT_K_ACCEPT);
        HIP_OK(launch_accept_reduce(accept_args(h, L, b0, b1, nullptr, it, key, nullptr),
                                    h->d_red_work, h->d_red_lb, run_out + 3 * i, h->stream));
      }
    }
  }
  // one all-gather of every iteration's three partials, whichever kernel path ran on this
  // rank (ranks may differ in path eligibility; the collective sequence must not)
  if (multi && ncclAllGather(h->d_run, h->d_run_gather, 3 * n_iter, ncclDouble, h->comm,
                             h->stream) != ncclSuccess)
    return fail(DMT_ERR_COMM, "ncclAllGather failed");
  return DMT_OK;
}

// Wait for a queued run and return its per-iteration results (rank-order tree over ranks).
static dmt_status mcmc_run_collect(dmt_ens* h, int64_t n_iter, double* out, bool multi) {
  if (!out) {
    HIP_OK(stream_wait(h));
    return DMT_OK;
  }
  if (!multi) {
    if (g_host_prof) g_hp[3] = hp_now();
    HIP_OK(stream_wait(h));
    if (g_host_prof) g_hp[4] = hp_now();
    std::memcpy(out, h->h_run, 24 * n_iter);
    if (g_host_prof)
      std::fprintf(stderr, "hostprof n=%lld pre=%.1f launch=%.1f post=%.1f wait=%.1f tail=%.1f\n",
                   (long long)n_iter, g_hp[1] - g_hp[0], g_hp[2] - g_hp[1], g_hp[3] - g_hp[2],
                   g_hp[4] - g_hp[3], hp_now() - g_hp[4]);
    return DMT_OK;
  }
  std::vector<double> all(3 * h->nranks * n_iter);
  HIP_OK(hipMemcpyAsync(all.data(), h->d_run_gather, all.size() * 8, hipMemcpyDeviceToHost,
                        h->stream));
  HIP_OK(stream_wait(h));
  combine_rank_partials(all.data(), h->nranks, n_iter, out);  // the tree of finish_reduction
  return DMT_OK;
}

dmt_status dmt_mcmc_run(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int64_t iter0,
                        int64_t n_iter, uint32_t salt, double* out) {
  return mcmc_run_impl(h, layout, b0, b1, iter0, n_iter, salt, out, true);
}

dmt_status dmt_mcmc_run_local(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int64_t iter0,
                              int64_t n_iter, uint32_t salt, double* out) {
  return mcmc_run_impl(h, layout, b0, b1, iter0, n_iter, salt, out, false);
}

// (Re-)launch the service's kernel from its iteration `base` (0: a new service).  The launch
// runs at most cap − base iterations, each once the host has posted it.
static dmt_status svc_launch(dmt_ens* h, uint64_t base) {
  auto& v = h->svc;
  Layout* L;
  DMT_TRY(get_layout(h, v.layout, &L));
  const int64_t nb = v.b1 - v.b0;
  SvcArgs sv{};
  void* dp = nullptr;
  HIP_OK(hipHostGetDevicePointer(&dp, h->svc_host, 0));
  sv.posted = (const uint64_t*)dp;
  sv.stop = (const uint32_t*)((char*)dp + 64);
  HIP_OK(hipHostGetDevicePointer(&dp, h->svc_rec, 0));
  sv.rec = (uint64_t*)dp;
  sv.go = h->d_svc_words;        // separate 128-byte lines
  sv.quit = h->d_svc_words + 16;
  HIP_OK(hipMemsetAsync(h->d_svc_words, 0, 32 * sizeof(uint64_t), h->stream));
  sv.idle_ticks = (uint64_t)(h->wall_khz * h->svc_idle_ms);
  sv.base = base;
#ifdef DMT_SVC_PROBE
  if (!h->d_svc_probe) {
    DMT_TRY(ens_alloc(h, &h->d_svc_probe, 8 * kSvcCap));
    HIP_OK(hipMemsetAsync(h->d_svc_probe, 0, 8 * kSvcCap * 8, h->stream));
  }
  sv.probe = h->d_svc_probe;
#endif
  AcceptArgs c = accept_args(h, L, v.b0, v.b1, nullptr, v.iter0 + (int64_t)base,
                             RngKey{0, v.salt}, nullptr);
  c.key_delta = (int64_t)v.key0 - v.iter0;
  auto fill = [&](auto& a) {
    fill_common(h, L, a);
    a.success = L->d_success;
    a.b0 = v.b0;
    a.b1 = v.b1;
    a.xd_flip = 1;  // MODE_PCN: start u, write u°, read u.W, write u°.W
    a.wd_flip = 1;
    a.salt = v.salt;
  };
  hipError_t e;
  if (h->key.precision == DMT_F64) {
    BlockArgs<double> a{};
    fill(a);
    e = launch_mcmc_service(h->key, &a, c, v.iter0 + (int64_t)base, v.cap - (int64_t)base,
                            nullptr, nb, h->resident_pc, (int)(h->n_simd / 4), sv,
                            h->stream);
  } else {
    BlockArgs<float> a{};
    fill(a);
    e = launch_mcmc_service(h->key, &a, c, v.iter0 + (int64_t)base, v.cap - (int64_t)base,
                            nullptr, nb, h->resident_pc, (int)(h->n_simd / 4), sv,
                            h->stream);
  }
  if (e != hipSuccess) return fail(DMT_ERR_HIP, std::string("resident service: ") + hipGetErrorString(e));
  return DMT_OK;
}

namespace {
dmt_status svc_relaunch(dmt_ens* h, uint64_t base) { return svc_launch(h, base); }
}  // namespace

// A new service on (layout, b0:b1) whose first iteration is mcmciter with stream key `key`
static dmt_status svc_start(dmt_ens* h, Layout* L, int32_t layout, int64_t b0, int64_t b1,
                            int64_t mcmciter, RngKey key) {
  const int64_t nb = b1 - b0;
  if (!h->svc_host) {
    HIP_OK(hipHostMalloc((void**)&h->svc_host, 256, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(h->svc_host, 0, 256);
    DMT_TRY(ens_alloc(h, &h->d_svc_words, 32));
  }
  const int64_t nwg = (nb + 3) / 4;  // the launch's workgroups (4 blocks each)
  if (nwg > h->svc_rec_nwg) {
    if (h->svc_rec) { (void)hipHostFree(h->svc_rec); h->svc_rec = nullptr; }
    h->svc_rec_nwg = 0;
    HIP_OK(hipHostMalloc((void**)&h->svc_rec, 2 * nwg * 64, hipHostMallocMapped | hipHostMallocCoherent));
    h->svc_rec_nwg = nwg;
  }
  std::memset(h->svc_rec, 0, 2 * nwg * 64);  // no tag of an earlier service can match
  auto& v = h->svc;
  v.nwg = nwg;
  v.done = 0;
  v.layout = layout;
  v.b0 = b0;
  v.b1 = b1;
  v.iter0 = mcmciter;
  v.key0 = key.iter;
  v.salt = key.salt;
  v.cap = L->hist_len > 0 ? std::min<int64_t>(kSvcCap, L->hist_len - mcmciter + 1) : kSvcCap;
  v.posted = 0;
  __atomic_store_n(svc_posted(h), (uint64_t)0, __ATOMIC_RELEASE);
  __atomic_store_n(svc_stopw(h), 0u, __ATOMIC_RELEASE);
  DMT_TRY(svc_launch(h, 0));
  ++h->svc_stats.starts;
  v.on = true;
  return DMT_OK;
}

dmt_status dmt_accept_reject(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, const double* E,
                             int64_t mcmciter, uint32_t salt, uint8_t* acc_out) {
  DMT_TRY(check_h(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  if (L->hist_len > 0 && (mcmciter < 1 || mcmciter > L->hist_len))
    return fail(DMT_ERR_INVALID, "mcmciter outside 1:ll_hist_len");
  const bool fuse = h->def.on && h->def.layout == layout && h->def.b0 == b0 &&
                    h->def.b1 == b1 && !E && !acc_out && mcmciter >= 1;
  h->fused.on = false;
  if (!fuse) {
    DMT_TRY(svc_stop(h));
    DMT_TRY(flush_deferred(h));
  }
  RngKey key;
  DMT_TRY(accept_key(h, mcmciter, salt, &key));
  if (fuse && key.iter == h->def.iter && key.salt == h->def.salt) {
    // the deferred draw and this decision with ONE stream key: one launch of the resident MCMC
    // kernel (draw, decision, histories, fetch_ll tree) — the launch dmt_mcmc_step makes — or
    // the next iteration of the running resident service
    h->def.on = false;
    if (h->service && h->resident_pc >= 1 && !h->comm && h->svc_fit_nb != b1 - b0) {
      h->svc_fit_nb = b1 - b0;
      h->svc_fit = mcmc_service_fits(h->key, b1 - b0, h->resident_pc, (int)(h->n_simd / 4));
    }
    if (h->service && h->resident_pc >= 1 && !h->comm && h->svc_fit) {
      const auto now = std::chrono::steady_clock::now();
      auto& v = h->svc;
      const bool cont =
          v.on && v.layout == layout && v.b0 == b0 && v.b1 == b1 && v.salt == key.salt &&
          key.iter == (uint32_t)(v.key0 + v.posted) && mcmciter == v.iter0 + (int64_t)v.posted &&
          (int64_t)v.posted < v.cap;
      if (!cont) {
        DMT_TRY(svc_stop(h));
        DMT_TRY(svc_start(h, L, layout, b0, b1, mcmciter, key));
      }
      const uint64_t slot = v.posted;
      // the records alternate between two sets: every earlier iteration is seen complete before
      // this one is posted, so that it never overwrites records not yet read (immediate when the
      // caller fetched the previous iteration)
      DMT_TRY(svc_wait_done(h, slot));
      if (cont && std::chrono::duration<double, std::milli>(now - v.t_last).count() >
                      0.5 * h->svc_idle_ms &&
          hipStreamQuery(h->stream) == hipSuccess) {
        // the host was away long enough for the launch to leave idle: launch it again from
        // this iteration at once (instead of finding out in svc_wait_done)
        ++h->svc_stats.relaunches;
        DMT_TRY(svc_relaunch(h, slot));
        svc_check_degraded(h);
      }
      v.posted = slot + 1;
      ++h->svc_stats.posts;
#ifdef DMT_SVC_PROBE
      if (h->svc_host_post.size() < (size_t)kSvcCap) h->svc_host_post.resize(kSvcCap, 0.0);
      if (h->svc_stats.starts == 1) h->svc_host_post[slot] = hp_now();
#endif
      v.t_last = now;
      __atomic_store_n(svc_posted(h), v.posted, __ATOMIC_RELEASE);
      h->fused.on = true;
      h->fused.layout = layout;
      h->fused.b0 = b0;
      h->fused.b1 = b1;
      h->fused.mcmciter = mcmciter;
      h->fused.slot = (int64_t)slot;
      return DMT_OK;
    }
    DMT_TRY(svc_stop(h));
    DMT_TRY(ensure_red_work(h, b1 - b0));
    DMT_TRY(mcmc_run_launch(h, L, b0, b1, mcmciter, 1, key.salt,
                            (int64_t)key.iter - mcmciter, false));
    h->fused.on = true;
    h->fused.layout = layout;
    h->fused.b0 = b0;
    h->fused.b1 = b1;
    h->fused.mcmciter = mcmciter;
    h->fused.slot = -1;
    return DMT_OK;
  }
  DMT_TRY(flush_deferred(h));  // a different key: the draw's own launch first
  const double* dE = nullptr;
  if (E) {
    DMT_TRY(ensure_Z(h, std::max<int64_t>(b1 - b0, 1)));
    HIP_OK(hipMemcpyAsync(h->d_Z, E, (b1 - b0) * 8, hipMemcpyHostToDevice, h->stream));
    dE = h->d_Z;
  }
  AcceptArgs a = accept_args(h, L, b0, b1, dE, mcmciter, key, acc_out ? L->d_acc : nullptr);
  {
    TimedScope ts(h, DMT_K_ACCEPT);
    HIP_OK(launch_accept(a, h->stream));
  }
  if (acc_out) {
    HIP_OK(hipMemcpyAsync(acc_out, L->d_acc, b1 - b0, hipMemcpyDeviceToHost, h->stream));
    HIP_OK(stream_wait(h));
  } else if (E) {
    HIP_OK(stream_wait(h));
  }
  return DMT_OK;
}

dmt_status dmt_loglikhd(dmt_ens* h, int32_t layout, int32_t unit, int64_t b0, int64_t b1) {
  DMT_TRY(enter(h));
  if (unit != DMT_U && unit != DMT_UPROP) return fail(DMT_ERR_INVALID, "bad unit");
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  DMT_TRY(law_ready(h, unit, L, b0, b1));
  DMT_TRY(run_block_kernel(h, L, 0, DMT_K_PATHLL, b0, b1, unit, unit, unit, unit, unit, nullptr, 0,
                           0, unit == DMT_U ? L->d_ll : L->d_llp, nullptr, true));
  return DMT_OK;
}

dmt_status dmt_recompute_path(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int32_t skip,
                              uint8_t* success_out) {
  DMT_TRY(enter(h));
  if (skip < 0) return fail(DMT_ERR_INVALID, "skip must be >= 0");
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  DMT_TRY(law_ready(h, 1, L, b0, b1));
  // law u°.PP (flip 1); start from u°.XX; write u°.XX; read u.WW (the accepted W)
  // skip: the last `skip` Euler steps of every segment add no Girsanov term (GuidedProposals'
  // solve_and_ll!(…; skip)); the path itself is solved to the end
  DMT_TRY(run_block_kernel(h, L, MODE_RECOMPUTE, DMT_K_RECOMPUTE, b0, b1, 1, 1, 1, 0, 0, nullptr, 0,
                           0, L->d_llp, success_out ? L->d_success : nullptr, 0, skip));
  if (success_out) {
    HIP_OK(hipMemcpyAsync(success_out, L->d_success + b0, b1 - b0, hipMemcpyDeviceToHost, h->stream));
    HIP_OK(stream_wait(h));
  }
  return DMT_OK;
}

dmt_status dmt_find_W_for_X(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1) {
  DMT_TRY(enter(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  DMT_TRY(law_ready(h, 0, L, b0, b1));
  // laws u.PP (+ P_last) (flip 0); read u.XX (flip 0); write u.WW in place (flip 0)
  DMT_TRY(run_block_kernel(h, L, MODE_RECOMPUTE, DMT_K_RECOMPUTE, b0, b1, 0, 0, 0, 0, 0, nullptr, 0,
                           0, nullptr, nullptr, 2));
  return DMT_OK;
}

dmt_status dmt_upload_obs(dmt_ens* h, const double* Hobs, const double* Fobs, const double* cobs,
                          double artificial_noise) {
  DMT_TRY(enter(h));
  if (!Hobs || !Fobs || !cobs || !(artificial_noise > 0.0))
    return fail(DMT_ERR_INVALID, "bad arguments to dmt_upload_obs");
  if (!h->d_obsH) {
    DMT_TRY(ens_alloc(h, &h->d_obsH, h->G * h->hp));
    DMT_TRY(ens_alloc(h, &h->d_obsF, h->G * h->d));
    DMT_TRY(ens_alloc(h, &h->d_obsc, h->G));
    DMT_TRY(ens_alloc(h, &h->d_obsv, h->G * h->d));
    DMT_TRY(ens_alloc(h, &h->d_fail, 1));
    HIP_OK(hipMemsetAsync(h->d_obsv, 0, h->G * h->d * 8, h->stream));
    // chunk offsets of the chunked filter: ceil((npts − 1) / 64) chunks per segment
    h->fchunk_off.assign(h->G + 1, 0);
    for (int64_t g = 0; g < h->G; ++g)
      h->fchunk_off[g + 1] =
          h->fchunk_off[g] + (h->seg_np[g] - 1 + flt::kFiltChunk - 1) / flt::kFiltChunk;
    DMT_TRY(ens_alloc(h, &h->d_fchunk_off, h->G + 1));
    DMT_TRY(ens_alloc(h, &h->d_segsel, h->G));
    HIP_OK(hipMemcpyAsync(h->d_fchunk_off, h->fchunk_off.data(), (h->G + 1) * 8,
                          hipMemcpyHostToDevice, h->stream));
  }
  HIP_OK(hipMemcpyAsync(h->d_obsH, Hobs, h->G * h->hp * 8, hipMemcpyHostToDevice, h->stream));
  HIP_OK(hipMemcpyAsync(h->d_obsF, Fobs, h->G * h->d * 8, hipMemcpyHostToDevice, h->stream));
  HIP_OK(hipMemcpyAsync(h->d_obsc, cobs, h->G * 8, hipMemcpyHostToDevice, h->stream));
  h->art_eps = artificial_noise;
  HIP_OK(stream_wait(h));
  return DMT_OK;
}

dmt_status dmt_set_obs(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1) {
  DMT_TRY(enter(h));
  if (!h->d_obsv) return fail(DMT_ERR_STATE, "dmt_upload_obs first");
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  HIP_OK(launch_set_obs(h->key.precision, h->tw, h->pk, h->d, h->d_X[0], h->d_X[1], h->d_X[2], h->d_sel[0],
                        h->d_tile_qoff, h->d_seg_rec, h->d_seg_q, h->d_seg_np, L->d_glast,
                        L->d_term, b0, b1, h->d_obsv, h->key.model, h->d_law[0][1],
                        h->d_law[1][1], h->stream));
  return DMT_OK;
}

}  // extern "C"

// the device backward filter over blocks [b0, b1) of `unit` (only the blocks flagged in
// `only`, when given)
static dmt_status guiding_term_device(dmt_ens* h, Layout* L, int64_t b0, int64_t b1, int32_t unit,
                                      const uint8_t* only) {
  if (!h->d_obsH) return fail(DMT_ERR_STATE, "dmt_upload_obs first");
  DMT_TRY(law_ready(h, unit, L, b0, b1));
  if (!h->d_t) return fail(DMT_ERR_STATE, "time grid not uploaded");
  for (int k = 0; k < 2; ++k)
    if (h->d_H[0][k] && h->H_shared[k])
      return fail(DMT_ERR_STATE, "the device filter writes per-point guiding tables; upload H per "
                                 "segment (not shared) to use recompute_guiding_term");
  FilterArgs a{};
  a.d = h->d;
  a.tw = h->tw;
  a.unit = unit;
  a.tile_qoff = h->d_tile_qoff;
  a.seg_rec = h->d_seg_rec;
  a.seg_q = h->d_seg_q;
  a.seg_np = h->d_seg_np;
  a.gfirst = L->d_gfirst;
  a.glast = L->d_glast;
  a.term = L->d_term;
  a.selPP = h->d_sel[2];
  a.selPPB = h->d_sel[3];
  a.b0 = b0;
  a.b1 = b1;
  for (int s = 0; s < 2; ++s)
    for (int k = 0; k < 2; ++k) {
      a.H[s][k] = h->d_H[s][k];
      a.F[s][k] = h->d_F[s][k];
      a.law[s][k] = h->d_law[s][k];
    }
  a.t = h->d_t;
  a.t_shared = h->grid_shared;
  a.aux[0] = h->d_aux[0];
  a.aux[1] = h->d_aux[1];
  a.obsH = h->d_obsH;
  a.obsF = h->d_obsF;
  a.obsc = h->d_obsc;
  a.obsv = h->d_obsv;
  a.art_eps = h->art_eps;
  a.fail = h->d_fail;
  a.only = only;
  a.pt_off = h->d_pt_off;
  a.fchunk_off = h->d_fchunk_off;
  a.segsel = h->d_segsel;
  HIP_OK(hipMemsetAsync(h->d_fail, 0, sizeof(int), h->stream));
  if (b1 - b0 >= kFiltFusedBlocks) {
    // enough blocks to fill the device: one wave per block, no transition scratch
    a.fused = 1;
    TimedScope ts(h, DMT_K_RECOMPUTE, false);
    HIP_OK(launch_backward_filter(h->key.precision, a, h->stream));
  } else {
  // batches of consecutive blocks whose points fit the transition scratch (kFiltBatchPoints,
  // or one block's points if larger)
  auto span = [&](int32_t gA, int32_t gB) { return h->pt_off[gB] + h->seg_np[gB] - h->pt_off[gA]; };
  int64_t need = 0;
  int32_t gmin = L->gfirst[b0], gmax = L->glast[b0];
  for (int64_t b = b0; b < b1; ++b) {
    need = std::max(need, span(L->gfirst[b], L->glast[b]));
    gmin = std::min(gmin, L->gfirst[b]);
    gmax = std::max(gmax, L->glast[b]);
  }
  const int64_t cap = std::max(need, std::min<int64_t>(span(gmin, gmax), kFiltBatchPoints));
  if (cap > h->qbuf_cap) {
    if (h->d_qbuf) {
      HIP_OK(stream_wait(h));
      HIP_OK(hipFree(h->d_qbuf));
      h->bytes -= h->qbuf_cap * kFiltNQ(h->d) * 8;
      h->d_qbuf = nullptr;
      h->qbuf_cap = 0;
    }
    DMT_TRY(ens_alloc(h, &h->d_qbuf, cap * kFiltNQ(h->d)));
    h->qbuf_cap = cap;
  }
  a.qbuf = h->d_qbuf;
  a.qcap = h->qbuf_cap;
  // stream events around all batches (three launches each: mark, scan, chain)
  {
  TimedScope ts(h, DMT_K_RECOMPUTE, false);
  for (int64_t bs = b0; bs < b1;) {
    int32_t gA = L->gfirst[bs], gB = L->glast[bs];
    int64_t be = bs + 1;
    for (; be < b1; ++be) {
      const int32_t nA = std::min(gA, L->gfirst[be]), nB = std::max(gB, L->glast[be]);
      if (span(nA, nB) > h->qbuf_cap) break;
      gA = nA;
      gB = nB;
    }
    a.b0 = bs;
    a.b1 = be;
    a.gA = gA;
    a.gB = gB;
    a.pA = h->pt_off[gA];
    a.fchunk_off_h0 = h->fchunk_off[gA];
    a.fchunk_off_h1 = h->fchunk_off[gB + 1];
    const int64_t items = a.fchunk_off_h1 - a.fchunk_off_h0;
    if (items > h->tbuf_cap) {
      if (h->d_tbuf) {
        HIP_OK(stream_wait(h));
        HIP_OK(hipFree(h->d_tbuf));
        h->bytes -= h->tbuf_cap * (h->hp + h->d + 1) * 8;
        h->d_tbuf = nullptr;
        h->tbuf_cap = 0;
      }
      DMT_TRY(ens_alloc(h, &h->d_tbuf, items * (h->hp + h->d + 1)));
      h->tbuf_cap = items;
    }
    a.tbuf = h->d_tbuf;
    HIP_OK(hipMemsetAsync(h->d_segsel + gA, 0, gB - gA + 1, h->stream));
    HIP_OK(launch_backward_filter(h->key.precision, a, h->stream));
    bs = be;
  }
  }
  }
  int failed = 0;
  HIP_OK(hipMemcpyAsync(&failed, h->d_fail, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  HIP_OK(stream_wait(h));
  if (failed) return fail(DMT_ERR_INVALID, "singular I + HK in the device backward filter");
  return DMT_OK;
}

extern "C" {

dmt_status dmt_recompute_guiding_term(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                                      int32_t unit) {
  DMT_TRY(enter(h));
  if (unit != DMT_U && unit != DMT_UPROP) return fail(DMT_ERR_INVALID, "bad unit");
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  return guiding_term_device(h, L, b0, b1, unit, nullptr);
}

dmt_status dmt_set_proposal_law(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int32_t n,
                                const int32_t* idx, const double* val, int32_t skip,
                                uint8_t* success_out, uint8_t* critical_out) {
  return dmt_set_proposal_law_cc(h, layout, b0, b1, n, idx, val, skip, -1, success_out,
                                 critical_out);
}

dmt_status dmt_set_proposal_law_cc(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int32_t n,
                                   const int32_t* idx, const double* val, int32_t skip,
                                   int32_t critical_change, uint8_t* success_out,
                                   uint8_t* critical_out) {
  DMT_TRY(enter(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  if (n < 0 || n > kMaxParams || (n > 0 && (!idx || !val)))
    return fail(DMT_ERR_INVALID, "bad parameter list");
  const int npar = h->key.model == DMT_MODEL_FHN      ? 5
                   : h->key.model == DMT_MODEL_LORENZ ? 3
                                                      : h->d * h->d + h->d;
  for (int k = 0; k < n; ++k)
    if (idx[k] < 0 || idx[k] >= npar) return fail(DMT_ERR_INVALID, "unknown parameter index");
  if (skip < 0) return fail(DMT_ERR_INVALID, "skip must be >= 0");
  if (critical_change < -1 || critical_change > 1)
    return fail(DMT_ERR_INVALID, "critical_change must be -1, 0 or 1");
  DMT_TRY(law_ready(h, 1, L, b0, b1));
  ParamArgs a{};
  a.cc_mode = critical_change;
  a.model = h->key.model;
  a.d = h->d;
  a.m = h->m;
  a.n = n;
  for (int k = 0; k < n; ++k) { a.idx[k] = idx[k]; a.val[k] = val[k]; }
  a.gfirst = L->d_gfirst;
  a.glast = L->d_glast;
  a.term = L->d_term;
  a.selPP = h->d_sel[2];
  a.selPPB = h->d_sel[3];
  for (int sl = 0; sl < 2; ++sl)
    for (int k = 0; k < 2; ++k) a.law[sl][k] = h->d_law[sl][k];
  if (!a.law[0][1] || !a.law[1][1]) a.law[0][1] = a.law[1][1] = nullptr;
  a.b0 = b0;
  a.b1 = b1;
  a.crit = L->d_crit;
  a.ncrit = L->d_ncrit;
  HIP_OK(hipMemsetAsync(L->d_ncrit, 0, sizeof(uint32_t), h->stream));
  HIP_OK(launch_set_prop_law(a, h->stream));
  uint32_t ncrit = 0;
  HIP_OK(hipMemcpyAsync(&ncrit, L->d_ncrit, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
  HIP_OK(stream_wait(h));
  if (ncrit > 0) DMT_TRY(guiding_term_device(h, L, b0, b1, DMT_UPROP, L->d_crit));
  if (critical_out)
    HIP_OK(hipMemcpyAsync(critical_out, L->d_crit + b0, b1 - b0, hipMemcpyDeviceToHost, h->stream));
  DMT_TRY(dmt_recompute_path(h, layout, b0, b1, skip, success_out));
  if (critical_out) HIP_OK(stream_wait(h));
  return DMT_OK;
}

dmt_status dmt_swap(dmt_ens* h, int32_t layout, int32_t what, int64_t b0, int64_t b1) {
  DMT_TRY(enter(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  if (what & ~(DMT_SWAP_XX | DMT_SWAP_WW | DMT_SWAP_PP | DMT_SWAP_LL))
    return fail(DMT_ERR_INVALID, "bad swap mask");
  uint8_t* s0 = (what & DMT_SWAP_XX) ? h->d_sel[0] : nullptr;
  uint8_t* s1 = (what & DMT_SWAP_WW) ? h->d_sel[1] : nullptr;
  uint8_t* s2 = (what & DMT_SWAP_PP) ? h->d_sel[2] : nullptr;
  uint8_t* s3 = (what & DMT_SWAP_PP) ? h->d_sel[3] : nullptr;
  // swap_PP!: BiBlock{true} swaps PP only; BiBlock{false} also P_last, P_excl, Pb_excl
  // (src/biblock.jl:180-199) — i.e. PPb of all its segments.
  HIP_OK(launch_flip(s0, s1, s2, s3, L->d_gfirst, L->d_glast, L->d_term, 1, b0, b1, h->stream));
  if (what & DMT_SWAP_PP) {
    for (int64_t b = b0; b < b1; ++b)
      for (int32_t g = L->gfirst[b]; g <= L->glast[b]; ++g) {
        h->h_selPP[g] ^= 1;
        if (!L->term[b]) h->h_selPPB[g] ^= 1;
      }
  }
  if (what & DMT_SWAP_LL) HIP_OK(launch_swap_ll(L->d_ll, L->d_llp, b0, b1, h->stream));
  return DMT_OK;
}

dmt_status dmt_save_ll(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int64_t mcmciter) {
  DMT_TRY(enter(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  if (mcmciter < 1 || mcmciter > L->hist_len) return fail(DMT_ERR_INVALID, "mcmciter outside 1:ll_hist_len");
  HIP_OK(launch_save_ll(L->d_ll, L->d_llp, L->d_llh, L->d_llph, L->nblocks, mcmciter - 1, b0, b1, h->stream));
  return DMT_OK;
}

dmt_status dmt_set_accepted(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int64_t mcmciter,
                            const uint8_t* v) {
  DMT_TRY(enter(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  if (mcmciter < 1 || mcmciter > L->hist_len) return fail(DMT_ERR_INVALID, "mcmciter outside 1:ll_hist_len");
  if (!v) return fail(DMT_ERR_INVALID, "null values");
  HIP_OK(hipMemcpyAsync(L->d_acch + (mcmciter - 1) * L->nblocks + b0, v, b1 - b0, hipMemcpyHostToDevice, h->stream));
  HIP_OK(stream_wait(h));
  return DMT_OK;
}

dmt_status dmt_set_ll(dmt_ens* h, int32_t layout, int32_t unit, int64_t b0, int64_t b1,
                      int64_t mcmciter, const double* v) {
  DMT_TRY(enter(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  if (unit != DMT_U && unit != DMT_UPROP) return fail(DMT_ERR_INVALID, "bad unit");
  if (mcmciter < 1 || mcmciter > L->hist_len) return fail(DMT_ERR_INVALID, "mcmciter outside 1:ll_hist_len");
  if (!v) return fail(DMT_ERR_INVALID, "null values");
  double* hist = unit == DMT_U ? L->d_llh : L->d_llph;
  HIP_OK(hipMemcpyAsync(hist + (mcmciter - 1) * L->nblocks + b0, v, (b1 - b0) * 8,
                        hipMemcpyHostToDevice, h->stream));
  HIP_OK(stream_wait(h));
  return DMT_OK;
}

static dmt_status block_state_ptr(Layout* L, int32_t what, void** p, size_t* esz, bool* hist) {
  *hist = false;
  switch (what) {
    case DMT_BLK_LL: *p = L->d_ll; *esz = 8; return DMT_OK;
    case DMT_BLK_LLPROP: *p = L->d_llp; *esz = 8; return DMT_OK;
    case DMT_BLK_LL_HIST: *p = L->d_llh; *esz = 8; *hist = true; break;
    case DMT_BLK_LLPROP_HIST: *p = L->d_llph; *esz = 8; *hist = true; break;
    case DMT_BLK_ACC_HIST: *p = L->d_acch; *esz = 1; *hist = true; break;
    default: return fail(DMT_ERR_INVALID, "bad block-state selector");
  }
  if (L->hist_len <= 0) return fail(DMT_ERR_STATE, "layout has no histories (ll_hist_len = 0)");
  return DMT_OK;
}

dmt_status dmt_get_block_state(dmt_ens* h, int32_t layout, int32_t what, int64_t b0, int64_t b1,
                               void* out) {
  DMT_TRY(enter(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  void* p; size_t esz; bool hist;
  DMT_TRY(block_state_ptr(L, what, &p, &esz, &hist));
  if (b1 > b0) {
    if (!hist) {
      HIP_OK(hipMemcpyAsync(out, (char*)p + b0 * esz, (b1 - b0) * esz, hipMemcpyDeviceToHost, h->stream));
    } else {
      HIP_OK(hipMemcpy2DAsync(out, (b1 - b0) * esz, (char*)p + b0 * esz, L->nblocks * esz, (b1 - b0) * esz,
                              L->hist_len, hipMemcpyDeviceToHost, h->stream));
    }
  }
  HIP_OK(stream_wait(h));
  return DMT_OK;
}

dmt_status dmt_set_block_state(dmt_ens* h, int32_t layout, int32_t what, int64_t b0, int64_t b1,
                               const void* in) {
  DMT_TRY(enter(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  void* p; size_t esz; bool hist;
  DMT_TRY(block_state_ptr(L, what, &p, &esz, &hist));
  if (b1 > b0) {
    if (!hist) {
      HIP_OK(hipMemcpyAsync((char*)p + b0 * esz, in, (b1 - b0) * esz, hipMemcpyHostToDevice, h->stream));
    } else {
      HIP_OK(hipMemcpy2DAsync((char*)p + b0 * esz, L->nblocks * esz, in, (b1 - b0) * esz, (b1 - b0) * esz,
                              L->hist_len, hipMemcpyHostToDevice, h->stream));
    }
  }
  HIP_OK(stream_wait(h));
  return DMT_OK;
}

static dmt_status fetch_ll_impl(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                                int64_t mcmciter, bool global, double* ll, double* ll_prop,
                                int64_t* n_acc) {
  DMT_TRY(check_h(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  if (h->fused.on && h->fused.layout == layout && h->fused.b0 == b0 && h->fused.b1 == b1 &&
      (mcmciter == 0 || mcmciter == h->fused.mcmciter) && !(h->comm && global)) {
    // the fused draw + accept of this range formed this very tree in its launch (same order,
    // same values): wait for it, no launch
    const double* r3 = h->h_run;
    double sv3[3];
    if (h->fused.slot >= 0) {
      DMT_TRY(svc_wait_done(h, (uint64_t)h->fused.slot + 1));
#ifdef DMT_SVC_PROBE
      if (h->svc_host_seen.size() < (size_t)kSvcCap) h->svc_host_seen.resize(kSvcCap, 0.0);
      if (h->svc_host_seen[h->fused.slot] == 0.0) h->svc_host_seen[h->fused.slot] = hp_now();
#endif
      svc_fold(h, (uint64_t)h->fused.slot, sv3);
      r3 = sv3;
    } else if (h->fused.slot == -2) {
      r3 = h->fused.vals;
    } else {
      HIP_OK(stream_wait(h));
    }
    if (ll) *ll = r3[0];
    if (ll_prop) *ll_prop = r3[1];
    if (n_acc) *n_acc = mcmciter > 0 ? (int64_t)r3[2] : 0;
    return DMT_OK;
  }
  DMT_TRY(enter(h));
  const uint8_t* acc = nullptr;
  if (mcmciter > 0) {
    if (mcmciter > L->hist_len) return fail(DMT_ERR_INVALID, "mcmciter outside 1:ll_hist_len");
    acc = L->d_acch + (mcmciter - 1) * L->nblocks + b0;
  }
  DMT_TRY(ensure_red_work(h, b1 - b0));
  {
    TimedScope ts(h, DMT_K_REDUCE, false);  // several tree launches
    HIP_OK(launch_block_sum(L->d_ll + b0, L->d_llp + b0, acc, b1 - b0, h->d_red_work, h->d_red,
                            h->stream));
  }
  double v[3];
  DMT_TRY(finish_reduction(h, v, global));
  if (ll) *ll = v[0];
  if (ll_prop) *ll_prop = v[1];
  if (n_acc) *n_acc = (int64_t)v[2];
  return DMT_OK;
}

dmt_status dmt_draw_success(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                            uint8_t* success_out) {
  DMT_TRY(check_h(h));
  Layout* L;
  DMT_TRY(get_layout(h, layout, &L));
  DMT_TRY(check_range(L, b0, b1));
  if (!success_out) return fail(DMT_ERR_INVALID, "null output");
  DMT_TRY(svc_stop(h));        // reading flags changes nothing: fused results stay valid
  DMT_TRY(flush_deferred(h));
  HIP_OK(hipMemcpyAsync(success_out, L->d_success + b0, b1 - b0, hipMemcpyDeviceToHost, h->stream));
  HIP_OK(stream_wait(h));
  return DMT_OK;
}

dmt_status dmt_fetch_ll(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1, int64_t mcmciter,
                        double* ll, double* ll_prop, int64_t* n_acc) {
  return fetch_ll_impl(h, layout, b0, b1, mcmciter, true, ll, ll_prop, n_acc);
}

dmt_status dmt_fetch_ll_local(dmt_ens* h, int32_t layout, int64_t b0, int64_t b1,
                              int64_t mcmciter, double* ll, double* ll_prop, int64_t* n_acc) {
  return fetch_ll_impl(h, layout, b0, b1, mcmciter, false, ll, ll_prop, n_acc);
}

dmt_status dmt_rng_counter(dmt_ens* h, uint64_t* next) {
  if (!h || !next) return fail(DMT_ERR_INVALID, "null argument");
  *next = h->rng_ctr;
  return DMT_OK;
}

dmt_status dmt_set_rng_counter(dmt_ens* h, uint64_t next) {
  if (!h) return fail(DMT_ERR_INVALID, "null handle");
  h->rng_ctr = next;
  h->rng_pending = false;
  return DMT_OK;
}

dmt_status dmt_rng_state(dmt_ens* h, uint64_t* next, uint64_t* last_draw, uint8_t* pending) {
  if (!h || !next || !last_draw || !pending) return fail(DMT_ERR_INVALID, "null argument");
  *next = h->rng_ctr;
  *last_draw = h->rng_last_draw;
  *pending = h->rng_pending ? 1 : 0;
  return DMT_OK;
}

dmt_status dmt_set_rng_state(dmt_ens* h, uint64_t next, uint64_t last_draw, uint8_t pending) {
  if (!h) return fail(DMT_ERR_INVALID, "null handle");
  h->rng_ctr = next;
  h->rng_last_draw = last_draw;
  h->rng_pending = pending != 0;
  return DMT_OK;
}

}  // extern "C"

template <int D>
// aux: nullptr (B̃ = Bt, β̃ = beta throughout) or [npts][ncols] per-point coefficients — B̃, β̃
// (ncols = d·d + d; ã = at throughout) or B̃, β̃, ã packed (ncols = d·d + d + hp; at unused) —
// step i taking the trapezoidal average of rows i and i + 1
static dmt_status guiding_linear_impl(const double* Bt, const double* beta, const double* aux,
                                      const double* at, int32_t npts, const double* t,
                                      const double* HT, const double* FT, double cT, double* H,
                                      double* F, double* c, int ncols = D * D + D) {
  constexpr int d = D, hp = d * (d + 1) / 2;
  const bool tda = aux && ncols == d * d + d + hp;
  flt::Mat<D> A = flt::mzero<D>(), Hc = flt::mzero<D>();
  for (int i = 0; i < d; ++i)
    for (int j = 0; j < d; ++j) {
      A(i, j) = tda ? 0.0 : at[dmt_packed(d, i, j)];
      Hc(i, j) = HT[dmt_packed(d, i, j)];
    }
  double Fc[D];
  for (int i = 0; i < d; ++i) Fc[i] = FT[i];
  double cc = cT;
  for (int i = 0; i + 1 < npts; ++i)
    if (!(t[i + 1] - t[i] > 0)) return fail(DMT_ERR_INVALID, "time grid must be strictly increasing");
  auto store = [&](int i, const flt::Mat<D>& Hs, const double* Fs, double cs) {
    for (int p = 0; p < d; ++p)
      for (int q = p; q < d; ++q) H[(int64_t)i * hp + dmt_packed(d, p, q)] = Hs(p, q);
    for (int p = 0; p < d; ++p) F[(int64_t)i * d + p] = Fs[p];
    c[i] = cs;
  };
  // step i's auxiliary drift: the law's, or the trapezoidal average of a time-dependent law's
  // coefficients at t_i and t_i+1 (second order; DESIGN.md §3, filt_aux_step on the device)
  auto coef = [&](int i, flt::Mat<D>& B, double* be, flt::Mat<D>& As) {
    if (!aux) {
      for (int k = 0; k < d * d; ++k) B.a[k] = Bt[k];
      for (int p = 0; p < d; ++p) be[p] = beta[p];
      return;
    }
    const double* r0 = aux + (int64_t)i * ncols;
    const double* r1 = r0 + ncols;
    for (int k = 0; k < d * d; ++k) B.a[k] = (r0[k] + r1[k]) * 0.5;
    for (int p = 0; p < d; ++p) be[p] = (r0[d * d + p] + r1[d * d + p]) * 0.5;
    if (tda)
      for (int p = 0; p < d; ++p)
        for (int q = 0; q < d; ++q) {
          const int e = d * d + d + dmt_packed(d, p, q);
          As(p, q) = (r0[e] + r1[e]) * 0.5;
        }
  };
  if (!flt::filter_segment<D>(coef, A, npts, [&](int i) { return t[i]; }, Hc, Fc, cc, store))
    return fail(DMT_ERR_INVALID, "singular I + HK in backward filter");
  return DMT_OK;
}

extern "C" {

dmt_status dmt_guiding_linear(int32_t d, const double* Bt, const double* beta, const double* at,
                              int32_t npts, const double* t, const double* HT, const double* FT,
                              double cT, double* H, double* F, double* c) {
  if (d < 1 || d > 3 || npts < 1 || !Bt || !beta || !at || !t || !HT || !FT || !H || !F || !c)
    return fail(DMT_ERR_INVALID, "bad arguments to dmt_guiding_linear");
  if (d == 1) return guiding_linear_impl<1>(Bt, beta, nullptr, at, npts, t, HT, FT, cT, H, F, c);
  if (d == 2) return guiding_linear_impl<2>(Bt, beta, nullptr, at, npts, t, HT, FT, cT, H, F, c);
  return guiding_linear_impl<3>(Bt, beta, nullptr, at, npts, t, HT, FT, cT, H, F, c);
}

dmt_status dmt_guiding_linear_td(int32_t d, const double* aux, const double* at, int32_t npts,
                                 const double* t, const double* HT, const double* FT, double cT,
                                 double* H, double* F, double* c) {
  if (d < 1 || d > 3 || npts < 1 || !aux || !at || !t || !HT || !FT || !H || !F || !c)
    return fail(DMT_ERR_INVALID, "bad arguments to dmt_guiding_linear_td");
  if (d == 1) return guiding_linear_impl<1>(nullptr, nullptr, aux, at, npts, t, HT, FT, cT, H, F, c);
  if (d == 2) return guiding_linear_impl<2>(nullptr, nullptr, aux, at, npts, t, HT, FT, cT, H, F, c);
  return guiding_linear_impl<3>(nullptr, nullptr, aux, at, npts, t, HT, FT, cT, H, F, c);
}

dmt_status dmt_guiding_linear_tda(int32_t d, const double* aux, int32_t npts, const double* t,
                                  const double* HT, const double* FT, double cT, double* H,
                                  double* F, double* c) {
  if (d < 1 || d > 3 || npts < 1 || !aux || !t || !HT || !FT || !H || !F || !c)
    return fail(DMT_ERR_INVALID, "bad arguments to dmt_guiding_linear_tda");
  const int nc = d * d + d + d * (d + 1) / 2;
  if (d == 1) return guiding_linear_impl<1>(nullptr, nullptr, aux, nullptr, npts, t, HT, FT, cT, H, F, c, nc);
  if (d == 2) return guiding_linear_impl<2>(nullptr, nullptr, aux, nullptr, npts, t, HT, FT, cT, H, F, c, nc);
  return guiding_linear_impl<3>(nullptr, nullptr, aux, nullptr, npts, t, HT, FT, cT, H, F, c, nc);
}

dmt_status dmt_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return fail(DMT_ERR_INVALID, "null id");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return fail(DMT_ERR_COMM, "ncclGetUniqueId failed");
  static_assert(sizeof(ncclUniqueId) == 128, "unexpected ncclUniqueId size");
  std::memcpy(id_out, &id, 128);
  return DMT_OK;
}

dmt_status dmt_comm_init(dmt_ens* h, int32_t nranks, int32_t rank, const uint8_t* id) {
  DMT_TRY(enter(h));
  if (nranks < 1 || rank < 0 || rank >= nranks || !id) return fail(DMT_ERR_INVALID, "bad comm args");
  if (h->comm) {
    (void)ncclCommDestroy(h->comm);
    h->comm = nullptr;
  }
  h->nranks = nranks;
  h->rank = rank;
  // one rank needs no communicator; DMT_COMM_FORCE=1 makes one anyway, so that the RCCL
  // all-gather path can be exercised on a single GPU (tests/test_multirank.py)
  if (nranks == 1 && !std::getenv("DMT_COMM_FORCE")) return DMT_OK;
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  if (ncclCommInitRank(&h->comm, nranks, uid, rank) != ncclSuccess)
    return fail(DMT_ERR_COMM, "ncclCommInitRank failed");
  return DMT_OK;
}

dmt_status dmt_comm_size(dmt_ens* h, int32_t* nranks) {
  DMT_TRY(enter(h));
  if (!nranks) return fail(DMT_ERR_INVALID, "null argument");
  if (!h->comm) {
    *nranks = 1;
    return DMT_OK;
  }
  int n = 0;
  if (ncclCommCount(h->comm, &n) != ncclSuccess) return fail(DMT_ERR_COMM, "ncclCommCount failed");
  *nranks = n;
  return DMT_OK;
}

dmt_status dmt_set_service(dmt_ens* h, int32_t enable, double idle_ms) {
  DMT_TRY(check_h(h));
  if (!(idle_ms >= 0.0) || idle_ms > 60000.0) return fail(DMT_ERR_INVALID, "idle_ms outside [0, 60000]");
  DMT_TRY(svc_stop(h));
  h->service = enable != 0 && idle_ms > 0.0;
  if (idle_ms > 0.0) h->svc_idle_ms = idle_ms;
  h->svc_stats.off = 0;
  h->svc_stats.posts0 = h->svc_stats.posts;  // the self-disable rule counts from here
  h->svc_stats.relaunches0 = h->svc_stats.relaunches;
  return DMT_OK;
}

dmt_status dmt_service_stats(dmt_ens* h, uint64_t* stats) {
  DMT_TRY(check_h(h));
  if (!stats) return fail(DMT_ERR_INVALID, "null argument");
  stats[0] = h->svc_stats.starts;
  stats[1] = h->svc_stats.relaunches;
  stats[2] = h->svc_stats.posts;
  stats[3] = h->svc_stats.waits;
  stats[4] = h->svc_stats.off;
  return DMT_OK;
}

dmt_status dmt_combine_rank_partials(const double* all, int32_t nranks, int64_t n_iter,
                                     double* out) {
  if (!all || !out) return fail(DMT_ERR_INVALID, "null argument");
  if (nranks < 1 || n_iter < 0) return fail(DMT_ERR_INVALID, "nranks < 1 or n_iter < 0");
  combine_rank_partials(all, nranks, n_iter, out);
  return DMT_OK;
}

dmt_status dmt_set_shard(dmt_ens* h, int64_t seg_base) {
  DMT_TRY(enter(h));
  if (seg_base < 0 || seg_base + h->G > (int64_t)UINT32_MAX)
    return fail(DMT_ERR_INVALID, "seg_base out of range");
  h->seg_base = (uint32_t)seg_base;
  return DMT_OK;
}

dmt_status dmt_sync(dmt_ens* h) {
  DMT_TRY(enter(h));
  HIP_OK(stream_wait(h));
  return DMT_OK;
}

dmt_status dmt_set_timing(dmt_ens* h, int32_t on) {
  DMT_TRY(enter(h));
  HIP_OK(stream_wait(h));
  drain_timing(h);
  for (int k = 0; k < DMT_K_COUNT; ++k) { h->t_ms[k] = 0; h->t_cnt[k] = 0; }
  h->timing = on < 0 ? 0xFFFFFFFFu : (uint32_t)on;
  // the events of the next timed launches are created here, not inside the caller's timed region
  // (hipEventCreate is a driver call; the bench times its K steps right after this)
  while (h->timing && h->free_events.size() < 16) {
    hipEvent_t e;
    HIP_OK(hipEventCreateWithFlags(&e, h->event_flags));
    h->free_events.push_back(e);
  }
  return DMT_OK;
}

dmt_status dmt_get_timing(dmt_ens* h, int32_t kernel, double* ms, int64_t* count) {
  DMT_TRY(enter(h));
  if (kernel < 0 || kernel >= DMT_K_COUNT) return fail(DMT_ERR_INVALID, "bad kernel id");
  HIP_OK(stream_wait(h));
  drain_timing(h);
  if (ms) *ms = h->t_ms[kernel];
  if (count) *count = h->t_cnt[kernel];
  return DMT_OK;
}

dmt_status dmt_memory_bytes(dmt_ens* h, int64_t* bytes) {
  if (!h || !bytes) return fail(DMT_ERR_INVALID, "null argument");
  *bytes = h->bytes;
  return DMT_OK;
}

dmt_status dmt_recent_kernels(char* buf, int64_t n) {
  if (!buf || n <= 0) return fail(DMT_ERR_INVALID, "null buffer");
  std::string out;
  const unsigned cnt = std::min<unsigned>(g_recent_n, kRecentKernels);
  for (unsigned i = 0; i < cnt; ++i) {
    const void* k = g_recent_k[(g_recent_n - 1 - i) % kRecentKernels];
    Dl_info info{};
    std::string name = "?";
    // a kernel's host stub carries the kernel's mangled name (exported from libdmt.so)
    if (dladdr(k, &info) && info.dli_sname) {
      int st = 0;
      char* dm = abi::__cxa_demangle(info.dli_sname, nullptr, nullptr, &st);
      name = (st == 0 && dm) ? dm : info.dli_sname;
      std::free(dm);
    }
    out += name;
    out += '\n';
  }
  const size_t m = std::min<size_t>(out.size(), (size_t)n - 1);
  std::memcpy(buf, out.data(), m);
  buf[m] = '\0';
  return DMT_OK;
}

dmt_status dmt_debug_philox(int32_t device, uint64_t seed, const uint32_t* ctr, int64_t n,
                            uint32_t* out) {
  if (!ctr || !out || n < 0) return fail(DMT_ERR_INVALID, "bad args");
  HIP_OK(hipSetDevice(device));
  uint32_t *dc, *dout;
  double* dn;
  HIP_OK(dalloc(&dc, 4 * n));
  HIP_OK(dalloc(&dout, 4 * n));
  HIP_OK(dalloc(&dn, 2 * n));
  HIP_OK(hipMemcpy(dc, ctr, n * 16, hipMemcpyHostToDevice));
  HIP_OK(launch_debug_philox(seed, dc, n, dout, dn, nullptr));
  HIP_OK(hipMemcpy(out, dout, n * 16, hipMemcpyDeviceToHost));
  (void)hipFree(dc); (void)hipFree(dout); (void)hipFree(dn);
  return DMT_OK;
}

dmt_status dmt_debug_normals(int32_t device, uint64_t seed, const uint32_t* ctr, int64_t n,
                             double* out) {
  if (!ctr || !out || n < 0) return fail(DMT_ERR_INVALID, "bad args");
  HIP_OK(hipSetDevice(device));
  uint32_t *dc, *dout;
  double* dn;
  HIP_OK(dalloc(&dc, 4 * n));
  HIP_OK(dalloc(&dout, 4 * n));
  HIP_OK(dalloc(&dn, 2 * n));
  HIP_OK(hipMemcpy(dc, ctr, n * 16, hipMemcpyHostToDevice));
  HIP_OK(launch_debug_philox(seed, dc, n, dout, dn, nullptr));
  HIP_OK(hipMemcpy(out, dn, n * 16, hipMemcpyDeviceToHost));
  (void)hipFree(dc); (void)hipFree(dout); (void)hipFree(dn);
  return DMT_OK;
}


// ---------------------------------------------------------------- path snapshots (§8(f) rank 4)
// The tutorials keep every k-th accepted path, `append!(paths, [deepcopy(bb.b.XX)])`
// (docs/src/tutorials/biblock/smoothing.md:55, block_ensemble/inference.md:124).  Here the
// copies stay in HBM (a ring of slots, reference layout, fp64), are taken on the handle's
// stream without a host round trip, and are written to disk in one pass when wanted.

dmt_status dmt_snapshot_reserve(dmt_ens* h, int32_t what_mask, int64_t n_slots) {
  DMT_TRY(enter(h));
  if (what_mask < 1 || what_mask > 3 || n_slots < 1)
    return fail(DMT_ERR_INVALID, "what_mask must be 1 (XX), 2 (WW) or 3, n_slots >= 1");
  HIP_OK(stream_wait(h));
  const int C[2] = {h->d, h->m};
  for (int k = 0; k < 2; ++k) {
    if (h->d_snap[k]) {
      (void)hipFree(h->d_snap[k]);
      h->bytes -= h->snap_slots * h->P * C[k] * 8;
      h->d_snap[k] = nullptr;
    }
  }
  h->snap_mask = 0;
  h->snap_slots = 0;
  for (int k = 0; k < 2; ++k)
    if (what_mask >> k & 1) DMT_TRY(ens_alloc(h, &h->d_snap[k], n_slots * h->P * C[k]));
  h->snap_mask = what_mask;
  h->snap_slots = n_slots;
  h->snap_iter.assign(n_slots, -1);
  h->snap_unit.assign(n_slots, -1);
  return DMT_OK;
}

dmt_status dmt_snapshot_take(dmt_ens* h, int32_t unit, int64_t slot, int64_t mcmciter) {
  DMT_TRY(enter(h));
  if (unit != DMT_U && unit != DMT_UPROP) return fail(DMT_ERR_INVALID, "bad unit");
  if (!h->snap_mask) return fail(DMT_ERR_STATE, "no snapshot slots (dmt_snapshot_reserve)");
  if (slot < 0 || slot >= h->snap_slots) return fail(DMT_ERR_INVALID, "slot out of range");
  for (int k = 0; k < 2; ++k) {
    if (!(h->snap_mask >> k & 1)) continue;
    const int C = k == 0 ? h->d : h->m;
    double* dst = h->d_snap[k] + slot * h->P * C;
    void** src = k == 0 ? h->d_X : h->d_W;
    if (k == 0)
      HIP_OK(launch_from_planes(h->key.precision, h->tw, dst, src[0], src[1], h->d_sel[0], unit, C,
                                h->P, h->d_pt_off, h->G, h->d_seg_rec, h->d_seg_q, h->d_tile_qoff,
                                h->stream, src[2], 1, h->pk));
    else  // increments -> cumulative Wiener path, as dmt_download_paths
      HIP_OK(launch_from_planes_incr(h->key.precision, h->tw, dst, src[0], src[1], h->d_sel[1], unit,
                                     C, h->G, h->d_pt_off, h->d_seg_np, h->d_seg_rec, h->d_seg_q,
                                     h->d_tile_qoff, h->stream, src[2], 1, h->pk));
  }
  h->snap_iter[slot] = mcmciter;
  h->snap_unit[slot] = unit;
  return DMT_OK;
}

dmt_status dmt_snapshot_download(dmt_ens* h, int32_t what, int64_t slot, double* out,
                                 int64_t* mcmciter) {
  DMT_TRY(enter(h));
  if ((what != 0 && what != 1) || !out) return fail(DMT_ERR_INVALID, "bad what/out");
  if (!(h->snap_mask >> what & 1)) return fail(DMT_ERR_STATE, "that path kind is not snapshotted");
  if (slot < 0 || slot >= h->snap_slots) return fail(DMT_ERR_INVALID, "slot out of range");
  const int C = what == 0 ? h->d : h->m;
  HIP_OK(hipMemcpyAsync(out, h->d_snap[what] + slot * h->P * C, h->P * C * 8,
                        hipMemcpyDeviceToHost, h->stream));
  HIP_OK(stream_wait(h));
  if (mcmciter) *mcmciter = h->snap_iter[slot];
  return DMT_OK;
}

dmt_status dmt_snapshot_write(dmt_ens* h, const char* path, int64_t s0, int64_t s1) {
  DMT_TRY(enter(h));
  if (!path) return fail(DMT_ERR_INVALID, "null path");
  if (!h->snap_mask) return fail(DMT_ERR_STATE, "no snapshot slots (dmt_snapshot_reserve)");
  if (s0 < 0 || s1 > h->snap_slots || s0 > s1) return fail(DMT_ERR_INVALID, "bad slot range");
  if (!h->have_t) return fail(DMT_ERR_STATE, "time grid not uploaded");
  // the grid in reference layout (one recording's points when shared)
  const int64_t nt = h->grid_shared ? h->Q0 : h->P;
  std::vector<double> t(nt);
  DMT_TRY(ensure_stage(h, nt));
  if (h->grid_shared)
    HIP_OK(launch_cast_back(h->key.precision, h->d_t, h->d_stage, nt, h->stream));
  else
    HIP_OK(launch_from_planes(h->key.precision, h->tw, h->d_stage, h->d_t, h->d_t, h->d_sel[0], 0,
                              1, h->P, h->d_pt_off, h->G, h->d_seg_rec, h->d_seg_q, h->d_tile_qoff,
                              h->stream));
  HIP_OK(hipMemcpyAsync(t.data(), h->d_stage, nt * 8, hipMemcpyDeviceToHost, h->stream));
  HIP_OK(stream_wait(h));
  std::FILE* f = std::fopen(path, "wb");
  if (!f) return fail(DMT_ERR_INVALID, std::string("cannot open ") + path);
  dmt_snapshot_header hd{};
  std::memcpy(hd.magic, "DMTPATH1", 8);
  hd.version = 1;
  hd.what_mask = (uint32_t)h->snap_mask;
  hd.d = h->d;
  hd.m = h->m;
  hd.grid_shared = h->grid_shared;
  hd.precision = h->key.precision;
  hd.n_recordings = h->R;
  hd.n_segments = h->G;
  hd.n_points = h->P;
  hd.n_t = nt;
  hd.n_slots = s1 - s0;
  hd.seg_base = h->seg_base;
  std::vector<int32_t> nseg(h->R);
  for (int64_t r = 0; r < h->R; ++r) nseg[r] = (int32_t)(h->rec_seg0[r + 1] - h->rec_seg0[r]);
  bool ok = std::fwrite(&hd, sizeof hd, 1, f) == 1 &&
            std::fwrite(nseg.data(), 4, h->R, f) == (size_t)h->R &&
            std::fwrite(h->seg_np.data(), 4, h->G, f) == (size_t)h->G &&
            std::fwrite(t.data(), 8, nt, f) == (size_t)nt;
  // slots stream through two pinned buffers: the copy of piece k+1 overlaps the write of piece k
  const int64_t piece = std::min<int64_t>(int64_t(8) << 20, std::max<int64_t>(h->P * 3, 1));  // doubles
  double* pin[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  for (int b = 0; b < 2 && ok; ++b) {
    ok = hipHostMalloc((void**)&pin[b], piece * 8, hipHostMallocDefault) == hipSuccess &&
         hipEventCreateWithFlags(&ev[b], hipEventDisableTiming) == hipSuccess;
  }
  struct Src { const double* p; int64_t n; };
  std::vector<Src> pieces;
  for (int64_t s = s0; s < s1 && ok; ++s) {
    for (int k = 0; k < 2; ++k) {
      if (!(h->snap_mask >> k & 1)) continue;
      const int64_t n = h->P * (k == 0 ? h->d : h->m);
      const double* base = h->d_snap[k] + s * n;
      for (int64_t o = 0; o < n; o += piece) pieces.push_back({base + o, std::min(piece, n - o)});
    }
  }
  // per slot: int64 mcmciter, int64 unit, then X (and/or W); the 16-byte slot header is
  // written before the slot's first piece
  std::vector<int64_t> first_piece_of_slot;
  {
    int64_t k = 0;
    for (int64_t s = s0; s < s1; ++s) {
      first_piece_of_slot.push_back(k);
      for (int kk = 0; kk < 2; ++kk)
        if (h->snap_mask >> kk & 1) {
          const int64_t n = h->P * (kk == 0 ? h->d : h->m);
          k += (n + piece - 1) / piece;
        }
    }
  }
  auto issue = [&](size_t k) -> bool {
    const int b = (int)(k & 1);
    return hipMemcpyAsync(pin[b], pieces[k].p, pieces[k].n * 8, hipMemcpyDeviceToHost, h->stream) ==
               hipSuccess &&
           hipEventRecord(ev[b], h->stream) == hipSuccess;
  };
  if (ok && !pieces.empty()) ok = issue(0);
  size_t slot_i = 0;
  for (size_t k = 0; k < pieces.size() && ok; ++k) {
    const int b = (int)(k & 1);
    ok = hipEventSynchronize(ev[b]) == hipSuccess;
    if (ok && k + 1 < pieces.size()) ok = issue(k + 1);
    if (ok && slot_i < first_piece_of_slot.size() && (int64_t)k == first_piece_of_slot[slot_i]) {
      const int64_t s = s0 + (int64_t)slot_i;
      const int64_t sh[2] = {h->snap_iter[s], h->snap_unit[s]};
      ok = std::fwrite(sh, 8, 2, f) == 2;
      ++slot_i;
    }
    if (ok) ok = std::fwrite(pin[b], 8, pieces[k].n, f) == (size_t)pieces[k].n;
  }
  (void)stream_wait(h);
  for (int b = 0; b < 2; ++b) {
    if (pin[b]) (void)hipHostFree(pin[b]);
    if (ev[b]) (void)hipEventDestroy(ev[b]);
  }
  if (std::fclose(f) != 0) ok = false;
  if (!ok) return fail(DMT_ERR_HIP, std::string("writing ") + path + " failed");
  return DMT_OK;
}

}  // extern "C"
