// dmt_internal.h — structures shared by the host runtime and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dmt {

constexpr int kLanes = 64;  // one recording per lane of a wave64 ("recording tile")
// spare point rows at the end of every tile (and of shared tables): the software
// prefetch reads up to 2*kChunk points past a segment end without bounds checks
constexpr int kPadPoints = 32;
// MAP_AUTO picks MAP_WAVE up to this many recordings (see DESIGN.md §2 for the measurement)
constexpr int64_t kAutoWaveMaxRecordings = 8192;

// Kernel modes of the per-block recursion kernel.
enum Mode : int {
  MODE_PCN = 0,        // draw_proposal_path!: pCN-mixed W°, proposal written to u°
  MODE_RECOMPUTE = 1,  // recompute_path!(b°, b.WW): given W, law u°.PP
  MODE_FRESH = 2,      // draw_proposal_path!(u::SamplingUnit): fresh W (ρ = 0), in place
};

// Path selectors (selX, selW; one byte per segment): bits 0-1 = the physical buffer holding
// u.XX[g] (u.WW[g]), bits 2-3 = the buffer holding u°'s.  A swap exchanges the two fields.
// Ensembles with two buffers keep u° = u ^ 1 (sel_two); MAP_LANE ensembles of non-linear models
// hold a third, and a draw writes every proposal of a wave to a buffer that holds none of the
// wave's u paths ("path buffers").  Law selectors (selPP, selPPB) stay 0/1 with
// the other slot implied.
__host__ __device__ __forceinline__ int sel_u(unsigned s) { return (int)(s & 3u); }
__host__ __device__ __forceinline__ int sel_p(unsigned s) { return (int)((s >> 2) & 3u); }
__host__ __device__ __forceinline__ int sel_buf(unsigned s, int flip) {  // flip: 0 u, 1 u°
  return flip ? sel_p(s) : sel_u(s);
}
__host__ __device__ __forceinline__ uint8_t sel_make(int u, int p) { return (uint8_t)(u | (p << 2)); }
__host__ __device__ __forceinline__ uint8_t sel_swap(unsigned s) { return sel_make(sel_p(s), sel_u(s)); }
__host__ __device__ __forceinline__ uint8_t sel_two(int u) { return sel_make(u, u ^ 1); }
constexpr uint8_t kSelInit = 4;  // sel_two(0): u in buffer 0, u° in buffer 1

// Element index in a plane of tile width tw: component c of C of plane row `row` (= the tile's
// first row tile_qoff + the point's row q within its recording) for tile slot `slot`.
//   pk = 0: the row layout ((row·C + c)·tw + slot) — a wave's 64 lanes touch 64 consecutive
//           elements per component;
//   pk > 0 (a power of two; the path planes X, W of an fp32 MAP_LANE ensemble, DESIGN.md §2
//           "lane packets"): each slot's pk consecutive rows of one component are contiguous —
//           64-byte pieces, so a lane's path never shares a piece of memory with another lane's
//           and per-lane MH decisions (each lane's u in its own buffer) cost no partial writes.
__host__ __device__ __forceinline__ int64_t plane_ix(int64_t row, int c, int C, int tw, int slot,
                                                      int pk) {
  if (pk == 0) return (row * C + c) * tw + slot;
  const int lg = __builtin_ctz((unsigned)pk);
  return (((row >> lg) * C + c) * tw + slot) * pk + (row & (pk - 1));
}
// lane-packet length of the path planes of an fp32 MAP_LANE ensemble: 32 points = 128 bytes, a
// whole cache line per lane and component, so a lane's stores never share a line with another
// lane's (round 6; 16 points = 64-byte pieces left every line shared by a lane pair, whose
// per-lane buffers differ after their MH decisions: partial lines, read-modify-write FETCH)
#ifndef DMT_PATH_PACKET
#define DMT_PATH_PACKET 32
#endif
constexpr int kPathPacket = DMT_PATH_PACKET;
// points a packet kernel stages in registers at a time (one 64-byte piece per component): the
// processing unit of k_block_pk / k_block_ps_pk, a divisor of kPathPacket
constexpr int kPkChunkPts = 16;
static_assert(kPathPacket % kPkChunkPts == 0, "whole register-staged pieces per lane packet");

// Thread mappings of the recursion (chosen per ensemble at dmt_create):
//   MAP_LANE: one lane per (recording, block); tile width tw = 64 recordings
//   MAP_WAVE: one wavefront per block, 64 consecutive steps per chunk; tw = 1
enum Mapping : int { MAP_AUTO = 0, MAP_LANE = 1, MAP_WAVE = 2 };

// Arguments of the block kernels.  Device-path arrays are "recording-tile planes" of tile
// width tw: element (recording r, point q of r, component c) of an array with C components
// lives at   ((tile_qoff[r/tw] + q) * C + c) * tw + r%tw.
// tw = 64 (MAP_LANE): the 64 lanes of a wave (64 recordings of one tile, same block index)
// touch 64 consecutive elements per component — one coalesced 512 B (fp64) access.
// tw = 1 (MAP_WAVE): recording-major, point-major, components interleaved (the reference's
// own Vector{SVector{d}} layout) — a wave's 64 lanes touch 64 consecutive points.
// Per-block record of a layout, precomputed on the host (one scalar load per block).
struct BlkInfo {
  int64_t tq;      // first point row of the block's recording tile
  int32_t g0, g1;  // global first / last segment
  int32_t ktot;    // chunks of 64 steps over the block's segments
  int32_t term;    // terminal block (BiBlock{true})
  int32_t np0;     // points of the first segment
  int32_t q0;      // seg_q of the first segment
  int32_t kfirst;  // chunks of the first segment
  int32_t pad_;
  double rho, srho;
};

template <class T>
struct BlockArgs {
  const BlkInfo* binfo;  // [nblocks] of the layout
  int64_t R;
  const int64_t* tile_qoff;  // [ntiles + 1]
  const int32_t* seg_q;      // [G] first point of the segment within its recording
  const int32_t* seg_np;     // [G] points of the segment
  const int64_t* st_off;     // [G] first step of the segment in reference (Z) order
  uint8_t* selX;             // [G] path selectors (sel_u / sel_p above; the lane kernel
                             // re-points them when it moves a path or picks u°'s buffer)
  uint8_t* selW;
  const uint8_t* selPP;
  const uint8_t* selPPB;
  T* X[3];                   // X[2], W[2]: the third path buffers (nullptr: two-buffer ensemble)
  T* W[3];
  int nbuf;                  // path buffers per container (2 or 3)
  int pk;                    // path planes in lane packets of pk points (0: row layout; plane_ix)
  int full_copy;             // consolidation rewrites every lane's u (whole lines; DMT_FULL_COPY)
  const T* t;
  int t_shared;
  const T* sdt;  // shared grid: sqrt(t[q+1] − t[q]) per point in T (dmt_upload_grid), else nullptr
  const T* H[2][2];  // [slot][kind]
  int H_shared[2][2];
  const T* F[2][2];
  const double* law[2][2];
  const T* aux[2];  // [kind] per-point B̃(t_i), β̃(t_i) (dmt_upload_aux), nullptr: none
  int64_t aux_n;    // elements of each aux table (the bounds the DMT_AUX_CHECK build checks)
  // layout
  const int64_t* blk_off;  // [R + 1]
  const int32_t* blk_rec;  // [nblocks] recording of each block
  const int32_t* gfirst;   // [nblocks] global segment ids
  const int32_t* glast;
  const uint8_t* term;
  const double* rho;
  const double* srho;
  int32_t MB;     // max blocks per recording in the layout
  int64_t tile0, tile1;
  int64_t b0, b1;
  // unit selection (xor-ed with the selectors)
  int law_flip, xs_flip, xd_flip, ws_flip, wd_flip;
  const double* Z;  // parity mode normals, reference step order, or nullptr
  uint64_t seed;
  uint32_t iter, salt;
  uint32_t seg_base;  // global id of local segment 0 (RNG streams; dmt_set_shard)
  double* ll_out;     // [nblocks]
  uint8_t* success;   // [nblocks] or nullptr
  int repair_div;     // MAP_LANE draws: consolidate a wave's u paths while the lanes outside the
  int repair_min;     // majority's buffer are <= 1/repair_div of it and >= repair_min (path_plan)
  int resident1;      // linear drift, layout of single-segment blocks of <= kResidentMaxSteps
                      // steps: one-shot draws on k_block_resident
  int lane_split;     // MAP_LANE draws: producer/consumer waves (k_block_ps); the runtime sets
                      // it only for layouts of single-segment blocks
  int lane_pair;      // MAP_LANE device-RNG draws: two lanes per recording (k_block_pair)
  int ll_skip;        // MODE_RECOMPUTE: the last ll_skip steps of every segment add no Girsanov
                      // term (recompute_path!(…; skip), GP.solve_and_ll!(…; skip))
};

struct AcceptArgs {
  int64_t b0, b1, nblocks;
  const int32_t* gfirst;
  const int32_t* glast;
  uint8_t* selX;
  uint8_t* selW;
  double* ll;
  double* llp;
  double* ll_hist;
  double* llp_hist;
  uint8_t* acc_hist;
  int64_t hist_len;
  int64_t mcmciter;  // 1-based (history index)
  const double* E;   // [b1-b0] or nullptr
  uint64_t seed;
  uint32_t salt;
  uint32_t key_iter;  // iteration word of the Exp(1) stream key (= mcmciter unless DMT_RNG_AUTO)
  int64_t key_delta;  // persistent runs: iteration it draws with key word it + key_delta
  uint32_t seg_base;
  uint8_t* acc_out;  // [b1-b0] or nullptr
};

// The resident MCMC service (include/dmt.h "deferred draws"): a launch of the
// register-resident producer/consumer kernel that runs the iterations the host posts one at a
// time, keeping every block's state in registers between the caller's separate calls.
struct SvcArgs {
  const uint64_t* posted;  // host memory: iterations posted so far (written by the host)
  const uint32_t* stop;    // host memory: 1 = leave at the next gate
  uint64_t* rec;           // host memory: [2][grid][4] 16-byte records (sum bits, sum bits ^
                           //   svc_mix(iteration + 1))
                           //   of every workgroup's (ll, ll°, accepted) sums, by iteration parity
  uint64_t* go;            // device: workgroup 0's answers to the other workgroups' gates —
  uint64_t* quit;          //   go / quit = base + r + 1 at gate r (zeroed before every launch)
  uint64_t idle_ticks;     // wall-clock ticks a waiting launch stays without a command
  uint64_t* probe;         // DMT_SVC_PROBE builds only: [capacity][8] wall-clock stamps
  uint64_t base;           // the launch's iteration r is the service's iteration base + r (a
                           // launch that left idle is re-launched from where it stopped)
};

// Check word of a service record (svc_record / svc_slot_ready): a record is (value bits,
// value bits ^ svc_mix(tag)).  The host accepts a record only when its two words agree for the
// tag it waits for, so a read that sees one word of the 16-byte store and not the other (no
// API promises that a 16-byte write to host memory is seen whole) is rejected and read again;
// a record of an older iteration never agrees with a newer tag.  splitmix64's finaliser.
__host__ __device__ __forceinline__ uint64_t svc_mix(uint64_t tag) {
  uint64_t z = tag + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Timing events attached to the next kernel dispatch (hipExtLaunchKernel): armed by the
// runtime for a timed launch, consumed (and cleared) by that kernel's launcher.
struct DispatchEvents {
  hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local DispatchEvents g_dispatch_events;
// the host stubs of the last kRecentKernels kernels this thread launched (dlaunch), most recent
// at g_recent_n - 1 (mod kRecentKernels): dmt_recent_kernels names them, so a caller (bench.py)
// can tell which kernel a call dispatched instead of restating the runtime's choice
constexpr int kRecentKernels = 8;
extern thread_local const void* g_recent_k[kRecentKernels];
extern thread_local unsigned g_recent_n;

// recompute_guiding_term! on the device (k_backward_filter): one thread per block.
struct FilterArgs {
  int d, tw, unit;
  const int64_t* tile_qoff;
  const int32_t* seg_rec;
  const int32_t* seg_q;
  const int32_t* seg_np;
  const int32_t* gfirst;
  const int32_t* glast;
  const uint8_t* term;
  const uint8_t* selPP;
  const uint8_t* selPPB;
  int64_t b0, b1;
  void* H[2][2];  // [slot][kind] per-point tables (T)
  void* F[2][2];
  double* law[2][2];
  const void* t;  // grid (T)
  int t_shared;
  const void* aux[2];  // [kind] per-point B̃(t_i), β̃(t_i) (T), nullptr: none
  const double* obsH;  // [G][hp] information of the observation at each segment's end
  const double* obsF;  // [G][d]
  const double* obsc;  // [G]
  const double* obsv;  // [G][d] artificial observation (set_obs!) of a P_last segment
  double art_eps;      // its variance (artificial_noise)
  int* fail;           // set to 1 if a filter step is singular
  const uint8_t* only;  // [nblocks] nullable: filter only the blocks flagged here
  // chunked filter (guiding term): one batch of blocks [b0, b1) covering segments [gA, gB]
  const int64_t* pt_off;      // [G] first point of each segment
  const int64_t* fchunk_off;  // [G + 1] prefix of the segments' chunk counts
  uint8_t* segsel;            // [G] 0 skip, 1 PP, 2 PPb (k_filter_mark)
  double* qbuf;               // [kFiltNQ(d)][qcap] composed transitions, point p at p − pA
  int64_t qcap, pA;
  int32_t gA, gB;
  int64_t fchunk_off_h0, fchunk_off_h1;  // fchunk_off[gA], fchunk_off[gB + 1] (host copies)
  int fused;  // many blocks: k_filter_fused (a wave per block, no scratch) instead of scan + chain
  double* tbuf;  // [items][hp + d + 1] guiding term at each chunk end (k_filter_chain → _points)
};
constexpr int kFiltNQ(int d) { return d * d + d + d * (d + 1) / 2; }

// set_proposal_law! on the device (k_set_prop_law): one thread per block.
constexpr int kMaxParams = 16;
struct ParamArgs {
  int model, d, m, n;
  int32_t idx[kMaxParams];
  double val[kMaxParams];
  const int32_t* gfirst;
  const int32_t* glast;
  const uint8_t* term;
  const uint8_t* selPP;
  const uint8_t* selPPB;
  double* law[2][2];  // [slot][kind]; law[·][1] null without PPb records
  int64_t b0, b1;
  uint8_t* crit;    // [nblocks] 1 if the block's auxiliary law (as the filter uses it) changed
  uint32_t* ncrit;  // count of such blocks
  int cc_mode;      // critical_change (src/biblock.jl:340-342): -1 a block is critical when its
                    // auxiliary law changed; 0 (false) only when equalizing u°'s law with u's
                    // changed it; 1 (true) every block
};

// Model/precision dispatch keys.
struct ModelKey {
  int model, precision, d, m;
};

// launchers (dmt_kernels.hip)
hipError_t launch_block_kernel(const ModelKey& k, int mapping, int mode, const void* args,
                               int64_t nwaves, hipStream_t s);
hipError_t launch_invsolve_kernel(const ModelKey& k, int mapping, const void* args,
                                  int64_t nwaves, hipStream_t s);
hipError_t launch_pathll_kernel(const ModelKey& k, int mapping, const void* args, int64_t nwaves,
                                hipStream_t s);
hipError_t launch_accept(const AcceptArgs& a, hipStream_t s);
// dmt_mcmc_run for linear drifts: n_iter iterations in one launch (k_mcmc_scan), per-iteration
// (ll, ll°, accepted) partials to part[n_iter][3][nwaves]; then their fetch_ll trees
// (resident: every block is one segment of ≤ kResidentMaxSteps steps and d ≤ 2 —
// k_mcmc_resident keeps the block's state in registers for the whole run)
constexpr int kPersistMaxSegments = 64;
// points per batch of the chunked device filter (its transition scratch: kFiltNQ(d) doubles each)
constexpr int64_t kFiltBatchPoints = int64_t(1) << 24;
// block counts from which the device filter runs k_filter_fused (one wave per block) instead of
// k_filter_scan + k_filter_chain (every chunk in parallel, a short serial chain per block)
constexpr int64_t kFiltFusedBlocks = 4096;
constexpr int kResidentMaxSteps = 512;
// part: [n_iter][3][nwaves] block partials followed by the tree nodes ([3 n_iter][ceil(nwaves /
// WPB)] then [3 n_iter][ceil(nwaves / (16 WPB))], WPB ≤ 4); out3[n_iter][3]: every iteration's
// fetch_ll; counter: ceil(nwaves / (16 WPB)) + 1 zeroed uint32 arrival counters (left zero)
hipError_t launch_mcmc_service(const ModelKey& k, const void* args, const AcceptArgs& c,
                               int64_t iter0, int64_t capacity, double* part, int64_t nwaves,
                               int producers, int n_cu, const SvcArgs& sv, hipStream_t s);
bool mcmc_service_fits(const ModelKey& k, int64_t nwaves, int producers, int n_cu);
hipError_t launch_mcmc_persistent(const ModelKey& k, const void* args, const AcceptArgs& c,
                                  int64_t iter0, int64_t n_iter, double* part, int64_t nwaves,
                                  int resident, double* out3, unsigned* counter, hipStream_t s);
hipError_t launch_backward_filter(int precision, const FilterArgs& a, hipStream_t s);
hipError_t launch_set_prop_law(const ParamArgs& a, hipStream_t s);
hipError_t launch_set_obs(int precision, int tw, int pk, int d, const void* X0, const void* X1,
                          const void* X2, const uint8_t* selX,
                          const int64_t* tile_qoff, const int32_t* seg_rec, const int32_t* seg_q,
                          const int32_t* seg_np, const int32_t* glast, const uint8_t* term,
                          int64_t b0, int64_t b1, double* obsv, int model, double* lawb0,
                          double* lawb1, hipStream_t s);
hipError_t launch_to_planes(int precision, int tw, const double* src, void* dst0, void* dst1,
                            const uint8_t* sel, int flip, int C, int64_t P, const int64_t* pt_off,
                            int64_t G, const int32_t* seg_rec, const int32_t* seg_q,
                            const int64_t* tile_qoff, hipStream_t s, int incr = 0,
                            void* dst2 = nullptr, int enc = 0, int pk = 0);
hipError_t launch_from_planes_incr(int precision, int tw, double* dst, const void* src0,
                                   const void* src1, const uint8_t* sel, int flip, int C,
                                   int64_t G, const int64_t* pt_off, const int32_t* seg_np,
                                   const int32_t* seg_rec, const int32_t* seg_q,
                                   const int64_t* tile_qoff, hipStream_t s,
                                   const void* src2 = nullptr, int enc = 0, int pk = 0);
hipError_t launch_from_planes(int precision, int tw, double* dst, const void* src0,
                              const void* src1, const uint8_t* sel, int flip, int C, int64_t P,
                              const int64_t* pt_off, int64_t G, const int32_t* seg_rec,
                              const int32_t* seg_q, const int64_t* tile_qoff, hipStream_t s,
                              const void* src2 = nullptr, int enc = 0, int pk = 0);
hipError_t launch_cast(int precision, const double* src, void* dst, int64_t n, hipStream_t s);
hipError_t launch_cast_back(int precision, const void* src, double* dst, int64_t n, hipStream_t s);
hipError_t launch_block_sum(const double* ll, const double* llp, const uint8_t* acc, int64_t n,
                            double* work, double* out3, hipStream_t s);
// work: multi-level tree scratch (6 per 1024-block group); lb: single-launch scratch
// (3 x 256 partials + a counter, zero-initialised once)
hipError_t launch_accept_reduce(const AcceptArgs& a, double* work, double* lb, double* out3,
                                hipStream_t s);
hipError_t launch_flip(uint8_t* sel0, uint8_t* sel1, uint8_t* sel2, uint8_t* sel3,
                       const int32_t* gfirst, const int32_t* glast, const uint8_t* term,
                       int32_t swap_ppb_nonterm_only, int64_t b0, int64_t b1, hipStream_t s);
hipError_t launch_swap_ll(double* ll, double* llp, int64_t b0, int64_t b1, hipStream_t s);
hipError_t launch_save_ll(const double* ll, const double* llp, double* llh, double* llph,
                          int64_t nblocks, int64_t it0, int64_t b0, int64_t b1, hipStream_t s);
hipError_t launch_debug_philox(uint64_t seed, const uint32_t* ctr, int64_t n, uint32_t* out,
                               double* normals, hipStream_t s);

}  // namespace dmt
