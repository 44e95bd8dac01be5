// picp_vo_runtime.cpp -- host side of the device-resident VO sequence (picp_vo.hip), C-ABI in
// include/picp_c.h (picp_vo_*).
//
// A handle owns one packed observation sequence in HBM (frame offsets, uv, descriptors) and,
// after picp_vo_set_segments, everything a run needs: per-segment maps, the PICP SoA planes,
// problem tables and states, match outputs, poses and step records.  A run is
//   1 (or ceil(frames/65535)) launch(es) matching every frame f against f+1,
//   1 bootstrap append, then per step: world match, gather, picp_block_kernel, append,
// enqueued back to back on the handle's stream and captured once into a hipGraph that is
// replayed by every later run.  No host round trip inside a run; no host fallback.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <utility>
#include <vector>

#include "picp_c.h"
#include "picp_host.h"
#include "picp_internal.h"

extern "C" hipError_t picp_launch_block(hipStream_t stream, int n_problems, int npt, const float* X,
                                        const float* Y, const float* Z, const float* U,
                                        const float* V, const PicpArgs* args,
                                        const PicpProblem* probs, const PicpState* st_in,
                                        PicpState* st_out, int max_n, int split,
                                        unsigned long long* xg, unsigned int* err,
                                        unsigned int* tagbase, unsigned long long timeout_ticks);
extern "C" hipError_t picp_launch_vo_gather(hipStream_t stream, const VoArgs* a, int t);
extern "C" int picp_vo_block_fusable(int npt, int64_t max_obs);
extern "C" int picp_build_packed_fp32(void);
extern "C" hipError_t picp_launch_vo_block(hipStream_t stream, const VoArgs* a, int t, int npt,
                                           const PicpArgs* args, int64_t max_obs);
extern "C" hipError_t picp_launch_vo_append(hipStream_t stream, const VoArgs* a, int t);

static_assert(sizeof(picp_vo_step) == sizeof(VoStep), "picp_vo_step must mirror VoStep");

#define VO_MATCH_DIST 0.2f   // DISTANCE_THRESHOLD, src/my_utilities.h:44
#define VO_MATCH_RATIO 0.8f  // RATIO_THRESHOLD, src/my_utilities.h:46
#define VO_MAX_GRID_Y 65535

// Diagnostic (PICP_VO_GUARD=1, read at create): every device buffer of the handle gets a
// VO_GUARD-byte pattern-filled pad before and after it; picp_vo_debug_guard counts pad bytes that
// no longer hold the pattern (an out-of-bounds store into or out of the buffer).
#define VO_GUARD (1 << 20)
#define VO_GUARD_BYTE 0xA5
struct VoGuarded {
  char* base;
  size_t bytes;
  const char* name;
};

struct picp_vo {
  int device = 0;
  hipStream_t stream = nullptr;
  int rows = 0, cols = 0, dim = 0;
  float K[9];
  int64_t n_frames = 0, n_obs = 0, max_obs = 0;
  std::vector<int64_t> frame_off;
  // sequence, resident
  int64_t* frame_off_d = nullptr;
  float2* uv_d = nullptr;
  float* desc_d = nullptr;
  int32_t *pm_bi = nullptr, *pm_acc = nullptr, *wm_bi = nullptr, *wm_acc = nullptr;
  float *pm_bd = nullptr, *pm_sd = nullptr, *wm_bd = nullptr, *wm_sd = nullptr;
  int dp = 16;                     // matcher prep row width (halves)
  _Float16* obs_h = nullptr;       // matcher prep of the observations
  float *obs_n1 = nullptr, *obs_n2 = nullptr;
  // segments
  int n_seg = 0, max_steps = 0, npt = 1;
  int64_t map_slots = 0, n_slots = 0, cap_c = 0;
  std::vector<VoSegment> segs;
  std::vector<MatchProblem> pprobs;
  void* seg_mem = nullptr;  // one allocation for everything sized by the segments
  PicpArgs pargs;
  VoArgs vargs;
  MatchProblem* pprobs_d = nullptr;
  MatchProblem* wprobs_d = nullptr;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // The default is the concurrent schedule (overlap on, two chains), enqueued launch by launch:
  // a hipGraph replay keeps neither the streams' priorities nor the chains' phase offset
  // (DESIGN.md §4.9).  The serial order (PICP_VO_OVERLAP=0 PICP_VO_CHAINS=1) is captured once
  // into a hipGraph and replayed (PICP_VO_GRAPH=0: enqueued).  Every schedule gives the same bits.
  bool use_graph = true;
  bool graph_env = false;
  // the frame->next match in chunks by step index (chunk k = frame f0+k of every segment with
  // more than k steps), chunks 1.. on a side stream that runs beside the step chain
  std::vector<size_t> chunk_off;  // pprobs[chunk_off[k] .. chunk_off[k+1]) is chunk k
  bool overlap = true;            // PICP_VO_OVERLAP=0: every chunk on the main stream, up front
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr;
  std::vector<hipEvent_t> ev_chunk;
  // the segments in `chains` contiguous groups, each group's step chain on its own stream
  // (group 0 on the handle's stream): one group's latency-bound PICP block kernel runs beside
  // another group's throughput-bound world match.  Group c starts after group c-1's first world
  // match (PICP_VO_PHASE=0: together), so the groups run out of phase.
  int chains = 2;  // PICP_VO_CHAINS (1: one step chain, the serial order)
  int chains_eff = 1;  // chains for the current segments (1 when two groups would query one frame)
  bool phase = true;
  std::vector<hipStream_t> cstream;  // [chains], [0] unused (the handle's stream)
  std::vector<hipEvent_t> ev_cj;     // [chains]: group c's end (join), [0]: fork
  std::vector<hipEvent_t> ev_ph;     // [chains]: group c's first world match done
  int accept_only = 1;  // the sequence reads only accepted matches (PICP_VO_MATCH_FULL=1: full form)
  // the matcher's reference-range split (picp_match_ksplit) for launches of few problems: each
  // chain's world match has its own scratch (the chains run concurrently), the frame->next
  // launches one between them (they run in stream order: chunk 0, then the side stream's)
  // Every launch's split count is fixed at picp_vo_set_segments (PICP_MATCH_KSPLIT read once there)
  // and the scratch sized from the same counts: a launch never uses more ranges than its scratch holds.
  std::vector<int> ks_w;          // [chains]
  std::vector<float4*> part_w;    // [chains]
  std::vector<int64_t> cap_w;     // [chains]: part_w's capacity, float4
  std::vector<std::pair<size_t, int>> ks_p;  // frame->next launch starting at problem .first: split .second
  // The world match split by map age (PICP_VO_SPLIT=1; off by default: measured slower at every C5
  // shape -- 8e 44.5k -> 31.4-32.9k frames/s, the per-rank shape 162k -> 75-77k, the default shape
  // 797k -> 561k -- because the early parts, running beside the step chains for most of a step,
  // slow the chains' short kernels: the append 20 -> 40-106 us, the merge 6 -> 40 us
  // (profiles/r06/t13, t16, t17); neither a smaller early split nor CU-masked early queues helped).
  // Step t matches frame f0+t+1 against the map
  // after step t-1's append.  The map is append-only, so that is the EARLY part -- the map as step
  // t-2's append left it, which needs nothing from step t-1 and runs on the chain's early stream
  // beside step t-1 -- and the LATE part, the points step t-1's append added.  Only the late part
  // and the merge stay on the chain: the merge kernel folds the early ranges and then the late one,
  // the reference's in-order scan over the whole map (the late indices are the map's: idx0).
  int split_env = 0;                  // PICP_VO_SPLIT: 0 off (default), 1 every chain, -1 auto
  std::vector<char> split_c;          // [chains]
  std::vector<float4*> part_e;        // [chains][2]: early ranges + the late slot, by step parity
  std::vector<int64_t> cap_e;         // [chains]
  std::vector<int> ks_e;              // [chains]: the early part's range split (PICP_VO_EKS forces)
  std::vector<hipStream_t> estream;   // [chains]
  std::vector<hipEvent_t> ev_app;     // [chains]: the chain's latest merged match
  std::vector<hipEvent_t> ev_early;   // [chains][2]: the early part of step t done (by parity)
  float4* part_p = nullptr;
  int64_t cap_p = 0;
  // the step's gather runs inside the PICP block kernel (picp_launch_vo_block) when every frame's
  // items fit on-chip; PICP_VO_FUSE=0 keeps vo_gather_kernel + the plain block launch (A/B: the
  // same items in the same order, the same bits)
  // (the append fused after the rounds and a world match split into an early and a late part were
  // built in round 4, bit-identical, and measured slower: DESIGN.md §4.14, commit 1ffa87f)
  int fuse = 1;  // PICP_VO_FUSE: 0 separate gather, 1 gather in the PICP kernel
  bool guard = false;
  std::vector<VoGuarded> guards;
#ifdef PICP_VO_DIAG
  char* snap = nullptr;  // picp_vo_debug_snap_set: per-step copies of the PICP launch's inputs/outputs
#endif
};


static hipError_t vo_malloc(picp_vo* h, void** p, size_t bytes, const char* name) {
  if (!h->guard) return hipMalloc(p, bytes);
  char* base = nullptr;
  hipError_t e = hipMalloc((void**)&base, bytes + 2 * (size_t)VO_GUARD);
  if (e != hipSuccess) return e;
  e = hipMemset(base, VO_GUARD_BYTE, bytes + 2 * (size_t)VO_GUARD);
  if (e != hipSuccess) return e;
  h->guards.push_back(VoGuarded{base, bytes, name});
  *p = base + VO_GUARD;
  return hipSuccess;
}

static void vo_dfree(picp_vo* h, void* p) {
  if (!h->guard) {
    hipFree(p);
    return;
  }
  for (size_t i = 0; i < h->guards.size(); ++i)
    if (h->guards[i].base + VO_GUARD == (char*)p) {
      hipFree(h->guards[i].base);
      h->guards.erase(h->guards.begin() + (long)i);
      return;
    }
}

static void vo_free_segments(picp_vo* h) {
  if (h->exec) hipGraphExecDestroy(h->exec);
  if (h->graph) hipGraphDestroy(h->graph);
  h->exec = nullptr;
  h->graph = nullptr;
  for (hipEvent_t e : h->ev_chunk)
    if (e) hipEventDestroy(e);
  h->ev_chunk.clear();
  if (h->seg_mem) vo_dfree(h, h->seg_mem);
  h->seg_mem = nullptr;
  h->n_seg = 0;
}

extern "C" int picp_vo_destroy(picp_vo_t* h) {
  if (!h) return PICP_OK;
  if (h->stream) hipStreamSynchronize(h->stream);
  vo_free_segments(h);
  void* bufs[] = {h->frame_off_d, h->uv_d, h->desc_d, h->pm_bi, h->pm_acc, h->wm_bi, h->wm_acc,
                  h->pm_bd, h->pm_sd, h->wm_bd, h->wm_sd, h->obs_h, h->obs_n1, h->obs_n2};
  for (void* p : bufs)
    if (p) vo_dfree(h, p);
  if (h->ev0) hipEventDestroy(h->ev0);
  if (h->ev1) hipEventDestroy(h->ev1);
  if (h->ev_fork) hipEventDestroy(h->ev_fork);
  if (h->side) hipStreamDestroy(h->side);
  for (hipEvent_t e : h->ev_cj)
    if (e) hipEventDestroy(e);
  for (hipEvent_t e : h->ev_ph)
    if (e) hipEventDestroy(e);
  for (hipEvent_t e : h->ev_app)
    if (e) hipEventDestroy(e);
  for (hipEvent_t e : h->ev_early)
    if (e) hipEventDestroy(e);
  for (hipStream_t c : h->estream)
    if (c) hipStreamDestroy(c);
  for (hipStream_t c : h->cstream)
    if (c) hipStreamDestroy(c);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return PICP_OK;
}

extern "C" int picp_vo_create(picp_vo_t** out, int device, int rows, int cols, const float K[9],
                              int64_t n_frames, const int64_t* frame_off, const float* uv,
                              const float* desc, int dim) {
  CHECK_ARG(out, "picp_vo_create: null output");
  *out = nullptr;
  CHECK_ARG(K && frame_off && rows > 0 && cols > 0, "picp_vo_create: bad camera or frame table");
  CHECK_ARG(n_frames >= 2, "picp_vo_create: need at least two frames");
  CHECK_ARG(dim >= 1 && dim <= 32, "picp_vo_create: dim must be in [1, 32]");
  CHECK_ARG(frame_off[0] == 0, "picp_vo_create: frame_off[0] must be 0");
  int64_t mx = 0;
  for (int64_t f = 0; f < n_frames; ++f) {
    CHECK_ARG(frame_off[f + 1] >= frame_off[f], "picp_vo_create: frame_off must be non-decreasing");
    mx = std::max(mx, frame_off[f + 1] - frame_off[f]);
  }
  CHECK_ARG(mx <= (1 << 30), "picp_vo_create: frame too large");
  const int64_t n_obs = frame_off[n_frames];
  CHECK_ARG(n_obs == 0 || (uv && desc), "picp_vo_create: null observation arrays");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  CHECK_ARG(device >= 0 && device < ndev, "picp_vo_create: no such HIP device");
  HIP_TRY(hipSetDevice(device));
  picp_vo* h = new picp_vo();
  h->device = device;
  h->rows = rows;
  h->cols = cols;
  h->dim = dim;
  memcpy(h->K, K, sizeof(h->K));
  h->n_frames = n_frames;
  h->n_obs = n_obs;
  h->max_obs = mx;
  h->frame_off.assign(frame_off, frame_off + n_frames + 1);
  if (const char* e = getenv("PICP_VO_GRAPH")) {
    h->use_graph = atoi(e) != 0;
    h->graph_env = true;
  }
  if (const char* e = getenv("PICP_VO_MATCH_FULL")) h->accept_only = atoi(e) != 0 ? 0 : 1;
  // A/B libraries built with packed FP32 (make PK=1): their concurrent schedules are not
  // bit-stable, so such a build defaults to the serial order and says so
  if (picp_build_packed_fp32()) {
    h->overlap = false;
    h->chains = 1;
    fprintf(stderr, "picp_vo_create: this library was built with packed FP32 (make PK=1, an A/B build): the "
                    "VO schedule defaults to the serial order; concurrent schedules are not bit-stable with it\n");
  }
  if (const char* e = getenv("PICP_VO_OVERLAP")) h->overlap = atoi(e) != 0;
  // at most two groups: three and four measured slower at the default shape (C5 592k / 404k vs
  // 597-600k frames/s with two, round 2), and so did four and eight at the
  // latency-bound shapes, where a step waits for its chain's slowest segment (round 6: 8e
  // 32.5k / 18.4k vs 42.0k frames/s, the N = 8 per-rank shape 90.2k / 50.0k vs 156.9k;
  // profiles/r06/t2/ab.log), also with 16 hardware queues (8e 30.1k / 28.5k, t6) and replayed
  // from a hipGraph (11.3k-25.8k, t7): the extra chains' world matches compete for the chip
  if (const char* e = getenv("PICP_VO_CHAINS")) h->chains = std::max(1, std::min(2, atoi(e)));
  if (const char* e = getenv("PICP_VO_PHASE")) h->phase = atoi(e) != 0;
  if (const char* e = getenv("PICP_VO_FUSE")) h->fuse = atoi(e) != 0;
  if (const char* e = getenv("PICP_VO_SPLIT")) h->split_env = atoi(e) < 0 ? -1 : (atoi(e) != 0 ? 1 : 0);
  if (!h->graph_env && (h->overlap || h->chains > 1)) h->use_graph = false;
  const size_t no = (size_t)std::max<int64_t>(n_obs, 1);
#define VO_TRY(expr)              \
  do {                            \
    int rc_ = (expr);             \
    if (rc_ != PICP_OK) {         \
      picp_vo_destroy(h);         \
      return rc_;                 \
    }                             \
  } while (0)
  if (const char* e = getenv("PICP_VO_GUARD")) h->guard = atoi(e) != 0;
  auto alloc = [&](void** p, size_t bytes) -> int {
    HIP_TRY(vo_malloc(h, p, bytes, "create"));
    return PICP_OK;
  };
  VO_TRY([&]() -> int {
    // the step chains' streams at the highest priority, the side stream at the lowest
    // (PICP_VO_PRIO=0: all at the default)
    int lo = 0;
    int hi = 0;
    const char* pe = getenv("PICP_VO_PRIO");
    if (!(pe && atoi(pe) == 0)) HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_TRY(hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, hi));
    // (a CU-masked side stream leaving every 2nd / 4th / 8th CU to the step chains measured equal
    // at every C5 shape, round 6, profiles/r06/t3/ab.log: not kept)
    if (h->overlap) HIP_TRY(hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking, lo));
    HIP_TRY(hipEventCreate(&h->ev0));
    HIP_TRY(hipEventCreate(&h->ev1));
    HIP_TRY(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
    h->cstream.assign((size_t)h->chains, nullptr);
    h->ev_cj.assign((size_t)h->chains, nullptr);
    h->ev_ph.assign((size_t)h->chains, nullptr);
    for (int c = 0; c < h->chains; ++c) {
      if (c > 0) HIP_TRY(hipStreamCreateWithPriority(&h->cstream[c], hipStreamNonBlocking, hi));
      HIP_TRY(hipEventCreateWithFlags(&h->ev_cj[c], hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&h->ev_ph[c], hipEventDisableTiming));
    }
    // the early world-match parts: throughput work beside the chains, at the side stream's priority
    if (h->split_env != 0) {
      h->estream.assign((size_t)h->chains, nullptr);
      h->ev_app.assign((size_t)h->chains, nullptr);
      h->ev_early.assign((size_t)2 * h->chains, nullptr);
      // A/B (PICP_VO_ECU_SKIP=k): the early parts on CU-masked queues leaving every k-th CU to
      // the step chains (a CU-masked stream has the default priority)
      const char* cm = getenv("PICP_VO_ECU_SKIP");
      std::vector<uint32_t> mask;
      if (cm && atoi(cm) >= 2) {
        int ncu = 0;
        HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
        const int k = atoi(cm);
        mask.assign((size_t)(ncu + 31) / 32, 0u);
        for (int i = 0; i < ncu; ++i)
          if (i % k != k - 1) mask[(size_t)i / 32] |= 1u << (i % 32);
      }
      for (int c = 0; c < h->chains; ++c) {
        if (!mask.empty())
          HIP_TRY(hipExtStreamCreateWithCUMask(&h->estream[c], (uint32_t)mask.size(), mask.data()));
        else
          HIP_TRY(hipStreamCreateWithPriority(&h->estream[c], hipStreamNonBlocking, lo));
        HIP_TRY(hipEventCreateWithFlags(&h->ev_app[c], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&h->ev_early[2 * c], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&h->ev_early[2 * c + 1], hipEventDisableTiming));
      }
    }
    return PICP_OK;
  }());
  VO_TRY(alloc((void**)&h->frame_off_d, (size_t)(n_frames + 1) * sizeof(int64_t)));
  VO_TRY(alloc((void**)&h->uv_d, no * sizeof(float2)));
  VO_TRY(alloc((void**)&h->desc_d, no * dim * sizeof(float)));
  VO_TRY(alloc((void**)&h->pm_bi, no * 4));
  VO_TRY(alloc((void**)&h->pm_acc, no * 4));
  VO_TRY(alloc((void**)&h->wm_bi, no * 4));
  VO_TRY(alloc((void**)&h->wm_acc, no * 4));
  VO_TRY(alloc((void**)&h->pm_bd, no * 4));
  VO_TRY(alloc((void**)&h->pm_sd, no * 4));
  VO_TRY(alloc((void**)&h->wm_bd, no * 4));
  VO_TRY(alloc((void**)&h->wm_sd, no * 4));
  h->dp = 16 * picp_match_prep_kch(dim);
  VO_TRY(alloc((void**)&h->obs_h, no * h->dp * sizeof(_Float16)));
  VO_TRY(alloc((void**)&h->obs_n1, no * 4));
  VO_TRY(alloc((void**)&h->obs_n2, no * 4));
  VO_TRY([&]() -> int {
    HIP_TRY(hipMemcpy(h->frame_off_d, frame_off, (size_t)(n_frames + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
    if (n_obs) {
      HIP_TRY(hipMemcpy(h->uv_d, uv, (size_t)n_obs * sizeof(float2), hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(h->desc_d, desc, (size_t)n_obs * dim * sizeof(float), hipMemcpyHostToDevice));
    }
    HIP_TRY(hipMemset(h->wm_acc, 0, no * 4));
    HIP_TRY(picp_launch_match_prep(nullptr, h->desc_d, n_obs, dim, h->obs_h, h->obs_n1, h->obs_n2));
    HIP_TRY(hipDeviceSynchronize());
    return PICP_OK;
  }());
#undef VO_TRY
  *out = h;
  return PICP_OK;
}

static int64_t frame_n(const picp_vo* h, int64_t f) { return h->frame_off[f + 1] - h->frame_off[f]; }

extern "C" int picp_vo_set_segments(picp_vo_t* h, int n_seg, const int64_t* first,
                                    const int32_t* steps, const float* boot_poses,
                                    const picp_params* prm) {
  CHECK_ARG(h && first && steps && boot_poses && prm, "picp_vo_set_segments: null argument");
  CHECK_ARG(n_seg >= 1 && n_seg <= VO_MAX_GRID_Y, "picp_vo_set_segments: n_seg must be in [1, 65535]");
  CHECK_ARG(prm->max_rounds >= 0 && prm->max_rounds <= 100000, "params.max_rounds out of range");
  CHECK_ARG(!(prm->threshold != prm->threshold), "params.threshold is NaN");
  // every argument is validated before the handle's current segments are released: a rejected
  // call leaves the handle as it was
  for (int s = 0; s < n_seg; ++s)
    CHECK_ARG(steps[s] >= 1 && first[s] >= 0 && first[s] + steps[s] < h->n_frames,
              "picp_vo_set_segments: segment out of range (needs frames first .. first+steps, steps >= 1)");
  // The world match writes its outputs (wm_*) at the query frame's observation offsets.  Step t of
  // segment s queries frame first[s] + t + 1, so two segments query one frame at the same step
  // exactly when their first frames are equal: they would write the same rows in one launch, and
  // that layout is rejected.  Segments querying one frame at different steps are fine in one step
  // chain (the launches are ordered) but not across chains (PICP_VO_CHAINS=2 runs the groups'
  // world matches concurrently), so such a layout runs the serial order.
  {
    std::vector<int64_t> f0s(first, first + n_seg);
    std::sort(f0s.begin(), f0s.end());
    for (int s = 1; s < n_seg; ++s)
      if (f0s[s] == f0s[s - 1])
        return picp_set_err(PICP_ERR_ARG, "picp_vo_set_segments: two segments start at frame %lld (they would "
                            "query frame %lld at the same step)", (long long)f0s[s], (long long)f0s[s] + 1);
  }
  int chains_eff = std::min(h->chains, n_seg);
  {
    std::vector<int> q_group((size_t)h->n_frames, -1);
    const int C = chains_eff;
    for (int s = 0; s < n_seg; ++s) {
      int grp = 0;
      while (grp + 1 < C && s >= (int)((int64_t)n_seg * (grp + 1) / C)) ++grp;
      for (int t = 0; t < steps[s]; ++t) {
        const int64_t f = first[s] + t + 1;
        if (q_group[f] >= 0 && q_group[f] != grp) chains_eff = 1;
        q_group[f] = grp;
      }
    }
  }
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipStreamSynchronize(h->stream));
  vo_free_segments(h);
  std::vector<VoSegment> segs((size_t)n_seg);
  std::vector<char> is_curr((size_t)h->n_frames, 0);
  int64_t map_slots = 0, n_slots = 0;
  int max_steps = 0;
  int64_t max_map = 0;  // the largest segment map (the world match's reference set)
  for (int s = 0; s < n_seg; ++s) {
    VoSegment& G = segs[s];
    G.f0 = first[s];
    G.steps = steps[s];
    G.pad = 0;
    G.map_off = map_slots;
    G.slot0 = n_slots;
    int64_t cap = frame_n(h, G.f0);  // bootstrap adds <= |frame f0|, step t adds <= |frame f0+t|
    for (int t = 0; t < G.steps; ++t) cap += frame_n(h, G.f0 + t);
    map_slots += std::max<int64_t>(cap, 1);
    max_map = std::max(max_map, cap);
    n_slots += G.steps + 1;
    max_steps = std::max(max_steps, (int)G.steps);
    for (int64_t f = G.f0; f < G.f0 + G.steps; ++f) is_curr[f] = 1;
  }
  // frame->next problems grouped by step index: chunk k holds frame f0+k of every segment with
  // more than k steps (the bootstrap and step 0 read chunk 0, step t reads chunk t).  Frames of
  // overlapping segments are matched once, in the first chunk that needs them.
  std::vector<MatchProblem> pprobs;
  std::vector<size_t> chunk_off(1, 0);
  std::vector<char> done((size_t)h->n_frames, 0);
  for (int k = 0; k < max_steps; ++k) {
    for (int s = 0; s < n_seg; ++s) {
      const int64_t f = first[s] + k;
      if (k < steps[s] && !done[f] && frame_n(h, f) > 0) {
        done[f] = 1;
        pprobs.push_back(MatchProblem{h->frame_off[f], frame_n(h, f), h->frame_off[f + 1], frame_n(h, f + 1)});
      }
    }
    chunk_off.push_back(pprobs.size());
  }
  int64_t cap_c = (std::max<int64_t>(h->max_obs, 1) + 3) / 4 * 4;
  // register-resident items per lane of picp_block_kernel: the largest power of two whose
  // 512 * npt slots the biggest frame fills (masked slots cost as much as live ones every
  // round; the few items past npt * 512 take the kernel's streamed-remainder path)
  int npt = 1;
  while (npt < 8 && (int64_t)npt * 2 * 512 <= h->max_obs) npt *= 2;

  // one allocation for everything sized by the segments
  struct Part { size_t off, bytes; };
  size_t total = 0;
  auto part = [&](size_t bytes) { Part p{total, bytes}; total += (bytes + 255) / 256 * 256; return p; };
  const Part p_segs = part(segs.size() * sizeof(VoSegment));
  const Part p_boot = part((size_t)n_seg * 32 * sizeof(float));
  const Part p_mxyz = part((size_t)map_slots * 3 * sizeof(float));
  const Part p_mdesc = part((size_t)map_slots * h->dim * sizeof(float));
  const Part p_mn = part((size_t)n_seg * sizeof(int64_t));
  const Part p_planes = part((size_t)5 * n_seg * cap_c * sizeof(float));
  const Part p_probs = part((size_t)n_seg * sizeof(PicpProblem));
  const Part p_stin = part((size_t)n_seg * sizeof(PicpState));
  const Part p_stout = part((size_t)n_seg * sizeof(PicpState));
  const Part p_wprobs = part((size_t)n_seg * sizeof(MatchProblem));
  const Part p_lprobs = part((size_t)n_seg * sizeof(MatchProblem));
  const Part p_eprobs = part((size_t)2 * n_seg * sizeof(MatchProblem));
  const Part p_pprobs = part(std::max<size_t>(pprobs.size(), 1) * sizeof(MatchProblem));
  const Part p_poses = part((size_t)n_slots * 16 * sizeof(float));
  const Part p_steps = part((size_t)n_slots * sizeof(VoStep));
  const Part p_pairs = part((size_t)n_seg * cap_c * sizeof(int2));
  const Part p_mh = part((size_t)map_slots * h->dp * sizeof(_Float16));
  const Part p_mn1 = part((size_t)map_slots * sizeof(float));
  const Part p_mn2 = part((size_t)map_slots * sizeof(float));
  // split scratch: each chain's world match (its n_seg_c problems) and the frame->next launches
  const int ks_force = picp_match_ksplit_env();
  // the split rule's form: the folded accept-only form needs dim <= 12 (bit 2)
  const int ks_form = h->accept_only | (h->dim <= 12 ? 4 : 0);
  std::vector<int> ks_w((size_t)chains_eff, 1);
  std::vector<int64_t> cap_w((size_t)chains_eff, 0);
  std::vector<Part> p_partw;
  for (int c = 0; c < chains_eff; ++c) {
    const int nsc = (int)((int64_t)n_seg * (c + 1) / chains_eff - (int64_t)n_seg * c / chains_eff);
    ks_w[c] = picp_match_ksplit_forced(nsc, h->max_obs, max_map, ks_form, ks_force);
    cap_w[c] = picp_match_split_scratch(ks_w[c], nsc, h->max_obs);
    p_partw.push_back(part((size_t)cap_w[c] * sizeof(float4)));
  }
  // the split by map age: a chain's early part takes the whole world match's range split, plus one
  // slot for the late part (2 buffers: step t's merge and step t+2's early part overlap)
  std::vector<char> split_c((size_t)chains_eff, 0);
  std::vector<int64_t> cap_e((size_t)chains_eff, 0);
  std::vector<int> ks_e((size_t)chains_eff, 1);
  const char* eks = getenv("PICP_VO_EKS");
  std::vector<Part> p_parte;
  for (int c = 0; c < chains_eff; ++c) {
    const int nsc = (int)((int64_t)n_seg * (c + 1) / chains_eff - (int64_t)n_seg * c / chains_eff);
    split_c[c] = !h->estream.empty() && (h->split_env == 1 || (h->split_env < 0 && ks_w[c] > 1));
    ks_e[c] = (eks && atoi(eks) > 0) ? std::max(picp_match_ksplit_forced(nsc, h->max_obs, max_map, ks_form,
                                                                         atoi(eks)), 1)
                                     : ks_w[c];
    if (split_c[c]) cap_e[c] = (int64_t)(ks_e[c] + 1) * nsc * std::max<int64_t>(h->max_obs, 1);
    p_parte.push_back(part((size_t)2 * cap_e[c] * sizeof(float4)));
  }
  // the frame->next launches, as vo_frame_match issues them: the whole table up front (overlap off)
  // or chunk by chunk, each in launches of at most VO_MAX_GRID_Y problems
  std::vector<std::pair<size_t, int>> ks_p;
  int64_t cap_p = 0;
  {
    auto plan = [&](size_t p0, size_t p1) {
      for (size_t q = p0; q < p1; q += VO_MAX_GRID_Y) {
        const int n = (int)std::min<size_t>(VO_MAX_GRID_Y, p1 - q);
        const int k = picp_match_ksplit_forced(n, h->max_obs, h->max_obs, ks_form, ks_force);
        ks_p.emplace_back(q, k);
        cap_p = std::max(cap_p, picp_match_split_scratch(k, n, h->max_obs));
      }
    };
    const size_t nck = chunk_off.size() - 1;
    if (h->overlap && nck > 1) {
      for (size_t k = 0; k < nck; ++k) plan(chunk_off[k], chunk_off[k + 1]);
    } else {
      plan(0, pprobs.size());
    }
  }
  const size_t part_p_bytes = (size_t)cap_p * sizeof(float4);
  const Part p_partp = part(part_p_bytes);
  HIP_TRY(vo_malloc(h, &h->seg_mem, total, "segments"));
  HIP_TRY(hipMemset(h->seg_mem, 0, total));  // every table defined before the first run
  char* m = (char*)h->seg_mem;
  h->ev_chunk.assign((size_t)max_steps, nullptr);
  for (auto& e : h->ev_chunk) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  h->chunk_off = chunk_off;
  h->chains_eff = chains_eff;
  h->ks_w = ks_w;
  h->cap_w = cap_w;
  h->ks_p = ks_p;
  h->cap_p = cap_p;
  h->part_w.assign((size_t)chains_eff, nullptr);
  for (int c = 0; c < chains_eff; ++c)
    if (p_partw[c].bytes) h->part_w[c] = (float4*)(m + p_partw[c].off);
  h->split_c = split_c;
  h->cap_e = cap_e;
  h->ks_e = ks_e;
  h->part_e.assign((size_t)2 * chains_eff, nullptr);
  for (int c = 0; c < chains_eff; ++c)
    if (split_c[c]) {
      h->part_e[2 * c] = (float4*)(m + p_parte[c].off);
      h->part_e[2 * c + 1] = h->part_e[2 * c] + cap_e[c];
    }
  h->part_p = part_p_bytes ? (float4*)(m + p_partp.off) : nullptr;
  h->segs = segs;
  h->pprobs = pprobs;
  h->n_seg = n_seg;
  h->max_steps = max_steps;
  h->npt = npt;
  h->map_slots = map_slots;
  h->n_slots = n_slots;
  h->cap_c = cap_c;
  HIP_TRY(hipMemcpy(m + p_segs.off, segs.data(), p_segs.bytes, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(m + p_boot.off, boot_poses, p_boot.bytes, hipMemcpyHostToDevice));
  if (!pprobs.empty()) HIP_TRY(hipMemcpy(m + p_pprobs.off, pprobs.data(), p_pprobs.bytes, hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(m + p_mn.off, 0, p_mn.bytes));
  HIP_TRY(hipMemset(m + p_steps.off, 0, p_steps.bytes));
  HIP_TRY(hipMemset(m + p_poses.off, 0, p_poses.bytes));
  HIP_TRY(hipMemset(m + p_planes.off, 0, p_planes.bytes));

  PicpArgs& A = h->pargs;
  memset(&A, 0, sizeof(A));
  memcpy(A.K, h->K, sizeof(A.K));
  A.maxx = (float)(h->cols - 1);
  A.maxy = (float)(h->rows - 1);
  A.threshold = prm->threshold;
  A.damping = prm->damping;
  A.conv_eps = prm->conv_eps;
  A.min_inliers = prm->min_inliers;
  A.keep_outliers = prm->keep_outliers ? 1 : 0;
  A.max_rounds = prm->max_rounds;
  A.uniform = 0;

  VoArgs& V = h->vargs;
  memset(&V, 0, sizeof(V));
  memcpy(V.K, h->K, sizeof(V.K));
  V.dim = h->dim;
  V.n_seg = n_seg;
  V.seg0 = 0;
  V.frame_off = h->frame_off_d;
  V.uv = h->uv_d;
  V.desc = h->desc_d;
  V.segs = (const VoSegment*)(m + p_segs.off);
  V.boot = (const float*)(m + p_boot.off);
  V.pm_bi = h->pm_bi;
  V.pm_acc = h->pm_acc;
  V.wm_bi = h->wm_bi;
  V.wm_acc = h->wm_acc;
  V.map_xyz = (float*)(m + p_mxyz.off);
  V.map_desc = (float*)(m + p_mdesc.off);
  V.map_n = (int64_t*)(m + p_mn.off);
  float* planes = (float*)(m + p_planes.off);
  const size_t plane = (size_t)n_seg * cap_c;
  V.X = planes;
  V.Y = planes + plane;
  V.Z = planes + 2 * plane;
  V.U = planes + 3 * plane;
  V.V = planes + 4 * plane;
  V.cap_c = cap_c;
  V.probs = (PicpProblem*)(m + p_probs.off);
  V.st_in = (PicpState*)(m + p_stin.off);
  V.st_out = (const PicpState*)(m + p_stout.off);
  V.wprobs = (MatchProblem*)(m + p_wprobs.off);
  V.lprobs = (MatchProblem*)(m + p_lprobs.off);
  V.eprobs = (MatchProblem*)(m + p_eprobs.off);
  V.seg_all = n_seg;
  // the append writes the split tables when any chain splits (one launch covers one chain)
  V.split = 0;
  for (int c = 0; c < chains_eff; ++c) V.split |= split_c[c] ? 1 : 0;
  V.poses = (float*)(m + p_poses.off);
  V.steps = (VoStep*)(m + p_steps.off);
  V.pairs = (int2*)(m + p_pairs.off);
  V.dp = h->dp;
  V.obs_h = h->obs_h;
  V.obs_n1 = h->obs_n1;
  V.obs_n2 = h->obs_n2;
  V.map_h = (_Float16*)(m + p_mh.off);
  V.map_n1 = (float*)(m + p_mn1.off);
  V.map_n2 = (float*)(m + p_mn2.off);
  h->wprobs_d = V.wprobs;
  h->pprobs_d = (MatchProblem*)(m + p_pprobs.off);
  return PICP_OK;
}

// frame->next match problems [p0, p1) on stream st, in launches of at most VO_MAX_GRID_Y problems
static hipError_t vo_frame_match(picp_vo* h, hipStream_t st, size_t p0, size_t p1) {
  hipError_t e = hipSuccess;
  for (; p0 < p1 && e == hipSuccess; p0 += VO_MAX_GRID_Y) {
    const int np = (int)std::min<size_t>(VO_MAX_GRID_Y, p1 - p0);
    // the split planned for this launch at set_segments (a launch it did not plan runs unsplit)
    auto it = std::lower_bound(h->ks_p.begin(), h->ks_p.end(), std::make_pair(p0, 0));
    const int ks = (it != h->ks_p.end() && it->first == p0) ? it->second : 1;
    e = picp_launch_match_mfma(st, np, h->max_obs, h->desc_d, h->desc_d, h->obs_h, h->obs_n1, h->obs_h,
                               h->obs_n1, h->obs_n2, h->pprobs_d + p0, h->dim, VO_MATCH_DIST, VO_MATCH_RATIO,
                               h->pm_bi, h->pm_bd, h->pm_sd, h->pm_acc, h->accept_only, ks, h->part_p, h->cap_p);
  }
  return e;
}

#ifdef PICP_VO_DIAG
// Diagnostic build only (tools/vo_snap.py): after step t's PICP launch over segments [s0, s1),
// copy its problems, initial and final states and SoA planes into snapshot t (layout:
// picp_vo_debug_snap_bytes).  Copies run on the launch's stream, so they see exactly the block
// kernel's inputs and outputs.
static size_t vo_snap_step_bytes(const picp_vo* h) {
  return (size_t)h->n_seg * (sizeof(PicpProblem) + 2 * sizeof(PicpState) + 5 * (size_t)h->cap_c * sizeof(float));
}
static hipError_t vo_snap(picp_vo* h, hipStream_t st, int t, int s0, int s1) {
  if (!h->snap) return hipSuccess;
  const VoArgs& V = h->vargs;
  char* d = h->snap + (size_t)t * vo_snap_step_bytes(h);
  const size_t ns = (size_t)h->n_seg, k = (size_t)(s1 - s0);
  hipError_t e = hipMemcpyAsync(d + s0 * sizeof(PicpProblem), V.probs + s0, k * sizeof(PicpProblem),
                                hipMemcpyDeviceToDevice, st);
  d += ns * sizeof(PicpProblem);
  if (e == hipSuccess)
    e = hipMemcpyAsync(d + s0 * sizeof(PicpState), V.st_in + s0, k * sizeof(PicpState), hipMemcpyDeviceToDevice, st);
  d += ns * sizeof(PicpState);
  if (e == hipSuccess)
    e = hipMemcpyAsync(d + s0 * sizeof(PicpState), V.st_out + s0, k * sizeof(PicpState), hipMemcpyDeviceToDevice, st);
  d += ns * sizeof(PicpState);
  const float* planes[5] = {V.X, V.Y, V.Z, V.U, V.V};
  for (int q = 0; q < 5 && e == hipSuccess; ++q)
    e = hipMemcpyAsync(d + ((size_t)q * ns + s0) * h->cap_c * sizeof(float), planes[q] + (size_t)s0 * h->cap_c,
                       k * h->cap_c * sizeof(float), hipMemcpyDeviceToDevice, st);
  return e;
}
extern "C" int picp_vo_debug_snap_bytes(picp_vo_t* h, int64_t* per_step, int* n_steps) {
  CHECK_ARG(h && per_step && n_steps && h->n_seg > 0, "picp_vo_debug_snap_bytes: bad argument");
  *per_step = (int64_t)vo_snap_step_bytes(h);
  *n_steps = h->max_steps;
  return PICP_OK;
}
extern "C" int picp_vo_debug_snap_set(picp_vo_t* h, void* dev_buf) {
  CHECK_ARG(h, "picp_vo_debug_snap_set: bad argument");
  h->snap = (char*)dev_buf;
  if (h->exec) {  // re-capture with (or without) the copies
    hipGraphExecDestroy(h->exec);
    h->exec = nullptr;
  }
  if (h->graph) {
    hipGraphDestroy(h->graph);
    h->graph = nullptr;
  }
  return PICP_OK;
}
#endif

// the whole sequence on the handle's stream.  With overlap on, the frame->next match chunks
// 1.. run on the side stream (forked after chunk 0, joined by each step's append, which waits
// for its own chunk): the step chain is a string of latency-bound one-block-per-segment
// kernels, and the throughput-bound match chunks fill the CUs it leaves idle.
static hipError_t vo_enqueue(picp_vo* h) {
#ifdef PICP_VO_DIAG
  // diagnostic build only (wrong results; never the shipped library): PICP_VO_DIAG_SKIP bit 1
  // gather, 2 append, 4 PICP, 8 world match launches left out of the sequence
  static const int skip = [] {
    const char* e = getenv("PICP_VO_DIAG_SKIP");
    return e ? atoi(e) : 0;
  }();
#else
  constexpr int skip = 0;
#endif
  const size_t nck = h->chunk_off.size() - 1;
  const bool ov = h->overlap && nck > 1;
  hipError_t e = vo_frame_match(h, h->stream, 0, ov ? h->chunk_off[1] : h->chunk_off[nck]);
  if (e == hipSuccess && ov) {
    e = hipEventRecord(h->ev_fork, h->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(h->side, h->ev_fork, 0);
    for (size_t k = 1; k < nck && e == hipSuccess; ++k) {
      e = vo_frame_match(h, h->side, h->chunk_off[k], h->chunk_off[k + 1]);
      if (e == hipSuccess) e = hipEventRecord(h->ev_chunk[k], h->side);
    }
  }
  if (e == hipSuccess && !(skip & 2)) e = picp_launch_vo_append(h->stream, &h->vargs, -1);
  const int C = std::min(h->chains_eff, h->n_seg);
  // step u's early world-match part of chain c (the map as step u-2's append left it) on the
  // chain's early stream; its ranges go to scratch slots 0.. of buffer u & 1
  auto early_part = [&](int c, const VoArgs& V, int u) {
    hipStream_t es = h->estream[c];
    const int p = u & 1;
    hipError_t r = hipSuccess;
    if (!(skip & 8))
      r = picp_launch_match_mfma_parts(es, V.n_seg, h->max_obs, h->desc_d, V.map_desc, h->obs_h, h->obs_n1,
                                       V.map_h, V.map_n1, V.map_n2, V.eprobs + (size_t)p * h->n_seg + V.seg0,
                                       h->dim, VO_MATCH_DIST, VO_MATCH_RATIO, h->accept_only, h->ks_e[c], 0,
                                       h->part_e[2 * c + p], h->cap_e[c]);
    if (r == hipSuccess) r = hipEventRecord(h->ev_early[2 * c + p], es);
    return r;
  };

  // one world-match launch over chain c's segments [s0, s0 + n): tables probs (+ s0)
  auto world_match = [&](hipStream_t st, const VoArgs& V, const MatchProblem* probs, int c) {
    return picp_launch_match_mfma(st, V.n_seg, h->max_obs, h->desc_d, V.map_desc, h->obs_h, h->obs_n1, V.map_h,
                                  V.map_n1, V.map_n2, probs + V.seg0, h->dim, VO_MATCH_DIST, VO_MATCH_RATIO,
                                  h->wm_bi, h->wm_bd, h->wm_sd, h->wm_acc, h->accept_only,
                                  h->part_w[c] ? h->ks_w[c] : 1, h->part_w[c], h->cap_w[c]);
  };
#ifdef PICP_VO_DIAG
  const bool fused = false;  // vo_snap and PICP_VO_DIAG_SKIP need the gather's planes and launch
#else
  const bool fused = h->fuse && picp_vo_block_fusable(h->npt, h->max_obs);
#endif
  if (e == hipSuccess && C > 1) e = hipEventRecord(h->ev_cj[0], h->stream);  // fork
  // the chains' launches are enqueued step by step, chain after chain within a step: enqueued
  // chain after chain, every later chain's first launch waited on the host for the earlier
  // chains' whole sequence (~120 launches each), which is how long the GPU ran without it at the
  // start of a timed region.  Each stream's own order, and so every result, is unchanged.
  std::vector<hipStream_t> cst((size_t)C);
  std::vector<VoArgs> cv((size_t)C, h->vargs);
  std::vector<int> csteps((size_t)C, 0);
  int max_steps = 0;
  for (int c = 0; c < C; ++c) {
    cst[c] = (c == 0) ? h->stream : h->cstream[c];
    const int s0 = (int)((int64_t)h->n_seg * c / C), s1 = (int)((int64_t)h->n_seg * (c + 1) / C);
    cv[c].seg0 = s0;
    cv[c].n_seg = s1 - s0;
    for (int s = s0; s < s1; ++s) csteps[c] = std::max(csteps[c], (int)h->segs[s].steps);
    max_steps = std::max(max_steps, csteps[c]);
  }

  for (int t = 0; t < max_steps && e == hipSuccess; ++t) {
    for (int c = 0; c < C && e == hipSuccess; ++c) {
      if (t >= csteps[c]) continue;
      hipStream_t st = cst[c];
      const VoArgs& V = cv[c];
      const int s0 = V.seg0, s1 = V.seg0 + V.n_seg;
      (void)s1;
      // chain c starts after chain c-1's first world match (enqueued just before, at t = 0)
      if (t == 0 && c > 0) e = hipStreamWaitEvent(st, (h->phase ? h->ev_ph[c - 1] : h->ev_cj[0]), 0);
      const bool sp = h->split_c[c] && t >= 1;
      if (sp) {
        // the late part into the slot after the early ranges, then the merge of both
        const int p = t & 1;
        e = hipStreamWaitEvent(st, h->ev_early[2 * c + p], 0);
        if (e == hipSuccess && !(skip & 8))
          e = picp_launch_match_mfma_parts(st, V.n_seg, h->max_obs, h->desc_d, V.map_desc, h->obs_h, h->obs_n1,
                                           V.map_h, V.map_n1, V.map_n2, V.lprobs + s0, h->dim, VO_MATCH_DIST,
                                           VO_MATCH_RATIO, h->accept_only, 1, h->ks_e[c], h->part_e[2 * c + p],
                                           h->cap_e[c]);
        if (e == hipSuccess && !(skip & 8))
          e = picp_launch_match_merge(st, V.eprobs + (size_t)p * h->n_seg + s0, V.n_seg, h->max_obs, h->ks_e[c],
                                      h->ks_e[c], h->part_e[2 * c + p], h->cap_e[c], VO_MATCH_DIST, VO_MATCH_RATIO,
                                      h->wm_bi, h->wm_bd, h->wm_sd, h->wm_acc);
      } else if (e == hipSuccess && !(skip & 8)) {
        e = world_match(st, V, h->wprobs_d, c);
      }
      // step t+1's early part (the map as step t-1's append left it), started once this step's
      // match is merged: it runs beside this step's latency-bound PICP kernel and append rather
      // than beside the next step's late part and merge (round 6, profiles/r06/t15/)
      if (h->split_c[c] && t + 1 < csteps[c] && e == hipSuccess) {
        e = hipEventRecord(h->ev_app[c], st);
        if (e == hipSuccess) e = hipStreamWaitEvent(h->estream[c], h->ev_app[c], 0);
        if (e == hipSuccess) e = early_part(c, V, t + 1);
      }
      if (e == hipSuccess && t == 0 && C > 1 && c + 1 < C) e = hipEventRecord(h->ev_ph[c], st);
      if (fused) {
        if (e == hipSuccess && !(skip & 4)) e = picp_launch_vo_block(st, &V, t, h->npt, &h->pargs, h->max_obs);
      } else {
        if (e == hipSuccess && !(skip & 1)) e = picp_launch_vo_gather(st, &V, t);
        if (e == hipSuccess && !(skip & 4))
          e = picp_launch_block(st, V.n_seg, h->npt, V.X, V.Y, V.Z, V.U, V.V, &h->pargs, V.probs + s0,
                                V.st_in + s0, (PicpState*)V.st_out + s0, (int)h->max_obs, 1, nullptr, nullptr,
                                nullptr, 0);
      }
#ifdef PICP_VO_DIAG
      if (e == hipSuccess) e = vo_snap(h, st, t, s0, s1);
#endif
      if (e == hipSuccess && ov && t >= 1) e = hipStreamWaitEvent(st, h->ev_chunk[t], 0);
      if (e == hipSuccess && !(skip & 2)) e = picp_launch_vo_append(st, &V, t);
    }
  }
  for (int c = 1; c < C && e == hipSuccess; ++c) e = hipEventRecord(h->ev_cj[c], cst[c]);
  for (int c = 1; c < C && e == hipSuccess; ++c) e = hipStreamWaitEvent(h->stream, h->ev_cj[c], 0);  // join
  return e;
}

static int vo_launch(picp_vo* h) {
  CHECK_ARG(h && h->n_seg > 0, "picp_vo: no segments set");
  HIP_TRY(hipSetDevice(h->device));
  if (!h->use_graph) {
    HIP_TRY(vo_enqueue(h));
    return PICP_OK;
  }
  if (!h->exec) {
    HIP_TRY(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    hipError_t e = vo_enqueue(h);
    hipGraph_t g = nullptr;
    hipError_t e2 = hipStreamEndCapture(h->stream, &g);
    if (e != hipSuccess || e2 != hipSuccess) {
      if (g) hipGraphDestroy(g);
      return picp_set_err(PICP_ERR_DEVICE, "picp_vo: graph capture failed: %s",
                          hipGetErrorString(e != hipSuccess ? e : e2));
    }
    h->graph = g;
    HIP_TRY(hipGraphInstantiate(&h->exec, g, nullptr, nullptr, 0));
  }
  HIP_TRY(hipGraphLaunch(h->exec, h->stream));
  return PICP_OK;
}

extern "C" int picp_vo_run_async(picp_vo_t* h) { return vo_launch(h); }

extern "C" int picp_vo_sync(picp_vo_t* h) {
  CHECK_ARG(h, "picp_vo_sync: null handle");
  HIP_TRY(hipStreamSynchronize(h->stream));
  return PICP_OK;
}

extern "C" int picp_vo_run(picp_vo_t* h) {
  int rc = vo_launch(h);
  if (rc != PICP_OK) return rc;
  return picp_vo_sync(h);
}

extern "C" int picp_vo_time(picp_vo_t* h, int reps, float* ms_per_run) {
  CHECK_ARG(h && ms_per_run && reps >= 1, "picp_vo_time: bad argument");
  int rc = PICP_OK;
  if (h->use_graph && !h->exec) {  // capture outside the timed events
    rc = vo_launch(h);
    if (rc != PICP_OK) return rc;
  }
  HIP_TRY(hipEventRecord(h->ev0, h->stream));
  for (int r = 0; r < reps; ++r) {
    rc = vo_launch(h);
    if (rc != PICP_OK) return rc;
  }
  HIP_TRY(hipEventRecord(h->ev1, h->stream));
  HIP_TRY(hipEventSynchronize(h->ev1));
  float ms = 0.0f;
  HIP_TRY(hipEventElapsedTime(&ms, h->ev0, h->ev1));
  *ms_per_run = ms / reps;
  return PICP_OK;
}

extern "C" int picp_vo_get_poses(picp_vo_t* h, float* poses) {
  CHECK_ARG(h && poses && h->n_seg > 0, "picp_vo_get_poses: bad argument");
  HIP_TRY(hipStreamSynchronize(h->stream));
  HIP_TRY(hipMemcpy(poses, h->vargs.poses, (size_t)h->n_slots * 16 * sizeof(float), hipMemcpyDeviceToHost));
  return PICP_OK;
}

extern "C" int picp_vo_get_steps(picp_vo_t* h, picp_vo_step* steps) {
  CHECK_ARG(h && steps && h->n_seg > 0, "picp_vo_get_steps: bad argument");
  HIP_TRY(hipStreamSynchronize(h->stream));
  HIP_TRY(hipMemcpy(steps, h->vargs.steps, (size_t)h->n_slots * sizeof(VoStep), hipMemcpyDeviceToHost));
  return PICP_OK;
}

extern "C" int picp_vo_get_map(picp_vo_t* h, int seg, int64_t cap, float* xyz, float* desc, int64_t* n) {
  CHECK_ARG(h && n && h->n_seg > 0 && seg >= 0 && seg < h->n_seg, "picp_vo_get_map: bad argument");
  HIP_TRY(hipStreamSynchronize(h->stream));
  int64_t mn = 0;
  HIP_TRY(hipMemcpy(&mn, h->vargs.map_n + seg, sizeof(int64_t), hipMemcpyDeviceToHost));
  *n = mn;
  const int64_t k = std::min(mn, std::max<int64_t>(cap, 0));
  const int64_t off = h->segs[seg].map_off;
  if (xyz && k)
    HIP_TRY(hipMemcpy(xyz, h->vargs.map_xyz + 3 * off, (size_t)k * 3 * sizeof(float), hipMemcpyDeviceToHost));
  if (desc && k)
    HIP_TRY(hipMemcpy(desc, h->vargs.map_desc + off * h->dim, (size_t)k * h->dim * sizeof(float),
                      hipMemcpyDeviceToHost));
  return PICP_OK;
}

extern "C" int picp_vo_debug_matches(picp_vo_t* h, int which, int32_t* dst) {
  CHECK_ARG(h && dst && which >= 0 && which <= 3, "picp_vo_debug_matches: bad argument");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  const int32_t* src[4] = {h->pm_bi, h->pm_acc, h->wm_bi, h->wm_acc};
  if (h->n_obs) HIP_TRY(hipMemcpy(dst, src[which], (size_t)h->n_obs * 4, hipMemcpyDeviceToHost));
  return PICP_OK;
}

extern "C" int picp_vo_debug_guard(picp_vo_t* h, int64_t* bad_bytes, int* bad_buffer) {
  CHECK_ARG(h && bad_bytes && bad_buffer, "picp_vo_debug_guard: bad argument");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());
  *bad_bytes = 0;
  *bad_buffer = -1;
  std::vector<unsigned char> pad(VO_GUARD);
  for (size_t i = 0; i < h->guards.size(); ++i) {
    const VoGuarded& g = h->guards[i];
    for (int side = 0; side < 2; ++side) {
      const char* src = side ? g.base + VO_GUARD + g.bytes : g.base;
      HIP_TRY(hipMemcpy(pad.data(), src, VO_GUARD, hipMemcpyDeviceToHost));
      int64_t bad = 0;
      for (unsigned char c : pad) bad += (c != VO_GUARD_BYTE);
      if (bad && *bad_buffer < 0) *bad_buffer = (int)(2 * i + side);
      *bad_bytes += bad;
    }
  }
  return PICP_OK;
}

extern "C" int picp_vo_info(picp_vo_t* h, int64_t* n_obs, int64_t* n_slots, int64_t* map_slots, int* npt) {
  CHECK_ARG(h, "picp_vo_info: null handle");
  if (n_obs) *n_obs = h->n_obs;
  if (n_slots) *n_slots = h->n_slots;
  if (map_slots) *map_slots = h->map_slots;
  if (npt) *npt = h->npt;
  return PICP_OK;
}
