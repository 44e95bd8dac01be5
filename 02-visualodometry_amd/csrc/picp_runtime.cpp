// picp_runtime.cpp -- host runtime behind the C-ABI (include/picp_c.h).
//
// Owns device memory, the HIP stream of each handle, the block partition of a batch and the
// hipGraph that replays the fused R-round solve (graph mode: 1 memcpy node + 1 ticket memset
// node + R round launches, each finished in-launch by its last arriving block).  No torch, no host fallback: every compute entry point runs the HIP
// kernels of picp_kernels.hip or fails with PICP_ERR_DEVICE.
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "picp_c.h"
#include "picp_comm.h"
#include "picp_host.h"
#include "picp_internal.h"

extern "C" hipError_t picp_launch_round(hipStream_t stream, int grid, int vec, const float* X,
                                        const float* Y, const float* Z, const float* U,
                                        const float* V, const PicpArgs* args,
                                        const PicpProblem* probs, const int4* blkinfo,
                                        const PicpState* st_in, PicpState* st_out,
                                        unsigned long long* part, unsigned int* tickets, int j);
extern "C" hipError_t picp_launch_persistent(hipStream_t stream, int grid, int npt, const float* X,
                                             const float* Y, const float* Z, const float* U,
                                             const float* V, const PicpArgs* args,
                                             const PicpState* st_in, PicpState* st_out,
                                             unsigned long long* gpart, unsigned long long* gpose,
                                             unsigned int* err, unsigned int* tagbase,
                                             unsigned long long* arrive, unsigned long long timeout_ticks);
extern "C" hipError_t picp_launch_block(hipStream_t stream, int n_problems, int npt, const float* X,
                                        const float* Y, const float* Z, const float* U,
                                        const float* V, const PicpArgs* args,
                                        const PicpProblem* probs, const PicpState* st_in,
                                        PicpState* st_out, int max_n, int split,
                                        unsigned long long* xg, unsigned int* err,
                                        unsigned int* tagbase, unsigned long long timeout_ticks);
extern "C" int picp_block_max_items(void);
extern "C" int picp_block_threads(int split);
extern "C" int picp_block_npt_cap(int split);
extern "C" int picp_persistent_block(void);
extern "C" hipError_t picp_persistent_occupancy(int npt, const float K[9], int* blocks_per_cu);
extern "C" hipError_t picp_block_occupancy(int npt, int split, int max_n, const float K[9], int* blocks_per_cu);
extern "C" hipError_t picp_launch_match(hipStream_t stream, int n_problems, int64_t max_nq,
                                        const float* q_desc, const float* r_desc,
                                        const MatchProblem* probs, int dim, float dist_thr,
                                        float ratio_thr, int32_t* best_idx, float* best_dist,
                                        float* second_dist, int32_t* accepted);
extern "C" __global__ void picp_rcp_check_kernel(int e_lo, int e_hi, unsigned long long* bad);
extern "C" hipError_t picp_launch_essential(hipStream_t stream, const EssArgs* args, const int64_t* offs,
                                           const float* p1, const float* p2, int32_t* idx, double* Es,
                                           int32_t* ns, int32_t* cnt, float* T_out, int32_t* inliers,
                                           int32_t* good, uint8_t* mask);
extern "C" hipError_t picp_launch_gather(hipStream_t stream, const float* world,
                                         const float* image, const int2* pairs, int64_t m,
                                         float* X, float* Y, float* Z, float* U, float* V,
                                         int64_t off);
extern "C" hipError_t picp_launch_triangulate(hipStream_t stream, const float* P1,
                                              const float* P2, const float2* uv1,
                                              const float2* uv2, int64_t q, float* xyz);

// ------------------------------------------------------------------------------------
// error plumbing
// ------------------------------------------------------------------------------------
static thread_local std::string g_err;

int picp_set_err(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
#define set_err picp_set_err

extern "C" const char* picp_last_error(void) { return g_err.c_str(); }
extern "C" int picp_abi_version(void) { return PICP_ABI_VERSION; }

extern "C" void picp_params_default(picp_params* p) {
  if (!p) return;
  p->threshold = 1000.0f;  // src/picp_solver.cpp:14
  p->damping = 1.0f;       // src/picp_solver.cpp:11
  p->min_inliers = 0;      // src/picp_solver.cpp:12
  p->keep_outliers = 0;    // exec/icp_test.cpp:95
  p->max_rounds = 50;      // exec/icp_test.cpp:88
  p->conv_eps = 1e-5f;     // exec/icp_test.cpp:91
}

extern "C" int picp_device_count(int* n) {
  CHECK_ARG(n, "picp_device_count: null output");
  int c = 0;
  HIP_TRY(hipGetDeviceCount(&c));
  *n = c;
  return PICP_OK;
}

// ------------------------------------------------------------------------------------
// pose helpers (column-major 4x4 <-> state R(col-major 3x3), t)
// ------------------------------------------------------------------------------------
static void pose_to_state(const float T[16], PicpState& s) {
  for (int j = 0; j < 3; ++j)
    for (int i = 0; i < 3; ++i) s.R[j * 3 + i] = T[j * 4 + i];
  for (int i = 0; i < 3; ++i) s.t[i] = T[12 + i];
}

static void state_to_pose(const PicpState& s, float T[16]) {
  memset(T, 0, 16 * sizeof(float));
  for (int j = 0; j < 3; ++j)
    for (int i = 0; i < 3; ++i) T[j * 4 + i] = s.R[j * 3 + i];
  for (int i = 0; i < 3; ++i) T[12 + i] = s.t[i];
  T[15] = 1.0f;
}

static void state_to_stats(const PicpState& s, picp_stats& st) {
  st.chi_in = s.chi_in;
  st.chi_out = s.chi_out;
  st.n_in = s.n_in;
  st.ok = s.ok;
  st.rounds = s.rounds;
  st.converged = s.converged;
  st.n_projected = s.n_proj;
  st.reserved = 0;
}

static int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

#define PICP_MODE_GRAPH 0
#define PICP_MODE_PERSISTENT 1
#define PICP_MODE_BLOCK 2
#define PICP_POSE_GRAN 16
#define PICP_MAX_PBLK 256

// ------------------------------------------------------------------------------------
// batch
// ------------------------------------------------------------------------------------
struct picp_batch {
  int64_t max_n = 0;           // largest problem (block mode sizes its LDS stage with it)
  int device = 0;
  hipStream_t stream = nullptr;
  int np = 0;
  int rows = 0, cols = 0;
  float K[9];
  std::vector<int64_t> offs;   // user correspondence offsets (np+1)
  std::vector<int64_t> plane_off;  // per problem offset into the SoA planes (mult. of 4)
  int64_t total = 0;           // correspondences
  int64_t plane_len = 0;       // padded plane length (floats)
  int64_t plane_cap = 0;       // allocated plane length
  float* planes = nullptr;     // 5 * plane_cap floats: X | Y | Z | U | V
  int nblk = 0;                // linearize blocks per launch
  int nblk_cap = 0;
  int np_cap = 0;
  std::vector<PicpProblem> probs_h;
  std::vector<int4> blk_h;
  PicpProblem* probs_d = nullptr;
  int4* blk_d = nullptr;
  PicpState* init_d = nullptr;
  PicpState* st_d[2] = {nullptr, nullptr};
  unsigned long long* part_d = nullptr;  // graph mode: published block partials (16 words each)
  unsigned int* tickets_d = nullptr;     // graph mode: per-problem arrival tickets
  PicpState* st_pinned = nullptr;  // np_cap states
  std::vector<PicpState> init_h;
  std::vector<PicpState> result_h;
  bool params_set = false;
  picp_params params;
  PicpArgs args;               // by-value kernel arguments (baked into the captured graph)
  int ipb = PICP_BLOCK;        // items per linearize block
  int vec = 1;                 // correspondences per lane per chunk (1 or 4)
  int uniform = 0;             // all problems the same size -> no block tables
  int n_u = 0;
  int64_t stride_u = 0;
  int num_cu = 256;            // compute units of the device
  int split = 1;               // block mode: blocks per problem (1, or 2 when 2*np fits the chip)
  int mode = PICP_MODE_GRAPH;  // PICP_MODE_GRAPH (launch per round) / PICP_MODE_PERSISTENT
  int npt = 1;                 // persistent: correspondences per lane held in registers
  unsigned char* sync = nullptr;   // persistent: [err 16 B | pose granules | partial granules | tag bases]
  size_t sync_bytes = 0, sync_cap = 0;
  uint64_t tag_rounds = 0;     // persistent: rounds enqueued since the sync area was last zeroed
  int result_idx = 0;          // st_d[] holding the final state of the last solve
  bool last_persistent = false;  // the last solve was a persistent launch (check its error word)
  unsigned long long timeout_ticks = 20000000ull;  // 200 ms of s_memrealtime (100 MHz)
  // co-residency (persistent and split block modes hand rounds between blocks of one launch)
  bool no_handoff = false;     // a hand-off wait timed out once: lay out without cross-block waits
  int fallbacks = 0;           // solves re-run in graph mode after a timed-out hand-off
  int handoff_grid = 0;        // blocks of the hand-off launch (0: the mode has none)
  int handoff_resident = 0;    // blocks the device holds at once for it (occupancy x CUs)
  // graph cache
  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  int g_rounds = -1;
  int last_rounds = 0;  // R of the last solve (final state in st_d[R&1])

  float* X() const { return planes; }
  float* Y() const { return planes + plane_cap; }
  float* Z() const { return planes + 2 * plane_cap; }
  float* U() const { return planes + 3 * plane_cap; }
  float* V() const { return planes + 4 * plane_cap; }
};

// persistent launches and split block launches hand off through granules and report a timed-out
// wait in the error word at the head of b->sync
static bool uses_err_word(const picp_batch* b) {
  return b->mode == PICP_MODE_PERSISTENT || (b->mode == PICP_MODE_BLOCK && b->split > 1);
}

// exchange granules / tag bases of a split block layout: the grid (one granule set per block)
static int64_t xg_grid(const picp_batch* b) {
  const int64_t ss = std::max(b->split, 1);
  return ((ss * b->np + 8 * ss - 1) / (8 * ss)) * (8 * ss);
}

static void drop_graph(picp_batch* b) {
  if (b->gexec) hipGraphExecDestroy(b->gexec);
  if (b->graph) hipGraphDestroy(b->graph);
  b->gexec = nullptr;
  b->graph = nullptr;
  b->g_rounds = -1;
}

static int items_per_block(int64_t total, int num_cu) {
  const char* env = getenv("PICP_ITEMS_PER_BLOCK");
  if (env) {
    int v = atoi(env);
    if (v >= 4) return (int)round_up(v, 4);
  }
  // Latency-bound single frames: one correspondence per lane (spread over every SIMD).
  // Large batches (HBM streaming): float4 per lane and several chunks per lane to amortise the
  // block reduction and the partial traffic.
  if (total <= ((int64_t)1 << 18)) return 2 * PICP_BLOCK;  // measured best for C2 (tools/sweep.py)
  // streaming: about two resident 256-thread blocks per CU (all blocks in flight at once),
  // each streaming its slice through the prefetch ring (profiles/r01/sweep_*m_*.log)
  if (total < (int64_t)2 << 20) return PICP_BLOCK * 4 * 2;
  if (total < (int64_t)8 << 20) return PICP_BLOCK * 4 * 8;
  // Round the block count to a multiple of 2 x CUs so every CU carries the same load: with 489
  // blocks on 256 CUs some CUs hold one block and some two, and the round waits for the slowest
  // (16M: 489 blocks 69.0 us/round, 512 blocks 66.5 us; at 2M/4M the difference is in the noise;
  // profiles/r01/sweep_balance.log).
  const int64_t target = PICP_BLOCK * 4 * 32;
  const int64_t unit = 2 * (int64_t)std::max(1, num_cu);
  int64_t nb = ((total + target - 1) / target + unit / 2) / unit * unit;
  nb = std::max(nb, unit);
  return (int)round_up((total + nb - 1) / nb, 4);
}

// Resident blocks per CU for a hand-off launch: the occupancy query of the exact kernel variant,
// capped by PICP_RESIDENT_BLOCKS_PER_CU (a test hook that emulates a device partly held by other
// work; 0 forces the layouts without cross-block waits).
static int resident_per_cu(hipError_t q, int occ) {
  if (q != hipSuccess) occ = 0;
  if (const char* e = getenv("PICP_RESIDENT_BLOCKS_PER_CU")) occ = std::min(occ, std::max(0, atoi(e)));
  return occ;
}

// (Re)build the partition for correspondence offsets `offs` (np+1 entries).
static int batch_layout(picp_batch* b, const int64_t* offs_in, int np) {
  const std::vector<int64_t> offs_copy(offs_in, offs_in + np + 1);  // offs_in may be b->offs itself
  const int64_t* offs = offs_copy.data();
  CHECK_ARG(np >= 1, "batch: n_problems must be >= 1");
  for (int i = 0; i < np; ++i)
    CHECK_ARG(offs[i + 1] >= offs[i] && offs[0] == 0, "batch: corr_offsets must be a prefix sum from 0");
  b->np = np;
  b->offs.assign(offs, offs + np + 1);
  b->total = offs[np];
  b->uniform = 1;
  for (int i = 1; i < np; ++i)
    if (offs[i + 1] - offs[i] != offs[1] - offs[0]) b->uniform = 0;
  b->n_u = (int)(offs[1] - offs[0]);
  b->stride_u = round_up(b->n_u, 4);
  // Execution mode:
  //  * BLOCK      -- one block per problem, all rounds in-block, problem held in registers:
  //                  batches of >= 2 problems of <= picp_block_max_items() correspondences;
  //  * PERSISTENT -- one launch, blocks of one problem hand off through granules: when every
  //                  block of the batch is resident at once (uniform problems);
  //  * GRAPH      -- one launch per round, replayed from a hipGraph: everything else.
  // PICP_MODE=graph|persistent|block forces a mode when the batch is eligible for it.
  int ipb = items_per_block(b->total, b->num_cu);
  b->mode = PICP_MODE_GRAPH;
  {
    const char* m = getenv("PICP_MODE");
    const bool force_graph = m && strcmp(m, "graph") == 0;
    const bool force_persist = m && strcmp(m, "persistent") == 0;
    const bool force_block = m && strcmp(m, "block") == 0;
    int64_t max_n = 0;
    for (int i = 0; i < np; ++i) max_n = std::max<int64_t>(max_n, offs[i + 1] - offs[i]);
    b->max_n = max_n;
    int bnpt = 0;  // block mode: register-resident correspondences per lane (rest streamed)
    {
      int cap = picp_block_max_items() / 512;
      if (const char* e = getenv("PICP_BLOCK_NPT")) cap = std::max(1, std::min(cap, atoi(e)));
      bnpt = 1;
      while (bnpt < cap && (int64_t)bnpt * 512 < max_n) bnpt *= 2;
      // one block per problem: only sensible while a problem is small enough for one CU
      if (max_n > ((int64_t)1 << 16)) bnpt = 0;
    }
    int pnpt = 0, pnb = 0;  // persistent mode partition
    {
      int bpp = b->num_cu / np;  // blocks per problem available
      if (const char* e = getenv("PICP_PERSIST_BLOCKS")) bpp = std::max(1, std::min(bpp, atoi(e)));
      const int pbs = picp_persistent_block();
      if (b->uniform && bpp >= 1) {
        const int64_t per_block = std::max<int64_t>(1, (b->n_u + bpp - 1) / bpp);
        int npt = 1;
        while ((int64_t)npt * pbs < per_block && npt < 32) npt *= 2;
        const int nb = (int)std::max<int64_t>(1, (b->n_u + (int64_t)npt * pbs - 1) / ((int64_t)npt * pbs));
        if (npt <= 8 && nb <= PICP_MAX_PBLK && (int64_t)nb * np <= b->num_cu) {
          pnpt = npt;
          pnb = nb;
        }
      }
    }
    // Persistent blocks wait on each other every round, so all of them must be resident at once:
    // launch that mode only when the occupancy query says the grid fits (otherwise, or after a
    // timed-out hand-off, the batch runs in graph mode).
    b->handoff_grid = 0;
    b->handoff_resident = 0;
    if (pnpt && b->no_handoff) pnpt = 0;
    if (pnpt) {
      int occ = 0;
      const int res = resident_per_cu(picp_persistent_occupancy(pnpt, b->K, &occ), occ) * b->num_cu;
      b->handoff_grid = pnb * np;
      b->handoff_resident = res;
      if ((int64_t)pnb * np > res) pnpt = 0;
    }
    if (force_graph) {
      b->mode = PICP_MODE_GRAPH;
    } else if (force_block && bnpt) {
      b->mode = PICP_MODE_BLOCK;
    } else if (force_persist && pnpt) {
      b->mode = PICP_MODE_PERSISTENT;
    } else if (np >= 2 && bnpt) {
      b->mode = PICP_MODE_BLOCK;
    } else if (pnpt) {
      b->mode = PICP_MODE_PERSISTENT;
    }
    b->split = 1;
    if (b->mode == PICP_MODE_PERSISTENT) {
      b->npt = pnpt;
      ipb = pnpt * picp_persistent_block();
    } else if (b->mode == PICP_MODE_BLOCK) {
      // two blocks per problem when every pair still gets its own CUs (C4: 128 frames on 256 CUs)
      // and the halves are big enough to pay for the per-round partner exchange;
      // PICP_BLOCK_SPLIT=1|2 forces
      auto grid_of = [&](int s) { return ((s * np + 8 * s - 1) / (8 * s)) * (8 * s); };
      int split = (grid_of(2) <= b->num_cu && max_n >= 4096) ? 2 : 1;
      // four 512-thread parts per problem, two blocks per CU from different problems, when four
      // times the problems still fit two per CU and a part keeps >= 2048 correspondences (the C4
      // per-rank shape at N = 8, 128 frames x 10k): one block's round tail (at issue priority 3)
      // runs under the other's linearize; 22.0-22.4M vs 21.2-21.4M it/s for split 2
      // (profiles/r04/p1/).  256-thread parts (round 1) were 5 % slower.
      if (grid_of(4) <= 2 * b->num_cu && max_n >= 8192 && picp_block_threads(4) == 512) split = 4;
      if (b->no_handoff) split = 1;
      if (const char* e = getenv("PICP_BLOCK_SPLIT")) {
        const int v = atoi(e);
        if (v == 1) split = 1;
        if (v == 2 && grid_of(2) <= b->num_cu) split = 2;
        if (v == 4 && grid_of(4) <= 2 * b->num_cu) split = 4;
        if (b->no_handoff) split = 1;
      }
      // the parts of a split problem wait on each other every round: keep the split only if the
      // occupancy query says the whole grid is resident at once
      while (split > 1) {
        const int64_t part = round_up((max_n + split - 1) / split, 4);
        const int bs = picp_block_threads(split);
        int cap = std::min(picp_block_max_items() / 512, picp_block_npt_cap(split));
        if (const char* e = getenv("PICP_BLOCK_NPT")) cap = std::max(1, std::min(cap, atoi(e)));
        int snpt = 1;
        while (snpt < cap && (int64_t)snpt * bs < part) snpt *= 2;
        int occ = 0;
        const int res = resident_per_cu(picp_block_occupancy(snpt, split, (int)max_n, b->K, &occ), occ) * b->num_cu;
        b->handoff_grid = grid_of(split);
        b->handoff_resident = res;
        if (grid_of(split) <= res) break;
        split = (split == 4) ? 2 : 1;
      }
      b->split = split;
      if (split > 1) {  // register items per lane for a part
        const int64_t part = round_up((max_n + split - 1) / split, 4);
        const int bs = picp_block_threads(split);
        int cap = std::min(picp_block_max_items() / 512, picp_block_npt_cap(split));
        if (const char* e = getenv("PICP_BLOCK_NPT")) cap = std::max(1, std::min(cap, atoi(e)));
        bnpt = 1;
        while (bnpt < cap && (int64_t)bnpt * bs < part) bnpt *= 2;
      }
      b->npt = bnpt;
    }
  }
  // report the hand-off grid of the layout in use only (a candidate the occupancy check rejected
  // leaves no hand-off behind: picp_batch_residency then reads 0/0)
  if (!(b->mode == PICP_MODE_PERSISTENT || (b->mode == PICP_MODE_BLOCK && b->split > 1))) {
    b->handoff_grid = 0;
    b->handoff_resident = 0;
  }
  b->ipb = ipb;
  b->vec = (ipb >= 4 * PICP_BLOCK && b->mode == PICP_MODE_GRAPH) ? 4 : 1;
  b->plane_off.resize(np);
  int64_t pos = 0;
  int nblk = 0;
  for (int i = 0; i < np; ++i) {
    b->plane_off[i] = pos;
    const int64_t n = offs[i + 1] - offs[i];
    CHECK_ARG(n <= INT32_MAX, "batch: a problem has more than 2^31-1 correspondences");
    pos = round_up(pos + n, 4);
    nblk += (int)std::max<int64_t>(1, (n + ipb - 1) / ipb);
  }
  b->plane_len = std::max<int64_t>(pos, 4);
  b->nblk = nblk;
  hipError_t e;
  HIP_TRY(hipSetDevice(b->device));
  if (b->plane_len > b->plane_cap) {
    if (b->planes) hipFree(b->planes);
    b->planes = nullptr;
    const int64_t cap = round_up(b->plane_len, 1024);
    e = hipMalloc(&b->planes, (size_t)cap * 5 * sizeof(float));
    if (e != hipSuccess) return set_err(PICP_ERR_NOMEM, "hipMalloc planes (%lld floats): %s", (long long)cap * 5, hipGetErrorString(e));
    HIP_TRY(hipMemsetAsync(b->planes, 0, (size_t)cap * 5 * sizeof(float), b->stream));
    b->plane_cap = cap;
  }
  if (nblk > b->nblk_cap) {
    if (b->blk_d) hipFree(b->blk_d);
    if (b->part_d) hipFree(b->part_d);
    b->blk_d = nullptr;
    b->part_d = nullptr;
    HIP_TRY(hipMalloc(&b->blk_d, (size_t)nblk * sizeof(int4)));
    HIP_TRY(hipMalloc(&b->part_d, (size_t)nblk * (PICP_NPART / 2) * sizeof(unsigned long long)));
    b->nblk_cap = nblk;
  }
  if (np > b->np_cap) {
    if (b->tickets_d) hipFree(b->tickets_d);
    b->tickets_d = nullptr;
    HIP_TRY(hipMalloc(&b->tickets_d, (size_t)np * sizeof(unsigned int)));
    HIP_TRY(hipMemsetAsync(b->tickets_d, 0, (size_t)np * sizeof(unsigned int), b->stream));
    if (b->probs_d) hipFree(b->probs_d);
    if (b->init_d) hipFree(b->init_d);
    for (int k = 0; k < 2; ++k) if (b->st_d[k]) hipFree(b->st_d[k]);
    if (b->st_pinned) hipHostFree(b->st_pinned);
    b->probs_d = nullptr; b->init_d = nullptr; b->st_d[0] = b->st_d[1] = nullptr; b->st_pinned = nullptr;
    HIP_TRY(hipMalloc(&b->probs_d, (size_t)np * sizeof(PicpProblem)));
    HIP_TRY(hipMalloc(&b->init_d, (size_t)np * sizeof(PicpState)));
    for (int k = 0; k < 2; ++k) {
      HIP_TRY(hipMalloc(&b->st_d[k], (size_t)np * sizeof(PicpState)));
      HIP_TRY(hipMemsetAsync(b->st_d[k], 0, (size_t)np * sizeof(PicpState), b->stream));
    }
    HIP_TRY(hipHostMalloc((void**)&b->st_pinned, (size_t)np * sizeof(PicpState), hipHostMallocDefault));
    b->np_cap = np;
  }
  if (uses_err_word(b)) {
    // persistent: error word (128-B line) | pose granule sets | partial granules (x2 parities);
    // split block: error word (128-B line) | exchange granules (x2 parities, 64 per block and
    // problem held) | tag bases
    const int64_t sgrid = xg_grid(b);
    b->sync_bytes = (b->mode == PICP_MODE_PERSISTENT)
                        ? (size_t)round_up(128 + (int64_t)np * PICP_POSE_SETS * PICP_POSE_GRAN * 8 + 2 * (int64_t)nblk * PICP_NPART * 8 +
                                               round_up((int64_t)np * 4, 128) + (int64_t)np * 128, 256)
                        : (size_t)round_up(128 + 2 * sgrid * 64 * 8 + sgrid * 4, 256);
    if (b->sync_bytes > b->sync_cap) {
      if (b->sync) hipFree(b->sync);
      b->sync = nullptr;
      HIP_TRY(hipMalloc(&b->sync, b->sync_bytes));
      b->sync_cap = b->sync_bytes;
    }
    // a new layout maps problems onto granules other problems tagged: start every tag from zero
    HIP_TRY(hipMemsetAsync(b->sync, 0, b->sync_bytes, b->stream));
    b->tag_rounds = 0;
  }
  // block table
  b->blk_h.resize(nblk);
  b->probs_h.resize(np);
  int blk = 0;
  for (int i = 0; i < np; ++i) {
    const int64_t n = offs[i + 1] - offs[i];
    PicpProblem& P = b->probs_h[i];
    memset(&P, 0, sizeof(P));
    P.offset = b->plane_off[i];
    P.n = (int32_t)n;
    P.blk0 = blk;
    const int nb = (int)std::max<int64_t>(1, (n + ipb - 1) / ipb);
    P.nblk = nb;
    for (int k = 0; k < nb; ++k) {
      const int64_t first = (int64_t)k * ipb;
      const int64_t cnt = std::max<int64_t>(0, std::min<int64_t>(ipb, n - first));
      b->blk_h[blk + k] = make_int4(i, (int)first, (int)cnt, 0);
    }
    blk += nb;
  }
  // Streaming single frame on two blocks per CU (nblk == 2 x CUs): the hardware issues the
  // older block of a CU first, so with equal slices the first num_cu blocks finish a round at
  // ~2/3 of the time the second ones need and their CUs then stream at half parallelism
  // (tools/stamps_place.py).  Pair block q with q + num_cu over a contiguous
  // range and give q the larger share (PICP_STREAM_SHARE, the first block's fraction).
  if (b->mode == PICP_MODE_GRAPH && np == 1 && b->vec == 4 && nblk == 2 * b->num_cu) {
    double share = 0.64;  // measured optimum (profiles/r01/sweep_share.log); 0.5 = equal slices
    if (const char* e = getenv("PICP_STREAM_SHARE")) share = atof(e);
    if (share > 0.5 && share < 0.9) {
      const int64_t n = offs[1] - offs[0];
      const int64_t pair = round_up((n + b->num_cu - 1) / b->num_cu, 4);
      const int64_t hi = round_up((int64_t)(pair * share), 4);
      for (int q = 0; q < b->num_cu; ++q) {
        const int64_t f0 = std::min<int64_t>(n, q * pair);
        const int64_t f1 = std::min<int64_t>(n, f0 + hi);
        const int64_t f2 = std::min<int64_t>(n, (q + 1) * pair);
        b->blk_h[q] = make_int4(0, (int)f0, (int)(f1 - f0), 0);
        b->blk_h[q + b->num_cu] = make_int4(0, (int)f1, (int)(f2 - f1), 0);
      }
      b->uniform = 0;  // the kernel reads the block table
    }
  }
  HIP_TRY(hipMemcpyAsync(b->blk_d, b->blk_h.data(), (size_t)nblk * sizeof(int4), hipMemcpyHostToDevice, b->stream));
  // identity initial poses by default
  b->init_h.assign(np, PicpState{});
  for (int i = 0; i < np; ++i) {
    memset(&b->init_h[i], 0, sizeof(PicpState));
    b->init_h[i].R[0] = b->init_h[i].R[4] = b->init_h[i].R[8] = 1.0f;
    // the loop state at entry (what a zero-round solve returns; the kernels set it again)
    b->init_h[i].chi_prev = FLT_MAX;
    b->init_h[i].ok = 1;
  }
  HIP_TRY(hipMemcpyAsync(b->init_d, b->init_h.data(), (size_t)np * sizeof(PicpState), hipMemcpyHostToDevice, b->stream));
  b->result_h.assign(np, PicpState{});
  HIP_TRY(hipMemcpyAsync(b->probs_d, b->probs_h.data(), (size_t)np * sizeof(PicpProblem), hipMemcpyHostToDevice, b->stream));
  b->params_set = false;
  drop_graph(b);
  HIP_TRY(hipStreamSynchronize(b->stream));
  return PICP_OK;
}

static int batch_upload_params(picp_batch* b, const picp_params* prm) {
  CHECK_ARG(prm, "null params");
  CHECK_ARG(prm->max_rounds >= 0 && prm->max_rounds <= 100000, "params.max_rounds out of range");
  CHECK_ARG(!(prm->threshold != prm->threshold), "params.threshold is NaN");
  if (b->params_set && memcmp(&b->params, prm, sizeof(picp_params)) == 0) return PICP_OK;
  PicpArgs& A = b->args;
  memset(&A, 0, sizeof(A));
  memcpy(A.K, b->K, sizeof(A.K));
  A.maxx = (float)(b->cols - 1);
  A.maxy = (float)(b->rows - 1);
  A.threshold = prm->threshold;
  A.damping = prm->damping;
  A.conv_eps = prm->conv_eps;
  A.min_inliers = prm->min_inliers;
  A.keep_outliers = prm->keep_outliers ? 1 : 0;
  A.max_rounds = prm->max_rounds;
  A.uniform = b->uniform;
  A.n_u = b->n_u;
  A.nblk_u = b->uniform ? b->nblk / b->np : 0;
  A.ipb = b->ipb;
  A.stride_u = b->stride_u;
  b->params = *prm;
  b->params_set = true;
  drop_graph(b);  // the arguments are baked into the captured launches
  return PICP_OK;
}

// graph mode: launch j reads st_d[(j+1)&1] and its last arrivers write st_d[j&1]; the initial
// states go to st_d[1], so after R launches the result is in st_d[(R-1)&1] (st_d[1] if R == 0)
static hipError_t launch_round(picp_batch* b, int j) {
  const int in_buf = (j + 1) & 1;
  return picp_launch_round(b->stream, b->nblk, b->vec, b->X(), b->Y(), b->Z(), b->U(), b->V(), &b->args,
                           b->probs_d, b->blk_d, b->st_d[in_buf], b->st_d[in_buf ^ 1], b->part_d,
                           b->tickets_d, j);
}

static int graph_result_idx(int R) { return R >= 1 ? ((R - 1) & 1) : 1; }

// graph-mode prologue of every solve: initial states in, arrival tickets zeroed
static hipError_t graph_prologue(picp_batch* b) {
  hipError_t e = hipMemcpyAsync(b->st_d[1], b->init_d, (size_t)b->np * sizeof(PicpState),
                                hipMemcpyDeviceToDevice, b->stream);
  if (e != hipSuccess) return e;
  return hipMemsetAsync(b->tickets_d, 0, (size_t)b->np * sizeof(unsigned int), b->stream);
}

// Enqueue a fused R-round solve on the stream: block / persistent mode one launch; graph mode
// the initial-state copy, the ticket memset and R round launches.
static hipError_t enqueue_solve(picp_batch* b, int R) {
  if (b->mode == PICP_MODE_BLOCK) {
    unsigned int* err = nullptr;
    unsigned long long* xg = nullptr;
    unsigned int* tagbase = nullptr;
    if (b->split > 1) {  // tags continue from the per-slot tag bases: no memset per launch
      const int64_t sgrid = xg_grid(b);
      err = reinterpret_cast<unsigned int*>(b->sync);
      // every block's 512-B granule set on whole 128-B lines: at sync + 16 each set shared a line
      // with its neighbour's, and C4 at 128 frames ran 3.5 % slower (profiles/r05/xg_align/)
      xg = reinterpret_cast<unsigned long long*>(b->sync + 128);
      tagbase = reinterpret_cast<unsigned int*>(xg + 2 * sgrid * 64);
    }
    return picp_launch_block(b->stream, b->np, b->npt, b->X(), b->Y(), b->Z(), b->U(), b->V(), &b->args,
                             b->probs_d, b->init_d, b->st_d[0], (int)b->max_n, b->split, xg, err, tagbase,
                             b->timeout_ticks);
  }
  if (b->mode == PICP_MODE_PERSISTENT) {
    // no memset per launch: granule tags continue from the per-problem tag bases the previous
    // launch left (picp_persistent.hip), so nothing a previous launch wrote can match
    unsigned int* err = reinterpret_cast<unsigned int*>(b->sync);
    // pose sets on 128-B lines of their own (an agent-scope store to a line drops it from the
    // XCD's L2, so an L2-kept set must not share a line with anything stored agent-scope)
    unsigned long long* gpose = reinterpret_cast<unsigned long long*>(b->sync + 128);
    unsigned long long* gpart = gpose + (size_t)b->np * PICP_POSE_SETS * PICP_POSE_GRAN;
    unsigned int* tagbase = reinterpret_cast<unsigned int*>(gpart + 2 * (size_t)b->nblk * PICP_NPART);
    // per-problem arrival counters on lines of their own, zeroed with the tag bases (A/B builds with
    // -DPICP_ARRIVAL count the blocks' publishes there; the shipped kernel does not touch them)
    unsigned long long* arrive =
        reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(tagbase) + round_up((int64_t)b->np * 4, 128));
    return picp_launch_persistent(b->stream, b->nblk, b->npt, b->X(), b->Y(), b->Z(), b->U(), b->V(),
                                  &b->args, b->init_d, b->st_d[0], gpart, gpose, err, tagbase, arrive,
                                  b->timeout_ticks);
  }
  hipError_t e = graph_prologue(b);
  if (e != hipSuccess) return e;
  for (int j = 0; j < R; ++j) {
    e = launch_round(b, j);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

static int ensure_graph(picp_batch* b, int R) {
  if (b->gexec && b->g_rounds == R) return PICP_OK;
  drop_graph(b);
  HIP_TRY(hipStreamBeginCapture(b->stream, hipStreamCaptureModeThreadLocal));
  hipError_t e = enqueue_solve(b, R);
  hipGraph_t g = nullptr;
  hipError_t e2 = hipStreamEndCapture(b->stream, &g);
  if (e != hipSuccess) { if (g) hipGraphDestroy(g); return set_err(PICP_ERR_DEVICE, "capture: %s", hipGetErrorString(e)); }
  if (e2 != hipSuccess) return set_err(PICP_ERR_DEVICE, "end capture: %s", hipGetErrorString(e2));
  b->graph = g;
  HIP_TRY(hipGraphInstantiate(&b->gexec, g, nullptr, nullptr, 0));
  b->g_rounds = R;
  return PICP_OK;
}

// Persistent and split block modes: the 32-bit granule tags grow by up to max_rounds per solve.
// Zero the sync area (tags and error word) on the stream before they could wrap (long before 2^32).
static hipError_t persistent_tag_guard(picp_batch* b, int R, int solves) {
  if (!uses_err_word(b) || !b->sync) return hipSuccess;
  const uint64_t add = (uint64_t)std::max(R, 1) * (uint64_t)solves;
  if (b->tag_rounds + add > (1ull << 31)) {
    hipError_t e = hipMemsetAsync(b->sync, 0, b->sync_bytes, b->stream);
    if (e != hipSuccess) return e;
    b->tag_rounds = 0;
  }
  b->tag_rounds += add;
  return hipSuccess;
}

// Enqueue one fused solve.  Persistent and block modes are ONE kernel launch: it goes to the
// stream directly (back-to-back launches queue behind each other with only the kernel-boundary
// gap; a one-node graph replay measured ~10 us more per solve).  Graph mode replays the captured
// prologue + R round launches.
static int enqueue_fused(picp_batch* b, int R) {
  if (b->mode == PICP_MODE_GRAPH) {
    int rc = ensure_graph(b, R);
    if (rc) return rc;
    HIP_TRY(hipGraphLaunch(b->gexec, b->stream));
  } else {
    HIP_TRY(enqueue_solve(b, R));
  }
  return PICP_OK;
}

static int batch_solve_async(picp_batch* b, const picp_params* prm) {
  HIP_TRY(hipSetDevice(b->device));
  int rc = batch_upload_params(b, prm);
  if (rc) return rc;
  const int R = prm->max_rounds;
  HIP_TRY(persistent_tag_guard(b, R, 1));
  rc = enqueue_fused(b, R);
  if (rc) return rc;
  b->last_rounds = R;
  b->result_idx = (b->mode == PICP_MODE_GRAPH) ? graph_result_idx(R) : 0;
  b->last_persistent = uses_err_word(b);
  return PICP_OK;
}

static int batch_layout(picp_batch* b, const int64_t* offs_in, int np);

// A cross-block hand-off wait timed out (the blocks were not all resident: another process or
// stream held CUs, or the device time-sliced the launch).  Lay the batch out again without
// hand-offs (persistent -> graph mode, split block -> one block per problem), keep its data and
// initial poses, and re-run the same solve; later solves keep that layout.
static int batch_rerun_without_handoff(picp_batch* b) {
  const std::vector<PicpState> init = b->init_h;
  const picp_params prm = b->params;
  const int R = b->last_rounds;
  b->no_handoff = true;
  b->fallbacks++;
  int rc = batch_layout(b, b->offs.data(), b->np);
  if (rc) return rc;
  b->init_h = init;
  HIP_TRY(hipMemcpyAsync(b->init_d, b->init_h.data(), (size_t)b->np * sizeof(PicpState), hipMemcpyHostToDevice, b->stream));
  picp_params p2 = prm;
  p2.max_rounds = R;
  rc = batch_upload_params(b, &p2);
  if (rc) return rc;
  rc = enqueue_fused(b, R);
  if (rc) return rc;
  b->last_rounds = R;
  b->result_idx = (b->mode == PICP_MODE_GRAPH) ? graph_result_idx(R) : 0;
  b->last_persistent = uses_err_word(b);
  return PICP_OK;
}

static int batch_read_results(picp_batch* b) {
  HIP_TRY(hipMemcpyAsync(b->st_pinned, b->st_d[b->result_idx], (size_t)b->np * sizeof(PicpState),
                         hipMemcpyDeviceToHost, b->stream));
  unsigned int err = 0;
  if (b->last_persistent && b->sync)
    HIP_TRY(hipMemcpyAsync(&err, b->sync, sizeof(err), hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  memcpy(b->result_h.data(), b->st_pinned, (size_t)b->np * sizeof(PicpState));
  if (err) {
    // the error word is sticky (persistent launches no longer zero it): reset the whole sync
    // area so the next solve starts clean, then report
    HIP_TRY(hipMemsetAsync(b->sync, 0, b->sync_bytes, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    b->tag_rounds = 0;
    if (b->no_handoff)  // cannot happen: that layout has no cross-block waits
      return set_err(PICP_ERR_DEVICE, "solve: a cross-block hand-off wait timed out (code %u)", err);
    int rc = batch_rerun_without_handoff(b);
    if (rc) return rc;
    return batch_read_results(b);
  }
  return PICP_OK;
}

static int batch_create(picp_batch** out, int device, int np, const int64_t* offs, int rows,
                        int cols, const float K[9]) {
  CHECK_ARG(out && offs && K, "picp_batch_create: null argument");
  CHECK_ARG(rows > 0 && cols > 0, "picp_batch_create: rows/cols must be positive");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  CHECK_ARG(device >= 0 && device < ndev, "picp_batch_create: no such HIP device");
  picp_batch* b = new picp_batch();
  b->device = device;
  b->rows = rows;
  b->cols = cols;
  memcpy(b->K, K, sizeof(b->K));
  picp_params_default(&b->params);
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&b->num_cu, hipDeviceAttributeMultiprocessorCount, device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking);
  if (const char* t = getenv("PICP_TIMEOUT_MS")) b->timeout_ticks = (unsigned long long)(atof(t) * 1e5);
  if (e != hipSuccess) {
    delete b;
    return set_err(PICP_ERR_DEVICE, "stream create: %s", hipGetErrorString(e));
  }
  int rc = batch_layout(b, offs, np);
  if (rc) {
    picp_batch_destroy(b);
    return rc;
  }
  *out = b;
  return PICP_OK;
}

extern "C" int picp_batch_create(picp_batch_t** out, int device, int n_problems,
                                 const int64_t* corr_offsets, int rows, int cols,
                                 const float K[9]) {
  return batch_create(out, device, n_problems, corr_offsets, rows, cols, K);
}

extern "C" int picp_batch_destroy(picp_batch_t* b) {
  if (!b) return PICP_OK;
  hipSetDevice(b->device);
  if (b->stream) hipStreamSynchronize(b->stream);
  drop_graph(b);
  if (b->planes) hipFree(b->planes);
  if (b->blk_d) hipFree(b->blk_d);
  if (b->probs_d) hipFree(b->probs_d);
  if (b->init_d) hipFree(b->init_d);
  for (int k = 0; k < 2; ++k)
    if (b->st_d[k]) hipFree(b->st_d[k]);
  if (b->part_d) hipFree(b->part_d);
  if (b->tickets_d) hipFree(b->tickets_d);
  if (b->st_pinned) hipHostFree(b->st_pinned);
  if (b->sync) hipFree(b->sync);
  if (b->stream) hipStreamDestroy(b->stream);
  delete b;
  return PICP_OK;
}

extern "C" int picp_batch_set_data(picp_batch_t* b, const float* xyz, const float* uv) {
  CHECK_ARG(b && (b->total == 0 || (xyz && uv)), "picp_batch_set_data: null argument");
  HIP_TRY(hipSetDevice(b->device));
  std::vector<float> host((size_t)b->plane_len * 5, 0.0f);
  float* hx = host.data();
  float* hy = hx + b->plane_len;
  float* hz = hy + b->plane_len;
  float* hu = hz + b->plane_len;
  float* hv = hu + b->plane_len;
  for (int i = 0; i < b->np; ++i) {
    const int64_t n = b->offs[i + 1] - b->offs[i], src = b->offs[i], dst = b->plane_off[i];
    for (int64_t k = 0; k < n; ++k) {
      hx[dst + k] = xyz[3 * (src + k) + 0];
      hy[dst + k] = xyz[3 * (src + k) + 1];
      hz[dst + k] = xyz[3 * (src + k) + 2];
      hu[dst + k] = uv[2 * (src + k) + 0];
      hv[dst + k] = uv[2 * (src + k) + 1];
    }
  }
  for (int c = 0; c < 5; ++c)
    HIP_TRY(hipMemcpyAsync(b->planes + (size_t)c * b->plane_cap, host.data() + (size_t)c * b->plane_len,
                           (size_t)b->plane_len * sizeof(float), hipMemcpyHostToDevice, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  return PICP_OK;
}

extern "C" int picp_batch_set_data_device(picp_batch_t* b, const float* dx, const float* dy,
                                          const float* dz, const float* du, const float* dv) {
  CHECK_ARG(b && (b->total == 0 || (dx && dy && dz && du && dv)), "picp_batch_set_data_device: null argument");
  HIP_TRY(hipSetDevice(b->device));
  const float* src[5] = {dx, dy, dz, du, dv};
  for (int i = 0; i < b->np; ++i) {
    const int64_t n = b->offs[i + 1] - b->offs[i];
    if (n == 0) continue;
    for (int c = 0; c < 5; ++c)
      HIP_TRY(hipMemcpyAsync(b->planes + (size_t)c * b->plane_cap + b->plane_off[i], src[c] + b->offs[i],
                             (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, b->stream));
  }
  HIP_TRY(hipStreamSynchronize(b->stream));
  return PICP_OK;
}

extern "C" int picp_batch_set_poses(picp_batch_t* b, const float* T) {
  CHECK_ARG(b && T, "picp_batch_set_poses: null argument");
  HIP_TRY(hipSetDevice(b->device));
  for (int i = 0; i < b->np; ++i) pose_to_state(T + 16 * (size_t)i, b->init_h[i]);
  HIP_TRY(hipMemcpyAsync(b->init_d, b->init_h.data(), (size_t)b->np * sizeof(PicpState), hipMemcpyHostToDevice, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  return PICP_OK;
}

extern "C" int picp_batch_get_poses(picp_batch_t* b, float* T) {
  CHECK_ARG(b && T, "picp_batch_get_poses: null argument");
  for (int i = 0; i < b->np; ++i) state_to_pose(b->result_h[i], T + 16 * (size_t)i);
  return PICP_OK;
}

extern "C" int picp_batch_get_stats(picp_batch_t* b, picp_stats* st) {
  CHECK_ARG(b && st, "picp_batch_get_stats: null argument");
  for (int i = 0; i < b->np; ++i) state_to_stats(b->result_h[i], st[i]);
  return PICP_OK;
}

extern "C" int picp_batch_solve_async(picp_batch_t* b, const picp_params* prm) {
  CHECK_ARG(b, "picp_batch_solve_async: null batch");
  return batch_solve_async(b, prm);
}

extern "C" int picp_batch_sync(picp_batch_t* b) {
  CHECK_ARG(b, "picp_batch_sync: null batch");
  HIP_TRY(hipSetDevice(b->device));
  return batch_read_results(b);
}

extern "C" int picp_batch_solve(picp_batch_t* b, const picp_params* prm) {
  CHECK_ARG(b, "picp_batch_solve: null batch");
  int rc = batch_solve_async(b, prm);
  if (rc) return rc;
  return batch_read_results(b);
}

extern "C" int picp_batch_info(picp_batch_t* b, int64_t* total, int* nblk, int* mode) {
  CHECK_ARG(b, "picp_batch_info: null batch");
  if (total) *total = b->total;
  if (nblk) *nblk = b->nblk;
  if (mode) *mode = b->mode;
  return PICP_OK;
}

// hipEvents destroyed on every return path
struct EventPair {
  hipEvent_t a = nullptr, b = nullptr;
  hipError_t create() {
    hipError_t e = hipEventCreate(&a);
    return e == hipSuccess ? hipEventCreate(&b) : e;
  }
  ~EventPair() {
    if (a) hipEventDestroy(a);
    if (b) hipEventDestroy(b);
  }
};

extern "C" int picp_batch_time(picp_batch_t* b, const picp_params* prm, int reps,
                               float* total_ms, float* launch_us) {
  CHECK_ARG(b && prm && reps > 0, "picp_batch_time: bad argument");
  HIP_TRY(hipSetDevice(b->device));
  // A hand-off wait that timed out inside the region is only seen by batch_read_results after
  // it, which re-runs the solve without hand-offs (fallbacks + 1).  The region's time then
  // includes the timed-out launches, so it is measured once more under the new layout.
  for (int attempt = 0;; ++attempt) {
    int rc = batch_upload_params(b, prm);
    if (rc) return rc;
    const int R = prm->max_rounds;
    if (b->mode == PICP_MODE_GRAPH) {
      rc = ensure_graph(b, R);  // captured before the timed region
      if (rc) return rc;
    }
    EventPair ev;
    HIP_TRY(ev.create());
    HIP_TRY(persistent_tag_guard(b, R, reps));
    HIP_TRY(hipEventRecord(ev.a, b->stream));
    for (int r = 0; r < reps; ++r) {
      rc = enqueue_fused(b, R);
      if (rc) return rc;
    }
    HIP_TRY(hipEventRecord(ev.b, b->stream));
    HIP_TRY(hipEventSynchronize(ev.b));
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, ev.a, ev.b));
    if (total_ms) *total_ms = ms;
    b->last_rounds = R;
    b->result_idx = (b->mode == PICP_MODE_GRAPH) ? graph_result_idx(R) : 0;
    b->last_persistent = uses_err_word(b);
    // mean launch period of the dominant kernel inside the region (graph mode: R round launches
    // per solve; otherwise one launch per solve); back-to-back launches, so this is the
    // per-launch duration a kernel trace reports plus the boundary gap
    const int launches = (b->mode == PICP_MODE_GRAPH) ? std::max(R, 1) : 1;
    if (launch_us) *launch_us = 1000.0f * ms / (float)(reps * launches);
    const int fb0 = b->fallbacks;
    rc = batch_read_results(b);
    if (rc || b->fallbacks == fb0) return rc;
    if (attempt >= 1)
      return set_err(PICP_ERR_STATE, "picp_batch_time: hand-off waits timed out again after the fallback");
  }
}

extern "C" int picp_batch_time_single(picp_batch_t* b, const picp_params* prm, float* us) {
  CHECK_ARG(b && prm && us, "picp_batch_time_single: bad argument");
  HIP_TRY(hipSetDevice(b->device));
  int rc = batch_upload_params(b, prm);
  if (rc) return rc;
  const int R = prm->max_rounds;
  HIP_TRY(persistent_tag_guard(b, R, 1));
  if (b->mode != PICP_MODE_GRAPH) {
    EventPair ev;
    HIP_TRY(ev.create());
    HIP_TRY(hipEventRecord(ev.a, b->stream));
    HIP_TRY(enqueue_solve(b, R));
    HIP_TRY(hipEventRecord(ev.b, b->stream));
    HIP_TRY(hipEventSynchronize(ev.b));
    float t = 0.0f;
    HIP_TRY(hipEventElapsedTime(&t, ev.a, ev.b));
    *us = 1000.0f * t;
    b->last_rounds = R;
    b->result_idx = 0;
    b->last_persistent = uses_err_word(b);
    return batch_read_results(b);
  }
  std::vector<EventPair> ev((size_t)std::max(R, 1));
  for (auto& e : ev) HIP_TRY(e.create());
  HIP_TRY(graph_prologue(b));
  for (int j = 0; j < R; ++j) {
    HIP_TRY(hipEventRecord(ev[j].a, b->stream));
    HIP_TRY(launch_round(b, j));
    HIP_TRY(hipEventRecord(ev[j].b, b->stream));
  }
  if (R > 0) HIP_TRY(hipEventSynchronize(ev[R - 1].b));
  double sum = 0.0;
  for (int j = 0; j < R; ++j) {
    float t = 0.0f;
    HIP_TRY(hipEventElapsedTime(&t, ev[j].a, ev[j].b));
    sum += 1000.0 * t;
  }
  *us = R > 0 ? (float)(sum / R) : 0.0f;
  b->last_rounds = R;
  b->result_idx = graph_result_idx(R);
  b->last_persistent = false;
  return batch_read_results(b);
}

extern "C" int picp_batch_residency(picp_batch_t* b, int* grid, int* resident, int* fallbacks) {
  CHECK_ARG(b, "picp_batch_residency: null batch");
  if (grid) *grid = b->handoff_grid;
  if (resident) *resident = b->handoff_resident;
  if (fallbacks) *fallbacks = b->fallbacks;
  return PICP_OK;
}

static void gather_to_poses(const PicpState* all, int64_t n_total, float* T_all, picp_stats* st_all) {
  for (int64_t k = 0; k < n_total; ++k) {
    state_to_pose(all[k], T_all + 16 * k);
    if (st_all) state_to_stats(all[k], st_all[k]);
  }
}

// Gather every rank's results of the batch split: this rank's batch holds the
// problems picp_shard_range(n_total, world, rank) gives it; after its solve, one RCCL all-gather
// of the 128-B per-problem states (on the batch's stream, device to device over xGMI) and one
// copy to the host give every rank all n_total poses and stats in problem order.
extern "C" int picp_batch_allgather(picp_batch_t* b, picp_comm_t* c, int64_t n_total, float* T_all,
                                    picp_stats* st_all) {
  CHECK_ARG(c, "picp_batch_allgather: null communicator");
  const int world = picp_comm_world(c), rank = picp_comm_rank(c);
  // Local checks first, agreed on by every rank before the collective: a rank that returned here
  // alone would leave the others blocked in the all-gather.
  int rc = PICP_OK;
  int64_t f0 = 0, f1 = 0;
  void* send = nullptr;
  const int64_t maxn = std::max<int64_t>(picp_shard_pad(n_total, world), 1);
  const size_t bytes = (size_t)maxn * sizeof(PicpState);
  if (!b || !T_all) rc = set_err(PICP_ERR_ARG, "picp_batch_allgather: null argument");
  else if (picp_comm_device(c) != b->device)
    rc = set_err(PICP_ERR_ARG, "picp_batch_allgather: communicator and batch are on different devices");
  else if ((rc = picp_shard_range(n_total, world, rank, &f0, &f1)) == PICP_OK && f1 - f0 != b->np)
    rc = set_err(PICP_ERR_ARG, "picp_batch_allgather: the batch does not hold this rank's shard of n_total");
  if (rc == PICP_OK && hipSetDevice(b->device) != hipSuccess)
    rc = set_err(PICP_ERR_DEVICE, "picp_batch_allgather: hipSetDevice failed");
  if (rc == PICP_OK) rc = batch_read_results(b);  // the solve is complete (re-run if a hand-off timed out)
  if (rc == PICP_OK && !(send = picp_comm_send_buffer(c, bytes)))
    rc = set_err(PICP_ERR_NOMEM, "picp_batch_allgather: staging buffer of %zu B", bytes);
  double fail = (rc == PICP_OK) ? 0.0 : 1.0;
  const std::string local_err = rc ? picp_last_error() : "";
  const int rc2 = picp_comm_allreduce_max(c, &fail, 1);
  if (rc) return set_err(rc, "%s", local_err.c_str());
  if (rc2) return rc2;
  if (fail != 0.0) return set_err(PICP_ERR_STATE, "picp_batch_allgather: another rank failed before the all-gather");
  HIP_TRY(hipMemcpyAsync(send, b->st_d[b->result_idx], (size_t)b->np * sizeof(PicpState), hipMemcpyDeviceToDevice,
                         b->stream));
  const void* recv = nullptr;
  rc = picp_comm_allgather_dev(c, send, bytes, b->stream, &recv);
  if (rc) return rc;
  std::vector<PicpState> padded((size_t)world * maxn), all((size_t)std::max<int64_t>(n_total, 1));
  HIP_TRY(hipMemcpyAsync(padded.data(), recv, padded.size() * sizeof(PicpState), hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  rc = picp_shard_unpack(n_total, world, sizeof(PicpState), padded.data(), all.data());
  if (rc) return rc;
  gather_to_poses(all.data(), n_total, T_all, st_all);
  return PICP_OK;
}

// The gather with a caller-supplied byte exchange (include/picp_c.h): the same shard check,
// completion and padded state layout as picp_batch_allgather, staged through host memory.  Each
// rank's send buffer is [16-B header: int32 status][maxn states]; one exchange carries both, so
// the failure agreement needs no second collective.
extern "C" int picp_batch_allgather_host(picp_batch_t* b, int world, int rank, picp_exchange_fn exchange,
                                         void* user, int64_t n_total, float* T_all, picp_stats* st_all) {
  CHECK_ARG(exchange && world >= 1 && rank >= 0 && rank < world && n_total >= 0,
            "picp_batch_allgather_host: bad exchange or world/rank");
  int rc = PICP_OK;
  int64_t f0 = 0, f1 = 0;
  const int64_t maxn = std::max<int64_t>(picp_shard_pad(n_total, world), 1);
  constexpr size_t HDR = 16;
  const size_t bytes = HDR + (size_t)maxn * sizeof(PicpState);
  if (!b || !T_all) rc = set_err(PICP_ERR_ARG, "picp_batch_allgather_host: null argument");
  else if ((rc = picp_shard_range(n_total, world, rank, &f0, &f1)) == PICP_OK && f1 - f0 != b->np)
    rc = set_err(PICP_ERR_ARG, "picp_batch_allgather_host: the batch does not hold this rank's shard of n_total");
  if (rc == PICP_OK && hipSetDevice(b->device) != hipSuccess)
    rc = set_err(PICP_ERR_DEVICE, "picp_batch_allgather_host: hipSetDevice failed");
  if (rc == PICP_OK) rc = batch_read_results(b);  // the solve is complete (re-run if a hand-off timed out)
  const std::string local_err = rc ? picp_last_error() : "";
  std::vector<char> send(bytes, 0), recv(bytes * (size_t)world, 0);
  const int32_t status = rc;
  memcpy(send.data(), &status, sizeof(status));
  if (rc == PICP_OK) memcpy(send.data() + HDR, b->result_h.data(), (size_t)b->np * sizeof(PicpState));
  const int xr = exchange(user, send.data(), recv.data(), bytes);
  if (rc) return set_err(rc, "%s", local_err.c_str());
  if (xr != 0) return set_err(PICP_ERR_STATE, "picp_batch_allgather_host: the exchange failed (%d)", xr);
  std::vector<PicpState> padded((size_t)world * maxn), all((size_t)std::max<int64_t>(n_total, 1));
  for (int r = 0; r < world; ++r) {
    int32_t st = 0;
    memcpy(&st, recv.data() + (size_t)r * bytes, sizeof(st));
    if (st != PICP_OK)
      return set_err(PICP_ERR_STATE, "picp_batch_allgather_host: rank %d failed before the exchange (%d)", r, st);
    memcpy(padded.data() + (size_t)r * maxn, recv.data() + (size_t)r * bytes + HDR, (size_t)maxn * sizeof(PicpState));
  }
  rc = picp_shard_unpack(n_total, world, sizeof(PicpState), padded.data(), all.data());
  if (rc) return rc;
  gather_to_poses(all.data(), n_total, T_all, st_all);
  return PICP_OK;
}

// ------------------------------------------------------------------------------------
// single-problem handle (the pr::PICPSolver drop-in)
// ------------------------------------------------------------------------------------
struct picp_handle {
  picp_batch* b = nullptr;
  float* world_d = nullptr;
  int64_t n_world = 0, cap_world = 0;
  float* image_d = nullptr;
  int64_t n_image = 0, cap_image = 0;
  int2* pairs_d = nullptr;
  int64_t cap_pairs = 0;
  std::vector<int32_t> pairs_h;  // cached copy of the current correspondences
  int64_t m = -1;                // -1: none set
  bool have_points = false;
  bool gathered = false;
  float pose[16];
};

static void identity16(float T[16]) {
  memset(T, 0, 16 * sizeof(float));
  T[0] = T[5] = T[10] = T[15] = 1.0f;
}

extern "C" int picp_create(picp_t** out, int device, int rows, int cols, const float K[9]) {
  CHECK_ARG(out && K, "picp_create: null argument");
  picp_handle* h = new picp_handle();
  identity16(h->pose);
  const int64_t offs[2] = {0, 0};
  int rc = batch_create(&h->b, device, 1, offs, rows, cols, K);
  if (rc) {
    delete h;
    return rc;
  }
  *out = h;
  return PICP_OK;
}

extern "C" int picp_destroy(picp_t* h) {
  if (!h) return PICP_OK;
  if (h->b) {
    hipSetDevice(h->b->device);
    hipStreamSynchronize(h->b->stream);
  }
  if (h->world_d) hipFree(h->world_d);
  if (h->image_d) hipFree(h->image_d);
  if (h->pairs_d) hipFree(h->pairs_d);
  picp_batch_destroy(h->b);
  delete h;
  return PICP_OK;
}

extern "C" int picp_set_camera(picp_t* h, int rows, int cols, const float K[9]) {
  CHECK_ARG(h && K, "picp_set_camera: null argument");
  CHECK_ARG(rows > 0 && cols > 0, "picp_set_camera: rows/cols must be positive");
  h->b->rows = rows;
  h->b->cols = cols;
  memcpy(h->b->K, K, sizeof(h->b->K));
  h->b->params_set = false;
  return PICP_OK;
}

static int grow(void** ptr, int64_t* cap, int64_t need, size_t elem) {
  if (need <= *cap) return PICP_OK;
  if (*ptr) hipFree(*ptr);
  *ptr = nullptr;
  const int64_t c = std::max<int64_t>(need, 256);
  hipError_t e = hipMalloc(ptr, (size_t)c * elem);
  if (e != hipSuccess) { *cap = 0; return set_err(PICP_ERR_NOMEM, "hipMalloc(%zu): %s", (size_t)c * elem, hipGetErrorString(e)); }
  *cap = c;
  return PICP_OK;
}

// The copy constructor of the reference's PICPSolver copies every member, including the
// non-owning world/image pointers (src/picp_solver.h:72-81), so a copy solves the same problem.
// Here the points live on the device: the clone gets its own copies of them, the current
// correspondences and the pose (the cached gather is redone lazily).
extern "C" int picp_clone(const picp_t* src, picp_t** out) {
  CHECK_ARG(src && out, "picp_clone: null argument");
  const picp_batch* sb = src->b;
  picp_t* h = nullptr;
  int rc = picp_create(&h, sb->device, sb->rows, sb->cols, sb->K);
  if (rc) return rc;
  memcpy(h->pose, src->pose, sizeof(h->pose));
  auto fail = [&](int code) {
    picp_destroy(h);
    return code;
  };
  if (src->have_points) {
    HIP_TRY(hipSetDevice(sb->device));
    rc = grow((void**)&h->world_d, &h->cap_world, 3 * src->n_world, sizeof(float));
    if (rc) return fail(rc);
    rc = grow((void**)&h->image_d, &h->cap_image, 2 * src->n_image, sizeof(float));
    if (rc) return fail(rc);
    // the source's stream is drained first: its uploads may still be in flight
    hipError_t e = hipStreamSynchronize(sb->stream);
    if (e == hipSuccess && src->n_world)
      e = hipMemcpyAsync(h->world_d, src->world_d, (size_t)src->n_world * 3 * sizeof(float),
                         hipMemcpyDeviceToDevice, h->b->stream);
    if (e == hipSuccess && src->n_image)
      e = hipMemcpyAsync(h->image_d, src->image_d, (size_t)src->n_image * 2 * sizeof(float),
                         hipMemcpyDeviceToDevice, h->b->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->b->stream);
    if (e != hipSuccess) return fail(set_err(PICP_ERR_DEVICE, "picp_clone: %s", hipGetErrorString(e)));
    h->n_world = src->n_world;
    h->n_image = src->n_image;
    h->have_points = true;
  }
  h->pairs_h = src->pairs_h;
  h->m = src->m;
  h->gathered = false;
  *out = h;
  return PICP_OK;
}

extern "C" int picp_set_points(picp_t* h, const float* world, int64_t n_world, const float* image,
                               int64_t n_image) {
  CHECK_ARG(h, "picp_set_points: null handle");
  CHECK_ARG(n_world >= 0 && n_image >= 0, "picp_set_points: negative size");
  CHECK_ARG((n_world == 0 || world) && (n_image == 0 || image), "picp_set_points: null array");
  HIP_TRY(hipSetDevice(h->b->device));
  int rc = grow((void**)&h->world_d, &h->cap_world, 3 * n_world, sizeof(float));
  if (rc) return rc;
  rc = grow((void**)&h->image_d, &h->cap_image, 2 * n_image, sizeof(float));
  if (rc) return rc;
  if (n_world) HIP_TRY(hipMemcpyAsync(h->world_d, world, (size_t)n_world * 3 * sizeof(float), hipMemcpyHostToDevice, h->b->stream));
  if (n_image) HIP_TRY(hipMemcpyAsync(h->image_d, image, (size_t)n_image * 2 * sizeof(float), hipMemcpyHostToDevice, h->b->stream));
  HIP_TRY(hipStreamSynchronize(h->b->stream));
  h->n_world = n_world;
  h->n_image = n_image;
  h->have_points = true;
  h->gathered = false;
  // the cached correspondences stay valid as indices but must be re-checked and re-gathered
  if (h->m >= 0) {
    for (int64_t k = 0; k < h->m; ++k) {
      if (h->pairs_h[2 * k] < 0 || h->pairs_h[2 * k] >= n_image || h->pairs_h[2 * k + 1] < 0 || h->pairs_h[2 * k + 1] >= n_world) {
        h->m = -1;
        h->pairs_h.clear();
        break;
      }
    }
  }
  return PICP_OK;
}

// Upload + gather the correspondences into the SoA planes if anything changed.
static int handle_prepare(picp_handle* h) {
  if (!h->have_points) return set_err(PICP_ERR_STATE, "points not set (call picp_set_points first)");
  if (h->m < 0) return set_err(PICP_ERR_STATE, "correspondences not set");
  if (h->gathered) return PICP_OK;
  picp_batch* b = h->b;
  HIP_TRY(hipSetDevice(b->device));
  if (b->total != h->m) {
    const int64_t offs[2] = {0, h->m};
    int rc = batch_layout(b, offs, 1);
    if (rc) return rc;
  }
  if (h->m > 0) {
    int rc = grow((void**)&h->pairs_d, &h->cap_pairs, h->m, sizeof(int2));
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(h->pairs_d, h->pairs_h.data(), (size_t)h->m * sizeof(int2), hipMemcpyHostToDevice, b->stream));
    HIP_TRY(picp_launch_gather(b->stream, h->world_d, h->image_d, h->pairs_d, h->m, b->X(), b->Y(), b->Z(), b->U(), b->V(), b->plane_off[0]));
  }
  HIP_TRY(hipStreamSynchronize(b->stream));
  h->gathered = true;
  return PICP_OK;
}

extern "C" int picp_set_correspondences(picp_t* h, const int32_t* pairs, int64_t m) {
  CHECK_ARG(h, "picp_set_correspondences: null handle");
  CHECK_ARG(m >= 0 && (m == 0 || pairs), "picp_set_correspondences: bad array");
  CHECK_ARG(m <= INT32_MAX, "picp_set_correspondences: too many correspondences");
  if (h->m == m && (m == 0 || memcmp(h->pairs_h.data(), pairs, (size_t)m * 2 * sizeof(int32_t)) == 0))
    return PICP_OK;  // same array as last time: keep the gathered planes
  if (!h->have_points) return set_err(PICP_ERR_STATE, "picp_set_correspondences: points not set");
  for (int64_t k = 0; k < m; ++k) {
    const int32_t ii = pairs[2 * k], wi = pairs[2 * k + 1];
    if (ii < 0 || ii >= h->n_image || wi < 0 || wi >= h->n_world)
      return set_err(PICP_ERR_RANGE, "correspondence %lld = (%d,%d) out of range (image %lld, world %lld)",
                     (long long)k, ii, wi, (long long)h->n_image, (long long)h->n_world);
  }
  h->pairs_h.assign(pairs, pairs + 2 * m);
  h->m = m;
  h->gathered = false;
  return PICP_OK;
}

extern "C" int picp_set_pose(picp_t* h, const float T[16]) {
  CHECK_ARG(h && T, "picp_set_pose: null argument");
  memcpy(h->pose, T, sizeof(h->pose));
  return PICP_OK;
}

extern "C" int picp_get_pose(picp_t* h, float T[16]) {
  CHECK_ARG(h && T, "picp_get_pose: null argument");
  memcpy(T, h->pose, sizeof(h->pose));
  return PICP_OK;
}

static int handle_upload_pose(picp_handle* h) {
  picp_batch* b = h->b;
  pose_to_state(h->pose, b->init_h[0]);
  HIP_TRY(hipMemcpyAsync(b->init_d, b->init_h.data(), sizeof(PicpState), hipMemcpyHostToDevice, b->stream));
  return PICP_OK;
}

extern "C" int picp_one_round(picp_t* h, float threshold, float damping, int min_inliers,
                              int keep_outliers, picp_stats* stats) {
  CHECK_ARG(h, "picp_one_round: null handle");
  int rc = handle_prepare(h);
  if (rc) return rc;
  picp_batch* b = h->b;
  picp_params prm;
  prm.threshold = threshold;
  prm.damping = damping;
  prm.min_inliers = min_inliers;
  prm.keep_outliers = keep_outliers;
  prm.max_rounds = 1;
  prm.conv_eps = -1.0f;  // the caller's loop owns the convergence test
  HIP_TRY(hipSetDevice(b->device));
  rc = batch_upload_params(b, &prm);
  if (rc) return rc;
  rc = handle_upload_pose(h);
  if (rc) return rc;
  HIP_TRY(graph_prologue(b));
  HIP_TRY(launch_round(b, 0));
  b->last_rounds = 1;
  b->result_idx = graph_result_idx(1);
  b->last_persistent = false;
  rc = batch_read_results(b);
  if (rc) return rc;
  const PicpState& s = b->result_h[0];
  if (stats) state_to_stats(s, *stats);
  if (!s.ok) return PICP_TOO_FEW_INLIERS;
  state_to_pose(s, h->pose);
  return PICP_OK;
}

extern "C" int picp_solve(picp_t* h, const picp_params* prm, picp_stats* stats) {
  CHECK_ARG(h && prm, "picp_solve: null argument");
  int rc = handle_prepare(h);
  if (rc) return rc;
  picp_batch* b = h->b;
  HIP_TRY(hipSetDevice(b->device));
  rc = handle_upload_pose(h);
  if (rc) return rc;
  rc = picp_batch_solve(b, prm);
  if (rc) return rc;
  const PicpState& s = b->result_h[0];
  if (stats) state_to_stats(s, *stats);
  state_to_pose(s, h->pose);
  return PICP_OK;
}

extern "C" int picp_linearize(picp_t* h, float threshold, int keep_outliers, double H[36],
                              double bvec[6], picp_stats* stats) {
  CHECK_ARG(h && H && bvec, "picp_linearize: null argument");
  int rc = handle_prepare(h);
  if (rc) return rc;
  picp_batch* b = h->b;
  picp_params prm;
  picp_params_default(&prm);
  prm.threshold = threshold;
  prm.keep_outliers = keep_outliers;
  prm.max_rounds = 1;
  prm.conv_eps = -1.0f;
  HIP_TRY(hipSetDevice(b->device));
  rc = batch_upload_params(b, &prm);
  if (rc) return rc;
  rc = handle_upload_pose(h);
  if (rc) return rc;
  HIP_TRY(graph_prologue(b));
  HIP_TRY(launch_round(b, 0));
  std::vector<float> part((size_t)b->nblk * PICP_NPART);  // the published words are float pairs
  HIP_TRY(hipMemcpyAsync(part.data(), b->part_d, part.size() * sizeof(float), hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  double tot[PICP_NPART] = {0};
  for (int k = 0; k < b->nblk; ++k)
    for (int e = 0; e < PICP_NPART; ++e) tot[e] += (double)part[(size_t)k * PICP_NPART + e];
  int idx = 0;
  for (int r = 0; r < 6; ++r)
    for (int c = r; c < 6; ++c) {
      H[c * 6 + r] = tot[PICP_P_H + idx];
      H[r * 6 + c] = tot[PICP_P_H + idx];
      ++idx;
    }
  for (int r = 0; r < 6; ++r) bvec[r] = tot[PICP_P_B + r];
  if (stats) {
    stats->chi_in = (float)tot[PICP_P_CHI_IN];
    stats->chi_out = (float)tot[PICP_P_CHI_OUT];
    stats->n_in = (int32_t)tot[PICP_P_N_IN];
    stats->n_projected = (int32_t)tot[PICP_P_N_PROJ];
    stats->ok = 1;
    stats->rounds = 0;
    stats->converged = 0;
    stats->reserved = 0;
  }
  return PICP_OK;
}

// ------------------------------------------------------------------------------------
// triangulation
// ------------------------------------------------------------------------------------
extern "C" int picp_projection_matrix(const float K[9], const float T_cw[16], float P[12]) {
  CHECK_ARG(K && T_cw && P, "picp_projection_matrix: null argument");
  // inverse of a rigid transform (Eigen Isometry3f::inverse), then K * [R|t]
  float Ri[9], ti[3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Ri[j * 3 + i] = T_cw[i * 4 + j];
  for (int i = 0; i < 3; ++i) {
    float s = Ri[0 * 3 + i] * T_cw[12 + 0];
    s = s + Ri[1 * 3 + i] * T_cw[12 + 1];
    s = s + Ri[2 * 3 + i] * T_cw[12 + 2];
    ti[i] = -s;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) {
      float m0 = (j < 3) ? Ri[j * 3 + 0] : ti[0];
      float m1 = (j < 3) ? Ri[j * 3 + 1] : ti[1];
      float m2 = (j < 3) ? Ri[j * 3 + 2] : ti[2];
      float s = K[0 * 3 + i] * m0;
      s = s + K[1 * 3 + i] * m1;
      s = s + K[2 * 3 + i] * m2;
      P[i * 4 + j] = s;
    }
  return PICP_OK;
}

extern "C" int picp_triangulate(int device, const float P1[12], const float P2[12],
                                const float* uv1, const float* uv2, int64_t q, float* xyz) {
  CHECK_ARG(P1 && P2, "picp_triangulate: null projection matrix");
  CHECK_ARG(q >= 0 && (q == 0 || (uv1 && uv2 && xyz)), "picp_triangulate: bad arrays");
  if (q == 0) return PICP_OK;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  CHECK_ARG(device >= 0 && device < ndev, "picp_triangulate: no such HIP device");
  HIP_TRY(hipSetDevice(device));
  const size_t bytes = 2 * 12 * sizeof(float) + (size_t)q * (2 + 2 + 3) * sizeof(float);
  char* buf = nullptr;
  HIP_TRY(hipMalloc(&buf, bytes));
  float* dP = (float*)buf;
  float* duv1 = dP + 24;
  float* duv2 = duv1 + 2 * q;
  float* dxyz = duv2 + 2 * q;
  hipError_t e = hipMemcpy(dP, P1, 12 * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dP + 12, P2, 12 * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(duv1, uv1, (size_t)q * 2 * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(duv2, uv2, (size_t)q * 2 * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = picp_launch_triangulate(nullptr, dP, dP + 12, (const float2*)duv1, (const float2*)duv2, q, dxyz);
  if (e == hipSuccess) e = hipMemcpy(xyz, dxyz, (size_t)q * 3 * sizeof(float), hipMemcpyDeviceToHost);
  hipFree(buf);
  if (e != hipSuccess) return set_err(PICP_ERR_DEVICE, "picp_triangulate: %s", hipGetErrorString(e));
  return PICP_OK;
}

// ------------------------------------------------------------------------------------
// essential-matrix bootstrap (src/cam.cpp:37-91: findEssentialMat + recoverPose)
// ------------------------------------------------------------------------------------
extern "C" void picp_essential_params_default(picp_essential_params* p) {
  if (!p) return;
  p->prob = 0.999;       // cv::findEssentialMat defaults (src/cam.cpp:49-54 passes none)
  p->threshold = 1.0;
  p->max_iters = 1000;
  p->dist = 50.0;        // cv::recoverPose distanceThresh default
}

extern "C" int picp_essential_batch(int device, int n_problems, const int64_t* offs, const float* p1,
                                    const float* p2, const float K[9], const picp_essential_params* prm,
                                    float* T_out, int32_t* inliers, int32_t* good, uint8_t* mask) {
  CHECK_ARG(n_problems >= 1 && offs && K && T_out && inliers && good, "picp_essential_batch: null argument");
  CHECK_ARG(offs[0] == 0, "picp_essential_batch: offsets must start at 0");
  for (int i = 0; i < n_problems; ++i)
    CHECK_ARG(offs[i + 1] >= offs[i] && offs[i + 1] - offs[i] <= INT32_MAX, "picp_essential_batch: bad offsets");
  const int64_t total = offs[n_problems];
  CHECK_ARG(total == 0 || (p1 && p2), "picp_essential_batch: null points");
  picp_essential_params dp;
  picp_essential_params_default(&dp);
  const picp_essential_params& P = prm ? *prm : dp;
  CHECK_ARG(P.max_iters >= 1 && P.max_iters <= 100000, "picp_essential_batch: max_iters out of range");
  CHECK_ARG(P.threshold > 0.0 && P.prob > 0.0 && P.prob < 1.0 && P.dist > 0.0, "picp_essential_batch: bad params");
  CHECK_ARG(K[0] != 0.0f && K[4] != 0.0f, "picp_essential_batch: K has a zero focal length");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  CHECK_ARG(device >= 0 && device < ndev, "picp_essential_batch: no such HIP device");
  HIP_TRY(hipSetDevice(device));
  EssArgs A;
  memset(&A, 0, sizeof(A));
  A.n_problems = n_problems;
  A.max_iters = P.max_iters;
  A.fx = K[0];  // column-major 3x3 (src/camera.h:45): K(0,0), K(1,1), K(0,2), K(1,2)
  A.fy = K[4];
  A.cx = K[6];
  A.cy = K[7];
  A.prob = P.prob;
  A.threshold = P.threshold;
  A.dist = P.dist;
  const size_t H = (size_t)n_problems * P.max_iters;
  const size_t pts = (size_t)std::max<int64_t>(total, 1) * 2 * sizeof(float);
  // one allocation carved into 256-byte-aligned sub-buffers (sizes rounded the same way)
  auto r256 = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t bytes = r256((size_t)(n_problems + 1) * 8) + 2 * r256(pts) + r256(H * 5 * 4) + r256(H * 90 * 8) +
                       r256(H * 4) + r256(H * 10 * 4) + r256((size_t)n_problems * 16 * 4) +
                       2 * r256((size_t)n_problems * 4) + r256((size_t)std::max<int64_t>(total, 1));
  char* buf = nullptr;
  HIP_TRY(hipMalloc(&buf, bytes));
  size_t at = 0;
  auto carve = [&](size_t b) { char* q = buf + at; at += r256(b); return q; };
  int64_t* d_offs = (int64_t*)carve((size_t)(n_problems + 1) * 8);
  float* d_p1 = (float*)carve(pts);
  float* d_p2 = (float*)carve(pts);
  int32_t* d_idx = (int32_t*)carve(H * 5 * 4);
  double* d_Es = (double*)carve(H * 90 * 8);
  int32_t* d_ns = (int32_t*)carve(H * 4);
  int32_t* d_cnt = (int32_t*)carve(H * 10 * 4);
  float* d_T = (float*)carve((size_t)n_problems * 16 * 4);
  int32_t* d_in = (int32_t*)carve((size_t)n_problems * 4);
  int32_t* d_good = (int32_t*)carve((size_t)n_problems * 4);
  uint8_t* d_mask = mask ? (uint8_t*)carve((size_t)std::max<int64_t>(total, 1)) : nullptr;
  hipError_t e = hipMemcpy(d_offs, offs, (size_t)(n_problems + 1) * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess && total > 0) e = hipMemcpy(d_p1, p1, (size_t)total * 2 * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess && total > 0) e = hipMemcpy(d_p2, p2, (size_t)total * 2 * sizeof(float), hipMemcpyHostToDevice);
  const char* stage = "upload";
  if (e == hipSuccess) {
    stage = "launch";
    e = picp_launch_essential(nullptr, &A, d_offs, d_p1, d_p2, d_idx, d_Es, d_ns, d_cnt, d_T, d_in, d_good, d_mask);
  }
  if (e == hipSuccess) {
    stage = "download T";
    e = hipMemcpy(T_out, d_T, (size_t)n_problems * 16 * 4, hipMemcpyDeviceToHost);
  }
  if (e == hipSuccess) {
    stage = "download inliers";
    e = hipMemcpy(inliers, d_in, (size_t)n_problems * 4, hipMemcpyDeviceToHost);
  }
  if (e == hipSuccess) {
    stage = "download good";
    e = hipMemcpy(good, d_good, (size_t)n_problems * 4, hipMemcpyDeviceToHost);
  }
  if (e == hipSuccess && mask && total > 0) {
    stage = "download mask";
    e = hipMemcpy(mask, d_mask, (size_t)total, hipMemcpyDeviceToHost);
  }
  hipFree(buf);
  if (e != hipSuccess) return set_err(PICP_ERR_DEVICE, "picp_essential_batch (%s): %s", stage, hipGetErrorString(e));
  return PICP_OK;
}

// ------------------------------------------------------------------------------------
// descriptor matching (match_points, src/my_utilities.h:70-120)
// ------------------------------------------------------------------------------------
extern "C" int picp_match_batch_form(int device, int n_problems, const int64_t* off1, const int64_t* off2,
                                     const float* desc1, const float* desc2, int dim, float dist_thr,
                                     float ratio_thr, int32_t* best_idx, float* best_dist,
                                     float* second_dist, int32_t* accepted, int form) {
  CHECK_ARG(form == PICP_MATCH_FORM_FULL || form == PICP_MATCH_FORM_ACCEPT_ONLY || form == PICP_MATCH_FORM_EXACT,
            "picp_match_batch_form: unknown form");
  CHECK_ARG(n_problems >= 1 && n_problems <= 65535 && off1 && off2, "picp_match_batch: bad problem table");
  CHECK_ARG(dim >= 1 && dim <= 32, "picp_match_batch: dim must be in [1, 32]");
  for (int i = 0; i < n_problems; ++i)
    CHECK_ARG(off1[0] == 0 && off2[0] == 0 && off1[i + 1] >= off1[i] && off2[i + 1] >= off2[i],
              "picp_match_batch: offsets must be prefix sums from 0");
  const int64_t n1 = off1[n_problems], n2 = off2[n_problems];
  CHECK_ARG((n1 == 0 || (desc1 && best_idx && best_dist && second_dist && accepted)) && (n2 == 0 || desc2),
            "picp_match_batch: null array");
  if (n1 == 0) return PICP_OK;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  CHECK_ARG(device >= 0 && device < ndev, "picp_match_batch: no such HIP device");
  HIP_TRY(hipSetDevice(device));
  std::vector<MatchProblem> probs((size_t)n_problems);
  int64_t max_nq = 0;
  for (int i = 0; i < n_problems; ++i) {
    probs[i] = MatchProblem{off1[i], off1[i + 1] - off1[i], off2[i], off2[i + 1] - off2[i]};
    max_nq = std::max(max_nq, probs[i].nq);
  }
  const size_t b_probs = probs.size() * sizeof(MatchProblem);
  const size_t b_d1 = (size_t)n1 * dim * sizeof(float), b_d2 = (size_t)std::max<int64_t>(n2, 1) * dim * sizeof(float);
  const size_t b_out = (size_t)n1 * 4;
  const int dp = 16 * picp_match_prep_kch(dim);
  const size_t n2a = (size_t)std::max<int64_t>(n2, 1);
  const size_t b_prep = ((size_t)n1 + n2a) * (dp * sizeof(_Float16) + 2 * sizeof(float));
  // the reference-range split's scratch (picp_match_ksplit: few problems against many references)
  int64_t max_nr = 0;
  for (const MatchProblem& q : probs) max_nr = std::max(max_nr, q.nr);
  // (form bit 2 for the split rule: the folded form needs dim <= 12)
  const int ks = picp_match_ksplit(n_problems, max_nq, max_nr, form | (dim <= 12 ? 4 : 0));
  const int64_t part_cap = picp_match_split_scratch(ks, n_problems, max_nq);
  const size_t b_part = (size_t)part_cap * sizeof(float4);
  char* buf = nullptr;
  HIP_TRY(hipMalloc(&buf, b_probs + b_d1 + b_d2 + 4 * b_out + b_prep + b_part + 512));
  char* cur = buf;
  auto carve = [&](size_t bytes) { char* r = cur; cur += (bytes + 15) / 16 * 16; return r; };
  MatchProblem* d_probs = (MatchProblem*)carve(b_probs);
  float* d_d1 = (float*)carve(b_d1);
  float* d_d2 = (float*)carve(b_d2);
  int32_t* d_bi = (int32_t*)carve(b_out);
  float* d_bd = (float*)carve(b_out);
  float* d_sd = (float*)carve(b_out);
  int32_t* d_acc = (int32_t*)carve(b_out);
  _Float16* q_h = (_Float16*)carve((size_t)n1 * dp * sizeof(_Float16));
  float* q_n1 = (float*)carve((size_t)n1 * 4);
  float* q_n2 = (float*)carve((size_t)n1 * 4);
  _Float16* r_h = (_Float16*)carve(n2a * dp * sizeof(_Float16));
  float* r_n1 = (float*)carve(n2a * 4);
  float* r_n2 = (float*)carve(n2a * 4);
  float4* d_part = ks > 1 ? (float4*)carve(b_part) : nullptr;
  hipError_t e = hipMemcpy(d_probs, probs.data(), b_probs, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_d1, desc1, b_d1, hipMemcpyHostToDevice);
  if (e == hipSuccess && n2) e = hipMemcpy(d_d2, desc2, (size_t)n2 * dim * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = picp_launch_match_prep(nullptr, d_d1, n1, dim, q_h, q_n1, q_n2);
  if (e == hipSuccess && n2) e = picp_launch_match_prep(nullptr, d_d2, n2, dim, r_h, r_n1, r_n2);
  if (e == hipSuccess)
    e = picp_launch_match_mfma(nullptr, n_problems, max_nq, d_d1, d_d2, q_h, q_n1, r_h, r_n1, r_n2, d_probs,
                               dim, dist_thr, ratio_thr, d_bi, d_bd, d_sd, d_acc, form, ks, d_part,
                               part_cap);
  if (e == hipSuccess) e = hipMemcpy(best_idx, d_bi, b_out, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(best_dist, d_bd, b_out, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(second_dist, d_sd, b_out, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(accepted, d_acc, b_out, hipMemcpyDeviceToHost);
  hipFree(buf);
  if (e != hipSuccess) return set_err(PICP_ERR_DEVICE, "picp_match_batch: %s", hipGetErrorString(e));
  return PICP_OK;
}

extern "C" int picp_match_batch(int device, int n_problems, const int64_t* off1, const int64_t* off2,
                                const float* desc1, const float* desc2, int dim, float dist_thr,
                                float ratio_thr, int32_t* best_idx, float* best_dist,
                                float* second_dist, int32_t* accepted) {
  return picp_match_batch_form(device, n_problems, off1, off2, desc1, desc2, dim, dist_thr, ratio_thr, best_idx,
                               best_dist, second_dist, accepted, PICP_MATCH_FORM_FULL);
}

extern "C" int picp_match(int device, const float* desc1, int64_t n1, const float* desc2, int64_t n2,
                          int dim, float dist_thr, float ratio_thr, int32_t* best_idx,
                          float* best_dist, float* second_dist, int32_t* accepted) {
  CHECK_ARG(n1 >= 0 && n2 >= 0, "picp_match: negative size");
  const int64_t o1[2] = {0, n1}, o2[2] = {0, n2};
  return picp_match_batch(device, 1, o1, o2, desc1, desc2, dim, dist_thr, ratio_thr, best_idx, best_dist,
                          second_dist, accepted);
}

// ------------------------------------------------------------------------------------
// self-test: the fast correctly rounded reciprocal of the projection (picp_device.h rcp_rn)
// ------------------------------------------------------------------------------------
extern "C" int picp_selftest_rcp(int device, int e_lo, int e_hi, uint64_t* mismatches) {
  CHECK_ARG(mismatches && e_lo >= -126 && e_hi <= 127 && e_lo < e_hi, "picp_selftest_rcp: bad argument");
  HIP_TRY(hipSetDevice(device));
  unsigned long long* d = nullptr;
  HIP_TRY(hipMalloc(&d, sizeof(unsigned long long)));
  hipError_t e = hipMemset(d, 0, sizeof(unsigned long long));
  const int64_t n = (int64_t)(e_hi - e_lo) << 24;
  if (e == hipSuccess) {
    hipLaunchKernelGGL(picp_rcp_check_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, e_lo, e_hi, d);
    e = hipGetLastError();
  }
  unsigned long long h = 0;
  if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
  hipFree(d);
  if (e != hipSuccess) return set_err(PICP_ERR_DEVICE, "picp_selftest_rcp: %s", hipGetErrorString(e));
  *mismatches = h;
  return PICP_OK;
}
