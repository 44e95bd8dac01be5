// picp_block.hip -- batched independent frames: ONE block per problem runs the whole
// exec/icp_test.cpp:88-107 loop.
//
// The first NPT*PICP_BBLOCK correspondences of a problem are loaded once into registers (NPT
// per lane); any remainder is re-read every round (two per lane per step, L2/MALL-resident
// after the first round).  Every round is: linearize in registers -> wave64 reduction (permlane/DPP) -> LDS
// combine of the 8 waves -> wave 0 finishes the round (fp32 LDL^T, Rx*Ry*Rz update,
// convergence; picp_device.h finish_round_pose, every lane the same values, the loop state in
// registers) -> barrier.  No inter-workgroup communication at all, no launch
// per round and no HBM re-read per round: a batch of frames is bound by VALU issue, not by
// hand-off latency or HBM.  Ragged batches read (offset, n) from the problem
// table.
//
// Split (split = 2 or 4): when S x the problems still fit on the chip (C4: 128 frames, 256 CUs),
// each problem runs on S blocks, each with 1/S of the correspondences, so no CU idles.  Per
// round each block publishes its 32-term partial as 64 granules {round, hi|lo} (the double sum
// as hi = (float)t, lo = (float)(t - hi)), polls its S - 1 partners', and all add the parts in
// part order: every part runs the identical solve, so no broadcast is needed.  Partners are
// blockIdx b, b + 8, b + 16, ... which round-robin placement puts on the same XCD (speed only:
// correctness rests on the tags).  Granules are double-buffered by round parity; their tags
// continue from per-slot tag bases the previous launch left, so the sync area is zeroed only once
// per layout (and before the tags could wrap), not per launch.  Every wait has an s_memrealtime
// deadline, refreshed each round (error word set, the problem stops, the host reports it and
// re-runs the solve in graph mode).  The host launches a split grid only when the occupancy query
// below says every block is resident at once.
// split = 4 runs two 512-thread blocks per CU from DIFFERENT problems (<= 128 VGPRs each): while
// one problem's parts exchange and solve (the CU idle in split = 2), the other's compute.
#include <type_traits>

#include "picp_vo_device.h"

using namespace picp;

#define PICP_BBLOCK 512  // 8 waves: 2 per SIMD at <= 256 VGPRs (split 1, 2); 4 per SIMD for split 4
#define PICP_BLDS_ITEMS 7680  // items staged in LDS: 5 x 4 B x 7680 = 150 KB of the 160 KB per CU
// partner polls run back to back: an s_sleep 1 between polls measured C4 1704-1711 us vs
// 1700-1706 us without it, 4 of 4 interleaved reps (profiles/r02/e4/ab_bspin.log).
#define PICP_XG 64            // exchange granules per block per round: 32 hi + 32 lo

typedef __attribute__((address_space(1))) unsigned long long bgu64_t;

// Diagnostic build only (-DPICP_STAMPS): s_memrealtime per phase of rounds 11 and 12 seen by
// thread 0 of blocks < 1024, and where each block ran (words 7, 8: HW_REG_XCC_ID, HW_REG_HW_ID)
// (tools/bstamps.py).
#ifdef PICP_STAMPS
#define PICP_BSTAMP_BLOCKS 1024
__device__ unsigned long long picp_bstamps[2][PICP_BSTAMP_BLOCKS][10];
#define BSTAMP(k)                                                                               \
  do {                                                                                          \
    if (threadIdx.x == 0 && (round == 11 || round == 12) && blockIdx.x < PICP_BSTAMP_BLOCKS)     \
      picp_bstamps[round - 11][blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();                \
  } while (0)
#define BSTAMP_PLACE()                                                                          \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < PICP_BSTAMP_BLOCKS) {                                   \
      unsigned xcc, hwid;                                                                       \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));                       \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));                       \
      picp_bstamps[0][blockIdx.x][7] = picp_bstamps[1][blockIdx.x][7] = xcc;                    \
      picp_bstamps[0][blockIdx.x][8] = picp_bstamps[1][blockIdx.x][8] = hwid;                   \
    }                                                                                           \
  } while (0)
extern "C" hipError_t picp_debug_bstamps(unsigned long long* out, size_t n_words) {
  const size_t cap = sizeof(picp_bstamps) / sizeof(unsigned long long);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(picp_bstamps), (n_words < cap ? n_words : cap) * 8, 0,
                             hipMemcpyDeviceToHost);
}
#else
#define BSTAMP(k) ((void)0)
#define BSTAMP_PLACE() ((void)0)
#endif

// The VO step's gather fused into the block kernel (VoT = VoArgs; the separate kernel is
// vo_gather_kernel, picp_vo.hip, which this restates): the next frame's observations that the
// world match accepted, compacted in observation order, become the block's items directly --
// items below NPT*BS into the registers (item o -> lane o % BS, slot o / BS, through an LDS
// slice of VOG_SLICE items per pass), the rest into the LDS stage -- instead of a kernel writing the SoA planes
// and this one reading them back.  Items past n take the last item's values as the plane loads'
// clamp did.  Needs n <= NPT*BS + lds_items and frames of <= VOG_CHUNKS*BS observations (the
// host's check).  Writes a.probs[s] (the append reads n) and returns n.
struct NoVo {};
#define VOG_CHUNKS 8  // observation chunks of BS held in registers: 4096 at BS 512
#define VOG_SLICE 256  // items per pass of the register transfer
template <int NPT, int BS>
__device__ __forceinline__ int vo_gather_items(const VoArgs& a, int s, int t, float* xs, float* ys, float* zs,
                                               float* us, float* vs, float* lx, float* ly, float* lz,
                                               float* lu, float* lv, int lds_items) {
  constexpr int NW = BS / 64;
  __shared__ int s_wc[VOG_CHUNKS][NW];          // flagged observations per (chunk, wave)
  __shared__ float s_sl[5][VOG_SLICE];          // the items of one pass
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const VoSegment G = a.segs[s];
  const int64_t base = (int64_t)s * a.cap_c;
  int64_t nn = 0, on = 0;
  if (t < G.steps) {  // a finished segment: an empty problem (its result is never read)
    on = a.frame_off[G.f0 + t + 1];
    nn = a.frame_off[G.f0 + t + 2] - on;
  }
  // every chunk's loads first (accept flag, map index, pixel; then the map point)
  bool fl[VOG_CHUNKS];
  int jb[VOG_CHUNKS];
  float px[VOG_CHUNKS], py[VOG_CHUNKS], pz[VOG_CHUNKS];
  float2 pu[VOG_CHUNKS];
#pragma unroll
  for (int c = 0; c < VOG_CHUNKS; ++c) {
    const int64_t i = (int64_t)c * BS + tid;
    fl[c] = i < nn && a.wm_acc[on + i] != 0;
    jb[c] = (i < nn) ? a.wm_bi[on + i] : 0;
    pu[c] = (i < nn) ? a.uv[on + i] : make_float2(0.0f, 0.0f);
  }
#pragma unroll
  for (int c = 0; c < VOG_CHUNKS; ++c) {
    const int64_t j = G.map_off + (fl[c] ? jb[c] : 0);
    px[c] = fl[c] ? a.map_xyz[3 * j + 0] : 0.0f;
    py[c] = fl[c] ? a.map_xyz[3 * j + 1] : 0.0f;
    pz[c] = fl[c] ? a.map_xyz[3 * j + 2] : 0.0f;
  }
  // the ordered compaction of all chunks with one barrier: per (chunk, wave) counts, then each
  // flagged observation's output index = flagged before its chunk + before its wave + its lane rank
  int rk[VOG_CHUNKS];
#pragma unroll
  for (int c = 0; c < VOG_CHUNKS; ++c) {
    const unsigned long long m = __ballot(fl[c]);
    rk[c] = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_wc[c][w] = __popcll(m);
  }
  __syncthreads();
  int n = 0;
#pragma unroll
  for (int c = 0; c < VOG_CHUNKS; ++c) {
    int pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      pre += (k < w) ? s_wc[c][k] : 0;
      tot += s_wc[c][k];
    }
    rk[c] += n + pre;
    n += tot;
  }
  // items past the registers go straight to the LDS stage
  const int r0 = NPT * BS;
#pragma unroll
  for (int c = 0; c < VOG_CHUNKS; ++c)
    if (fl[c] && rk[c] >= r0 && rk[c] - r0 < lds_items) {
      const int o = rk[c] - r0;
      lx[o] = px[c];
      ly[o] = py[c];
      lz[o] = pz[c];
      lu[o] = pu[c].x;
      lv[o] = pu[c].y;
    }
  // register slot k = o / BS: the items pass by pass through an LDS slice of VOG_SLICE items
  // (five planes of 5 KB: beside this block a CU still holds four matcher blocks); lanes whose
  // slot is past item n - 1 take that item's values (the plane loads' clamp)
  const int last = max(n - 1, 0);
  const int qlast = last / VOG_SLICE;
  float lastv[5];
  for (int q = 0; q <= qlast && q * VOG_SLICE < NPT * BS; ++q) {  // uniform: n is the block's
#pragma unroll
    for (int c = 0; c < VOG_CHUNKS; ++c)
      if (fl[c] && rk[c] / VOG_SLICE == q) {
        const int o = rk[c] - q * VOG_SLICE;
        s_sl[0][o] = px[c];
        s_sl[1][o] = py[c];
        s_sl[2][o] = pz[c];
        s_sl[3][o] = pu[c].x;
        s_sl[4][o] = pu[c].y;
      }
    __syncthreads();
    constexpr int HPS = BS / VOG_SLICE;  // passes per register slot
    const int k = q / HPS, o = tid - (q % HPS) * VOG_SLICE;
#pragma unroll
    for (int kk = 0; kk < NPT; ++kk)  // register-indexed writes unrolled into selects
      if (kk == k && o >= 0 && o < VOG_SLICE) {
        xs[kk] = s_sl[0][o];
        ys[kk] = s_sl[1][o];
        zs[kk] = s_sl[2][o];
        us[kk] = s_sl[3][o];
        vs[kk] = s_sl[4][o];
      }
    if (q == qlast) {  // no item at all (n == 0): zeros, never the slice's unwritten words
#pragma unroll
      for (int v = 0; v < 5; ++v) lastv[v] = (n > 0) ? s_sl[v][last - q * VOG_SLICE] : 0.0f;
    }
    __syncthreads();
  }
  if (qlast * VOG_SLICE >= NPT * BS) {  // item n - 1 is in the LDS stage
    lastv[0] = lx[last - NPT * BS];
    lastv[1] = ly[last - NPT * BS];
    lastv[2] = lz[last - NPT * BS];
    lastv[3] = lu[last - NPT * BS];
    lastv[4] = lv[last - NPT * BS];
  }
#pragma unroll
  for (int k = 0; k < NPT; ++k)
    if (k * BS + tid > last) {
      xs[k] = lastv[0];
      ys[k] = lastv[1];
      zs[k] = lastv[2];
      us[k] = lastv[3];
      vs[k] = lastv[4];
    }
  if (tid == 0) a.probs[s] = PicpProblem{base, (int32_t)n, 0, 1, 0};
  return n;
}

// Issue priority of a block's waves by phase (on by default; -DPICP_BPRIO=0 for A/B): the round's
// tail (the wave reduction, the combine and partner exchange, the one-wave solve) is a dependency
// chain; when a second block shares the CU (split 4), its linearize would take the SIMDs' issue
// slots ahead of it.  C4 at 128 frames, split 4: 20.4M -> 22.9M it/s; split 2 and the VO step
// kernel within noise (profiles/r04/c4_128/, profiles/r04/pair2/).
#ifndef PICP_BPRIO
#define PICP_BPRIO 1
#endif
#if PICP_BPRIO
#define BPRIO_TAIL() __builtin_amdgcn_s_setprio(3)
#define BPRIO_LIN() __builtin_amdgcn_s_setprio(0)
#else
#define BPRIO_TAIL() ((void)0)
#define BPRIO_LIN() ((void)0)
#endif

// MINW: waves per SIMD the register budget must allow (2: <= 256 VGPRs, one 512-thread block per
// CU; 4: <= 128 VGPRs, two 512-thread blocks per CU -- split 4's layout)
template <int NPT, int PH, int BS, typename VoT = NoVo, int MINW = 2>
__global__ __launch_bounds__(BS, MINW) void picp_block_kernel(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const float* __restrict__ U, const float* __restrict__ V, const PicpArgs A,
    const PicpProblem* __restrict__ probs, const PicpState* __restrict__ st_in,
    PicpState* __restrict__ st_out, int lds_items, int split, int n_problems,
    unsigned long long* xg, unsigned int* err, unsigned int* tagbase, unsigned long long timeout_ticks,
    const VoT vo, int vo_t) {
  constexpr bool VOG = std::is_same<VoT, VoArgs>::value;  // the VO step's gather fused in
  BSTAMP_PLACE();
  extern __shared__ float s_lds[];  // [5][lds_items]: the problem's items past the registers
  // wave sums, term-major: the lane combining term e reads its BS/64 wave sums as 16-B loads
  __shared__ __attribute__((aligned(16))) float s_wave[PICP_NPART][BS / 64];
  __shared__ float s_tot[PICP_NPART];  // the totals as finish_round_f words (total_word)
  __shared__ float s_pose[12];
  __shared__ int s_done;
  __shared__ int s_tmo;  // a partner wait timed out (the error word is for the host)
  __shared__ PicpState s_st;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int p = blockIdx.x, h = 0;
  if (split > 1) {  // partners b + 8k (same XCD); h = which part of the problem
    const int s = (int)blockIdx.x >> 3;
    h = s % split;
    p = (s / split) * 8 + ((int)blockIdx.x & 7);
    if (p >= n_problems) return;  // grid padding (whole partner groups only)
  }
  int64_t base = 0;
  int n = 0;
  if constexpr (VOG) {
    // set by vo_gather_items below (split is 1)
  } else if (A.uniform) {
    base = (int64_t)p * A.stride_u;
    n = A.n_u;
  } else {
    const PicpProblem P = probs[p];
    base = P.offset;
    n = P.n;
  }
  if (split > 1) {  // parts start on a multiple of 4 (the planes' alignment)
    const int part = (((n + split - 1) / split) + 3) & ~3;
    const int first = min(n, h * part);
    n = min(n, first + part) - first;
    if (n > 0) base += first;  // an empty part keeps a valid base (its loads are clamped to it)
  }
  bgu64_t* const xgg = (bgu64_t*)xg;
  // split: exchange tags are tbase + round, tbase = the rounds this grid slot ran in earlier
  // launches on these buffers (partners run identical solves, so their bases stay equal); stale
  // granules never match and no memset has to clear them between launches
  const unsigned tbase = (split > 1) ? tagbase[blockIdx.x] : 0u;
  int last_round = 0;

  // the problem, loaded once into registers (coalesced: item = tid + k*BLOCK)
  float xs[NPT], ys[NPT], zs[NPT], us[NPT], vs[NPT];
  // items NPT*BLOCK .. NPT*BLOCK + n_lds - 1 are staged in LDS once (read every round at LDS
  // latency); any beyond that are streamed from L2/MALL every round
  const int r0 = NPT * BS;
  float* lx = s_lds;
  float* ly = s_lds + lds_items;
  float* lz = s_lds + 2 * lds_items;
  float* lu = s_lds + 3 * lds_items;
  float* lv = s_lds + 4 * lds_items;
  if constexpr (VOG) {
    const int s = vo.seg0 + p;
    base = (int64_t)s * vo.cap_c;
    n = vo_gather_items<NPT, BS>(vo, s, vo_t, xs, ys, zs, us, vs, lx, ly, lz, lu, lv, lds_items);
  } else {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int ic = min(tid + k * BS, max(n - 1, 0));
      xs[k] = X[base + ic];
      ys[k] = Y[base + ic];
      zs[k] = Z[base + ic];
      us[k] = U[base + ic];
      vs[k] = V[base + ic];
    }
  }
  const int n_lds = max(0, min(n - r0, lds_items));
  for (int i = tid; i < n_lds && !VOG; i += BS) {
    lx[i] = X[base + r0 + i];
    ly[i] = Y[base + r0 + i];
    lz[i] = Z[base + r0 + i];
    lu[i] = U[base + r0 + i];
    lv[i] = V[base + r0 + i];
  }

  if (tid == 0) {  // initial state (as launch 0 of the multi-launch path)
    PicpState s = st_in[p];
    s.chi_prev = FLT_MAX;  // exec/icp_test.cpp:89
    s.chi_in = s.chi_out = 0.0f;
    s.n_in = s.n_proj = 0;
    s.rounds = 0;
    s.done = (A.max_rounds <= 0) ? 1 : 0;
    s.ok = 1;
    s.converged = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) s_pose[i] = s.R[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) s_pose[9 + i] = s.t[i];
    s_done = s.done;
    s_tmo = 0;
    s_st = s;
  }
  __syncthreads();

  Cam C;
  C.k00 = A.K[0]; C.k10 = A.K[1]; C.k20 = A.K[2];
  C.k01 = A.K[3]; C.k11 = A.K[4]; C.k21 = A.K[5];
  C.k02 = A.K[6]; C.k12 = A.K[7]; C.k22 = A.K[8];
  C.maxx = A.maxx;
  C.maxy = A.maxy;
  const float thr = A.threshold;
  const float inv_thr = 1.0f / thr;
  const bool keep = A.keep_outliers != 0;

  // the icp_test loop state a round reads: the pose (s_pose, every wave) and chi_prev (wave 0,
  // which finishes the rounds, keeps it in a register)
  float chi_prev = FLT_MAX;  // exec/icp_test.cpp:89
  for (int round = 1; !s_done; ++round) {
    BSTAMP(0);
    BPRIO_LIN();
    Pose T;
    T.r00 = s_pose[0]; T.r10 = s_pose[1]; T.r20 = s_pose[2];
    T.r01 = s_pose[3]; T.r11 = s_pose[4]; T.r21 = s_pose[5];
    T.r02 = s_pose[6]; T.r12 = s_pose[7]; T.r22 = s_pose[8];
    T.t0 = s_pose[9]; T.t1 = s_pose[10]; T.t2 = s_pose[11];
    // accumulation form by register-resident items per lane (picp_device.h acc_pairs): two slots
    // for NPT 8, one slot below
    float v[PICP_NPART];
    Cnt nr = {0u, 0u}, nd = {0u, 0u};  // counts: register items (uniform), divergent loops (lane 0)
    if constexpr (acc_pairs(NPT)) {
      Acc2 a;
      acc2_zero(a);
      accumulate_regs<PH, NPT>(T, C, thr, inv_thr, keep, xs, ys, zs, us, vs, tid, BS, n, a, nr);
      for (int i = tid; i < n_lds; i += 2 * BS) {  // LDS-staged items, in pairs
        const int i2 = min(i + BS, n_lds - 1);
        // scalar locals first: building the f2 operands from the LDS reads directly made the
        // compiler round-trip them through scratch every round
        const float x0 = lx[i], y0 = ly[i], z0 = lz[i], u0 = lu[i], v0 = lv[i];
        const float x1 = lx[i2], y1 = ly[i2], z1 = lz[i2], u1 = lu[i2], v1 = lv[i2];
        accumulate2<PH>(T, C, thr, inv_thr, keep, (f2){x0, x1}, (f2){y0, y1}, (f2){z0, z1}, (f2){u0, u1},
                        (f2){v0, v1}, true, i + BS < n_lds, a, nd);
      }
      for (int i = r0 + n_lds + tid; i < n; i += 2 * BS) {  // streamed remainder
        const int i2 = min(i + BS, n - 1);
        const float x0 = X[base + i], y0 = Y[base + i], z0 = Z[base + i], u0 = U[base + i], v0 = V[base + i];
        const float x1 = X[base + i2], y1 = Y[base + i2], z1 = Z[base + i2], u1 = U[base + i2], v1 = V[base + i2];
        accumulate2<PH>(T, C, thr, inv_thr, keep, (f2){x0, x1}, (f2){y0, y1}, (f2){z0, z1}, (f2){u0, u1},
                        (f2){v0, v1}, true, i + BS < n, a, nd);
      }
      BSTAMP(1);
      acc2_fold(a, v);
    } else {
      Acc a;
      acc_zero(a);
      accumulate_regs1<PH, NPT>(T, C, thr, inv_thr, keep, xs, ys, zs, us, vs, tid, BS, n, a, nr);
      accumulate_stream1<PH>(T, C, thr, inv_thr, keep, tid, BS, n_lds,  // LDS-staged items
                             [&](int i, float& x, float& y, float& z, float& u, float& v) {
                               x = lx[i]; y = ly[i]; z = lz[i]; u = lu[i]; v = lv[i];
                             }, a, nd);
      accumulate_stream1<PH>(T, C, thr, inv_thr, keep, r0 + n_lds + tid, BS, n,  // streamed remainder
                             [&](int i, float& x, float& y, float& z, float& u, float& v) {
                               x = X[base + i]; y = Y[base + i]; z = Z[base + i]; u = U[base + i]; v = V[base + i];
                             }, a, nd);
      BSTAMP(1);
      acc_fold(a, v);
    }
    BPRIO_TAIL();
    const float wred = wave_reduce32(v, lane);
    const float wsum = wave_counts(wred, lane, (Cnt){nr.n_in + nd.n_in, nr.n_proj + nd.n_proj});
    if ((lane & 1) == 0) s_wave[lane >> 1][wave] = wsum;
    BSTAMP(2);
    __syncthreads();
    BSTAMP(3);
    // the finishing wave's pose, re-read here (three 16-B LDS loads, landing during the combine)
    // rather than kept live through the linearize, where it spilled; s_pose changes only after
    // this round's finish
    float pr[9], pt[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) pr[i] = s_pose[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) pt[i] = s_pose[9 + i];
    if (tid < PICP_NPART) {  // fixed-order combine of the 8 waves, one lane per term
      float ws[BS / 64];  // every load issued before the first add (one LDS wait)
#pragma unroll
      for (int w = 0; w < BS / 64; ++w) ws[w] = s_wave[tid][w];
      double t = (double)ws[0];
#pragma unroll
      for (int w = 1; w < BS / 64; ++w) t += (double)ws[w];
      if (split > 1) {
        // publish {round, hi}, {round, lo}; poll the partners'; add the parts in part order
        const float hi = (float)t, lo = (float)(t - (double)hi);
        const size_t slot = (size_t)(round & 1) * gridDim.x;
        bgu64_t* mine = xgg + (slot + blockIdx.x) * PICP_XG;
        const unsigned tag = tbase + (unsigned)round;
        __hip_atomic_store(mine + tid, ((unsigned long long)tag << 32) | __float_as_uint(hi),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(mine + PICP_NPART + tid, ((unsigned long long)tag << 32) | __float_as_uint(lo),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + timeout_ticks;
        const unsigned g0 = ((blockIdx.x >> 3) / (unsigned)split) * (unsigned)split;  // part 0's group
        double part_t[4];
        unsigned pending = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          part_t[q] = 0.0;
          if (q < split && q != h) pending |= 1u << q;
        }
        part_t[h & 3] = (double)hi + (double)lo;
        for (;;) {
          // every partner's two granules loaded before any tag is checked (the partners are a
          // block-uniform set, so the loads issue back to back): one round trip per poll.  Checking
          // each partner right after its loads (round 3's form) waited one round trip per
          // partner, three per poll at split 4.
          unsigned long long gh[4], gl[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            gh[q] = gl[q] = 0ull;
            if (q < split && q != h) {
              const bgu64_t* theirs = xgg + (slot + (((g0 + q) << 3) | (blockIdx.x & 7u))) * PICP_XG;
              gh[q] = __hip_atomic_load(theirs + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              gl[q] = __hip_atomic_load(theirs + PICP_NPART + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if ((pending & (1u << q)) && (unsigned)(gh[q] >> 32) == tag && (unsigned)(gl[q] >> 32) == tag) {
              part_t[q] = (double)__uint_as_float((unsigned)gh[q]) + (double)__uint_as_float((unsigned)gl[q]);
              pending &= ~(1u << q);
            }
          }
          if (!pending) break;
          if (__builtin_amdgcn_s_memrealtime() > deadline) {
            __hip_atomic_store(err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_tmo = 1;
            break;
          }
        }
        t = part_t[0];
#pragma unroll
        for (int q = 1; q < 4; ++q)
          if (q < split) t += part_t[q];
      }
      s_tot[tid] = total_word(A, tid, t);  // lane e converts total e
    }
    // the totals (and s_tmo) were written by lanes < 32 of wave 0, which also runs the solve:
    // a wave barrier orders them, the other waves wait at the block barrier after the solve
#ifdef PICP_FINISH_SYNC
    __syncthreads();
#else
    __builtin_amdgcn_wave_barrier();
#endif
    BSTAMP(4);
    if (wave == 0) {  // the wave finishes the round (every lane the same values, state in registers)
      RoundOut o;
      finish_round_pose<PICP_FINISH_WAVE>(A, s_tot, round, pr, pt, chi_prev, o);
      if (s_tmo) o.done = 1;  // a partner wait timed out: stop (the host reports the error)
      if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 9; ++i) s_pose[i] = pr[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) s_pose[9 + i] = pt[i];
        s_done = o.done;
        if (o.done) store_state(&s_st, pr, pt, chi_prev, o, round);
      }
    }
    BSTAMP(5);
    last_round = round;
    __syncthreads();
    BSTAMP(6);
  }
  // every partner read its base before publishing round 1, and has finished its last round
  if (split > 1 && tid == 0) tagbase[blockIdx.x] = tbase + (unsigned)last_round;
  if (h == 0 && tid < 32)
    reinterpret_cast<int32_t*>(&st_out[p])[tid] = reinterpret_cast<const int32_t*>(&s_st)[tid];
}

extern "C" int picp_block_max_items(void) { return 8 * PICP_BBLOCK; }  // register-resident part (BS 512)

// Threads per block: 512 for every split; split 4 runs two blocks per CU (two waves per SIMD each,
// <= 128 VGPRs: MINW 4).  256-thread split-4 parts (round 1) measured 5-7 % slower
// (profiles/r01/c4_split4_ab.log, profiles/r04/c4_128/).
extern "C" int picp_block_threads(int split) { return (void)split, PICP_BBLOCK; }

// dynamic LDS of a launch: the part of a problem (or of its 1/split share) past the
// register-resident npt x BS items, capped by the stage
static size_t block_lds_bytes(int npt, int split, int max_n, int* lds_items_out) {
  const int per_block = (split > 1) ? ((((max_n + split - 1) / split) + 3) & ~3) : max_n;
  const int bs = picp_block_threads(split);
  const int lds_cap = (split == 4) ? PICP_BLDS_ITEMS / 2 : PICP_BLDS_ITEMS;  // two blocks share a CU's LDS
  const int lds_items = (per_block > npt * bs) ? min(per_block - npt * bs, lds_cap) : 0;
  if (lds_items_out) *lds_items_out = lds_items;
  return (size_t)5 * lds_items * sizeof(float);
}

// the kernel of a launch: waves per SIMD 2 (split 1, 2) or split 4's 4
template <int N, int W>
static const void* block_kernel_nw(int var) {
  switch (var) {
    case PICP_V_PINHOLE: return (const void*)picp_block_kernel<N, PICP_V_PINHOLE, PICP_BBLOCK, NoVo, W>;
    case PICP_V_PINHOLE_KEEP: return (const void*)picp_block_kernel<N, PICP_V_PINHOLE_KEEP, PICP_BBLOCK, NoVo, W>;
    default: return (const void*)picp_block_kernel<N, PICP_V_GENERAL, PICP_BBLOCK, NoVo, W>;
  }
}

template <int N>
static const void* block_kernel_n(int var, int split) {
  if (split == 4) {
    if constexpr (N <= 4) return block_kernel_nw<N, 4>(var);  // <= 128 VGPRs: NPT <= 4
    return nullptr;
  }
  return block_kernel_nw<N, 2>(var);
}

static const void* block_kernel_ptr(int npt, int var, int split) {
  switch (npt) {
    case 1: return block_kernel_n<1>(var, split);
    case 2: return block_kernel_n<2>(var, split);
    case 4: return block_kernel_n<4>(var, split);
    case 8: return block_kernel_n<8>(var, split);
    default: return nullptr;
  }
}

// Register items per lane the split-4 layout allows (its 128-VGPR budget); 8 otherwise.
extern "C" int picp_block_npt_cap(int split) { return (split == 4) ? 4 : 8; }

// Blocks of the variants a launch with these arguments may use that one CU holds at once (the
// hardware limit from registers, LDS and waves; other work on the device is not counted; the
// smaller of the two pinhole variants, since keep_outliers is a per-solve argument).  The host
// multiplies by the CU count and launches a split grid (whose blocks wait on each other) only if
// the whole grid fits.
extern "C" hipError_t picp_block_occupancy(int npt, int split, int max_n, const float K[9], int* blocks_per_cu) {
  if (!blocks_per_cu || (split != 1 && split != 2 && split != 4)) return hipErrorInvalidValue;
  const int bs = picp_block_threads(split);
  const size_t lds_bytes = block_lds_bytes(npt, split, max_n, nullptr);
  int best = -1;
  for (int keep = 0; keep < 2; ++keep) {
    const void* fn = block_kernel_ptr(npt, picp_variant(K, keep), split);
    if (!fn) return hipErrorInvalidValue;
    if (lds_bytes > 65536) {
      hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
      if (e != hipSuccess) return e;
    }
    int occ = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, bs, lds_bytes);
    if (e != hipSuccess) return e;
    best = (best < 0 || occ < best) ? occ : best;
  }
  *blocks_per_cu = best;
  return hipSuccess;
}

// max_n: the largest problem of the launch (sizes the LDS stage: max_n/split - npt*BS items,
// capped).  split = 1: grid = n_problems blocks of 512.  split = 2: grid = round_up(2 n_problems,
// 16) blocks of 512, one per CU; split = 4: grid = round_up(4 n_problems, 32) blocks of 512, two
// per CU; all co-resident (the caller checks the grid against the
// CUs), xg = 2 * grid * 64 u64 granules, tagbase = grid u32 tag bases (both zeroed once per
// layout), err the error word.
extern "C" hipError_t picp_launch_block(hipStream_t stream, int n_problems, int npt, const float* X,
                                        const float* Y, const float* Z, const float* U,
                                        const float* V, const PicpArgs* args,
                                        const PicpProblem* probs, const PicpState* st_in,
                                        PicpState* st_out, int max_n, int split,
                                        unsigned long long* xg, unsigned int* err,
                                        unsigned int* tagbase, unsigned long long timeout_ticks) {
  if (n_problems <= 0 || !args || (split != 1 && split != 2 && split != 4)) return hipErrorInvalidValue;
  if (split > 1 && (!xg || !err || !tagbase)) return hipErrorInvalidValue;
  const int grid = (split > 1) ? ((split * n_problems + 8 * split - 1) / (8 * split)) * (8 * split) : n_problems;
  const int var = picp_variant(args->K, args->keep_outliers);
  const int bs = picp_block_threads(split);
  const void* fn = block_kernel_ptr(npt, var, split);
  if (!fn) return hipErrorInvalidValue;
  int lds_items = 0;
  const size_t lds_bytes = block_lds_bytes(npt, split, max_n, &lds_items);
  if (lds_bytes > 65536) hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
  NoVo novo{};
  int zero = 0;
  void* kargs[] = {(void*)&X, (void*)&Y, (void*)&Z, (void*)&U, (void*)&V, (void*)args, (void*)&probs,
                   (void*)&st_in, (void*)&st_out, (void*)&lds_items, (void*)&split, (void*)&n_problems,
                   (void*)&xg, (void*)&err, (void*)&tagbase, (void*)&timeout_ticks, (void*)&novo, (void*)&zero};
  hipError_t e = hipLaunchKernel(fn, dim3(grid), dim3(bs), kargs, lds_bytes, stream);
  return (e != hipSuccess) ? e : hipGetLastError();
}

// The VO step's PICP with its gather fused in (vo_gather_items): segments a->seg0 .. + n_seg of
// step t, one 512-thread block each, npt register items per lane and the LDS stage sized for
// max_obs (every item of a frame of <= max_obs observations is on-chip).  The caller checks
// picp_vo_block_fusable(npt, max_obs) first; otherwise it runs vo_gather_kernel + the plain launch.
extern "C" int picp_vo_block_fusable(int npt, int64_t max_obs) {
  int lds_items = 0;
  block_lds_bytes(npt, 1, (int)max_obs, &lds_items);
  return max_obs <= (int64_t)VOG_CHUNKS * PICP_BBLOCK && max_obs <= (int64_t)npt * PICP_BBLOCK + lds_items &&
         (npt == 1 || npt == 2 || npt == 4 || npt == 8);
}

extern "C" hipError_t picp_launch_vo_block(hipStream_t stream, const VoArgs* a, int t, int npt,
                                           const PicpArgs* args, int64_t max_obs) {
  if (!a || !args || a->n_seg <= 0 || !picp_vo_block_fusable(npt, max_obs)) return hipErrorInvalidValue;
  int lds_items = 0;
  const size_t lds_bytes = block_lds_bytes(npt, 1, (int)max_obs, &lds_items);
  const int var = picp_variant(args->K, args->keep_outliers);
#define PICP_LAUNCH_VB3(N, P)                                                                              \
  {                                                                                                        \
    if (lds_bytes > 65536)                                                                                 \
      hipFuncSetAttribute((const void*)picp_block_kernel<N, P, PICP_BBLOCK, VoArgs>,                       \
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);                     \
    hipLaunchKernelGGL((picp_block_kernel<N, P, PICP_BBLOCK, VoArgs>), dim3(a->n_seg), dim3(PICP_BBLOCK),  \
                       lds_bytes, stream, a->X, a->Y, a->Z, a->U, a->V, *args, a->probs + a->seg0,          \
                       a->st_in + a->seg0, (PicpState*)a->st_out + a->seg0, lds_items, 1, a->n_seg,         \
                       nullptr, nullptr, nullptr, 0ull, *a, t);                                            \
  }
#define PICP_LAUNCH_VB(N)                                                        \
  if (var == PICP_V_PINHOLE) PICP_LAUNCH_VB3(N, PICP_V_PINHOLE)                   \
  else if (var == PICP_V_PINHOLE_KEEP) PICP_LAUNCH_VB3(N, PICP_V_PINHOLE_KEEP)    \
  else PICP_LAUNCH_VB3(N, PICP_V_GENERAL)
  switch (npt) {
    case 1: PICP_LAUNCH_VB(1); break;
    case 2: PICP_LAUNCH_VB(2); break;
    case 4: PICP_LAUNCH_VB(4); break;
    case 8: PICP_LAUNCH_VB(8); break;
    default: return hipErrorInvalidValue;
  }
#undef PICP_LAUNCH_VB
#undef PICP_LAUNCH_VB3
  return hipGetLastError();
}
