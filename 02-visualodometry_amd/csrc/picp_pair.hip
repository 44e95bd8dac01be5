// picp_pair.hip -- batched independent frames, TWO frames per block, their rounds interleaved so
// that one frame's serial tail runs while the other frame is linearized.
//
// The block kernel (picp_block.hip) runs one frame's exec/icp_test.cpp:88-107 loop per block (or
// per group of `split` blocks).  Every round ends in a serial tail -- the wave sums combined, the
// partner exchange of a split frame, the damped 6x6 solve and the pose update on one wave -- during
// which the CU's other waves wait at a barrier: at the 128-frame per-rank shape of an 8-GPU C4 run
// that tail is a third of the round.  Here a block holds part h of frame A and
// part h of frame B (the same `split` blocks hold both frames), with 8 worker waves and two
// finishing waves, one per frame:
//   * the workers linearize A (round r), publish their wave sums to LDS and go straight on to B
//     (round r), then to A (round r + 1) as soon as its pose is there, ... -- no block barrier;
//   * A's finishing wave (issue priority 3: its chain of dependent instructions goes first when it
//     is ready) takes A's sums when all 8 workers have arrived, combines them, exchanges them with
//     A's other parts, solves and publishes A's next pose to LDS -- while the workers linearize B;
//     B's finishing wave does the same for B, overlapping A's (one finishing wave for both frames
//     measured slower than split 4 alone: its two tails in series were longer than a linearize).
// Hand-offs inside the block are LDS counters with workgroup-scope release/acquire: arrivals
// (cumulative, 8 per round) and a per-frame generation (the rounds whose pose is in s_pose).
//
// Results are bit-identical to the block kernel at the same split and register items per lane:
// every item is in the same lane and slot (item = tid + k * 512, then the LDS stage, then the
// streamed remainder), every wave reduces the same way, the finishing wave adds the 8 wave sums
// in wave order (double) and the parts in part order, and runs the same finish_round_pose.
//
// Partners are blocks b, b + 8, b + 16, ... (pair g, part h at ((g / 8) * split + h) * 8 + g % 8):
// round-robin placement puts them on one XCD (speed only).  Exchange granules {tag, hi | lo} are
// double-buffered by round parity, per (block, frame); tags continue from per-(block, frame) tag
// bases, as in the block kernel.  Every wait -- partner polls and the LDS hand-offs -- has an
// s_memrealtime deadline; a timeout sets the error word and ends the frame (the host reports it
// and re-runs the batch without hand-offs).
#include "picp_device.h"

using namespace picp;

#define PP_WORK 512              // worker threads: 8 waves, 2 per SIMD
#define PP_BS (PP_WORK + 128)    // + one finishing wave per frame
#define PP_NW (PP_WORK / 64)
#define PP_XG 64                 // exchange granules per (block, frame, round parity)
#define PP_LDS_ITEMS 3840        // LDS stage per frame: 2 x 5 x 4 B x 3840 = 150 KB

typedef __attribute__((address_space(1))) unsigned long long pgu64_t;

// Diagnostic build only (-DPICP_STAMPS, tools/pair_stamps.py): s_memrealtime of rounds 11 and 12
// of blocks < 256, per frame f: [0] worker wave 0 has the pose, [1] it has published its sums,
// [2] the finishing wave has every arrival, [3] its partner exchange is done, [4] the new pose is
// published.
#ifdef PICP_STAMPS
__device__ unsigned long long picp_pair_stamps[2][256][2][8];
#define PSTAMPF(round, f, k)                                                                       \
  do {                                                                                             \
    if ((threadIdx.x & 63) == 0 && ((round) == 11 || (round) == 12) && blockIdx.x < 256)           \
      picp_pair_stamps[(round) - 11][blockIdx.x][f][k] = __builtin_amdgcn_s_memrealtime();         \
  } while (0)
extern "C" hipError_t picp_debug_pair_stamps(unsigned long long* out, size_t n_words) {
  const size_t cap = sizeof(picp_pair_stamps) / sizeof(unsigned long long);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(picp_pair_stamps), (n_words < cap ? n_words : cap) * 8, 0,
                             hipMemcpyDeviceToHost);
}
#else
#define PSTAMPF(round, f, k) ((void)0)
#endif

__device__ __forceinline__ int lds_acquire(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Spin until *p >= target (LDS, written by another wave of the block); false on the deadline.
__device__ __forceinline__ bool lds_wait_ge(const int* p, int target, unsigned long long timeout_ticks) {
  if (lds_acquire(p) >= target) return true;
  const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + timeout_ticks;
  for (;;) {
    __builtin_amdgcn_s_sleep(1);
    if (lds_acquire(p) >= target) return true;
    if (__builtin_amdgcn_s_memrealtime() > deadline) return false;
  }
}

template <int NPT, int PH>
__global__ __launch_bounds__(PP_BS) void picp_pair_kernel(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const float* __restrict__ U, const float* __restrict__ V, const PicpArgs A,
    const PicpState* __restrict__ st_in, PicpState* __restrict__ st_out, int lds_items, int split,
    int n_problems, unsigned long long* xg, unsigned int* err, unsigned int* tagbase,
    unsigned long long timeout_ticks) {
  extern __shared__ float s_lds[];  // [frame][5][lds_items]
  __shared__ __attribute__((aligned(16))) float s_wave[2][PICP_NPART][PP_NW];
  __shared__ float s_tot[2][PICP_NPART];
  __shared__ float s_pose[2][12];
  __shared__ int s_done[2];
  __shared__ int s_gen[2];  // rounds finished: s_pose[f] is the pose after s_gen[f] rounds
  __shared__ int s_arr[2];  // worker-wave arrivals (cumulative: 8 per round)
  __shared__ PicpState s_st[2];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int s = (int)blockIdx.x >> 3;
  const int h = s % split;
  const int g = (s / split) * 8 + ((int)blockIdx.x & 7);  // pair g: frames 2g, 2g + 1
  if (2 * g >= n_problems) return;  // grid padding (whole partner groups only)

  // this block's part of each frame (uniform batches: every frame has n_u items)
  int64_t base[2];
  int n[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int p = 2 * g + f;
    base[f] = (int64_t)min(p, n_problems - 1) * A.stride_u;
    n[f] = (p < n_problems) ? A.n_u : 0;
    if (split > 1) {  // parts start on a multiple of 4 (the planes' alignment)
      const int part = (((n[f] + split - 1) / split) + 3) & ~3;
      const int first = min(n[f], h * part);
      n[f] = min(n[f], first + part) - first;
      if (n[f] > 0) base[f] += first;
    }
  }
  const int r0 = NPT * PP_WORK;
  int n_lds[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) n_lds[f] = max(0, min(n[f] - r0, lds_items));

  // both frames' items: registers (workers) and the LDS stage
  float xs[2][NPT], ys[2][NPT], zs[2][NPT], us[2][NPT], vs[2][NPT];
  if (wave < PP_NW) {
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int64_t ic = base[f] + min(tid + k * PP_WORK, max(n[f] - 1, 0));
        xs[f][k] = X[ic];
        ys[f][k] = Y[ic];
        zs[f][k] = Z[ic];
        us[f][k] = U[ic];
        vs[f][k] = V[ic];
      }
  }
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    float* l = s_lds + (size_t)f * 5 * lds_items;
    for (int i = tid; i < n_lds[f]; i += PP_BS) {
      const int64_t ic = base[f] + r0 + i;
      l[i] = X[ic];
      l[lds_items + i] = Y[ic];
      l[2 * lds_items + i] = Z[ic];
      l[3 * lds_items + i] = U[ic];
      l[4 * lds_items + i] = V[ic];
    }
  }
  if (tid < 2) {  // initial state of frame tid (as launch 0 of the multi-launch path)
    const int f = tid, p = 2 * g + f;
    PicpState st = st_in[min(p, n_problems - 1)];
    st.chi_prev = FLT_MAX;  // exec/icp_test.cpp:89
    st.chi_in = st.chi_out = 0.0f;
    st.n_in = st.n_proj = 0;
    st.rounds = 0;
    st.done = (A.max_rounds <= 0 || p >= n_problems) ? 1 : 0;
    st.ok = 1;
    st.converged = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) s_pose[f][i] = st.R[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) s_pose[f][9 + i] = st.t[i];
    s_done[f] = st.done;
    s_gen[f] = 0;
    s_arr[f] = 0;
    s_st[f] = st;
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

  if (wave < PP_NW) {
    // ---------------- workers: A round r, B round r, A round r + 1, ...
    bool fin[2] = {s_done[0] != 0, s_done[1] != 0};
    int rr[2] = {1, 1};
    while (!(fin[0] && fin[1])) {
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        if (fin[f]) continue;
        if (!lds_wait_ge(&s_gen[f], rr[f] - 1, timeout_ticks)) {  // the finishing wave is gone
          __hip_atomic_store(err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          fin[0] = fin[1] = true;
          break;
        }
        if (s_done[f]) {
          fin[f] = true;
          continue;
        }
        if (wave == 0) PSTAMPF(rr[f], f, 0);
        Pose T;
        T.r00 = s_pose[f][0]; T.r10 = s_pose[f][1]; T.r20 = s_pose[f][2];
        T.r01 = s_pose[f][3]; T.r11 = s_pose[f][4]; T.r21 = s_pose[f][5];
        T.r02 = s_pose[f][6]; T.r12 = s_pose[f][7]; T.r22 = s_pose[f][8];
        T.t0 = s_pose[f][9]; T.t1 = s_pose[f][10]; T.t2 = s_pose[f][11];
        const float* l = s_lds + (size_t)f * 5 * lds_items;
        float v[PICP_NPART];
        Cnt nr = {0u, 0u}, nd = {0u, 0u};
        if constexpr (acc_pairs(NPT)) {
          Acc2 a;
          acc2_zero(a);
          accumulate_regs<PH, NPT>(T, C, thr, inv_thr, keep, xs[f], ys[f], zs[f], us[f], vs[f], tid, PP_WORK, n[f],
                                   a, nr);
          for (int i = tid; i < n_lds[f]; i += 2 * PP_WORK) {  // LDS-staged items, in pairs
            const int i2 = min(i + PP_WORK, n_lds[f] - 1);
            const float x0 = l[i], y0 = l[lds_items + i], z0 = l[2 * lds_items + i], u0 = l[3 * lds_items + i],
                        v0 = l[4 * lds_items + i];
            const float x1 = l[i2], y1 = l[lds_items + i2], z1 = l[2 * lds_items + i2], u1 = l[3 * lds_items + i2],
                        v1 = l[4 * lds_items + i2];
            accumulate2<PH>(T, C, thr, inv_thr, keep, (f2){x0, x1}, (f2){y0, y1}, (f2){z0, z1}, (f2){u0, u1},
                            (f2){v0, v1}, true, i + PP_WORK < n_lds[f], a, nd);
          }
          for (int i = r0 + n_lds[f] + tid; i < n[f]; i += 2 * PP_WORK) {  // streamed remainder
            const int i2 = min(i + PP_WORK, n[f] - 1);
            const int64_t b = base[f];
            const float x0 = X[b + i], y0 = Y[b + i], z0 = Z[b + i], u0 = U[b + i], v0 = V[b + i];
            const float x1 = X[b + i2], y1 = Y[b + i2], z1 = Z[b + i2], u1 = U[b + i2], v1 = V[b + i2];
            accumulate2<PH>(T, C, thr, inv_thr, keep, (f2){x0, x1}, (f2){y0, y1}, (f2){z0, z1}, (f2){u0, u1},
                            (f2){v0, v1}, true, i + PP_WORK < n[f], a, nd);
          }
          acc2_fold(a, v);
        } else {
          Acc a;
          acc_zero(a);
          accumulate_regs1<PH, NPT>(T, C, thr, inv_thr, keep, xs[f], ys[f], zs[f], us[f], vs[f], tid, PP_WORK, n[f],
                                    a, nr);
          accumulate_stream1<PH>(T, C, thr, inv_thr, keep, tid, PP_WORK, n_lds[f],  // LDS-staged items
                                 [&](int i, float& x, float& y, float& z, float& u, float& v) {
                                   x = l[i]; y = l[lds_items + i]; z = l[2 * lds_items + i];
                                   u = l[3 * lds_items + i]; v = l[4 * lds_items + i];
                                 }, a, nd);
          const int64_t b = base[f];
          accumulate_stream1<PH>(T, C, thr, inv_thr, keep, r0 + n_lds[f] + tid, PP_WORK, n[f],  // streamed remainder
                                 [&](int i, float& x, float& y, float& z, float& u, float& v) {
                                   x = X[b + i]; y = Y[b + i]; z = Z[b + i]; u = U[b + i]; v = V[b + i];
                                 }, a, nd);
          acc_fold(a, v);
        }
        const float wred = wave_reduce32(v, lane);
        const float wsum = wave_counts(wred, lane, (Cnt){nr.n_in + nd.n_in, nr.n_proj + nd.n_proj});
        if ((lane & 1) == 0) s_wave[f][lane >> 1][wave] = wsum;
        // arrival: the release orders this wave's s_wave stores before the count
        if (lane == 0) __hip_atomic_fetch_add(&s_arr[f], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (wave == 0) PSTAMPF(rr[f], f, 1);
        ++rr[f];
      }
    }
    return;
  }

  // ---------------- the finishing waves: wave 8 + f finishes frame f's rounds, so the two frames'
  // tails (each a dependent chain: the combine, the partner exchange, the solve) overlap each other
  // as well as the workers' linearize
  __builtin_amdgcn_s_setprio(3);
  const int f = wave - PP_NW;
  pgu64_t* const xgg = (pgu64_t*)xg;
  const unsigned tbase = (split > 1) ? tagbase[2 * blockIdx.x + f] : 0u;
  float pr[9], pt[3], chi_prev = FLT_MAX;
#pragma unroll
  for (int i = 0; i < 9; ++i) pr[i] = s_pose[f][i];
#pragma unroll
  for (int i = 0; i < 3; ++i) pt[i] = s_pose[f][9 + i];
  int last_round = 0;
  const unsigned g0 = ((blockIdx.x >> 3) / (unsigned)split) * (unsigned)split;  // part 0's group
  bool done = s_done[f] != 0;
  for (int round = 1; !done; ++round) {
    bool tmo = !lds_wait_ge(&s_arr[f], PP_NW * round, timeout_ticks);
    PSTAMPF(round, f, 2);
    if (lane < PICP_NPART && !tmo) {  // fixed-order combine of the 8 waves, one lane per term
      float ws[PP_NW];
#pragma unroll
      for (int w = 0; w < PP_NW; ++w) ws[w] = s_wave[f][lane][w];
      double t = (double)ws[0];
#pragma unroll
      for (int w = 1; w < PP_NW; ++w) t += (double)ws[w];
      if (split > 1) {
        // publish {round, hi}, {round, lo}; poll the partners'; add the parts in part order
        const float hi = (float)t, lo = (float)(t - (double)hi);
        const size_t slot = (size_t)(round & 1) * gridDim.x;
        pgu64_t* mine = xgg + ((slot + blockIdx.x) * 2 + f) * PP_XG;
        const unsigned tag = tbase + (unsigned)round;
        __hip_atomic_store(mine + lane, ((unsigned long long)tag << 32) | __float_as_uint(hi), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(mine + PICP_NPART + lane, ((unsigned long long)tag << 32) | __float_as_uint(lo),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + timeout_ticks;
        double part_t[4];
        unsigned pending = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          part_t[q] = 0.0;
          if (q < split && q != h) pending |= 1u << q;
        }
        part_t[h & 3] = (double)hi + (double)lo;
        for (;;) {
          // every partner's granules loaded before any tag is checked: one round trip per poll
          // (picp_block.hip PICP_XG_BATCH)
          unsigned long long gh[4], gl[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            gh[q] = gl[q] = 0ull;
            if (q < split && q != h) {
              const pgu64_t* theirs = xgg + ((slot + (((g0 + q) << 3) | (blockIdx.x & 7u))) * 2 + f) * PP_XG;
              gh[q] = __hip_atomic_load(theirs + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              gl[q] = __hip_atomic_load(theirs + PICP_NPART + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
            tmo = true;
            break;
          }
        }
        t = part_t[0];
#pragma unroll
        for (int q = 1; q < 4; ++q)
          if (q < split) t += part_t[q];
      }
      s_tot[f][lane] = total_word(A, lane, t);  // lane e converts total e
    }
    PSTAMPF(round, f, 3);
    tmo = __any(tmo);  // wave-uniform
    if (tmo) __hip_atomic_store(err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_wave_barrier();
    RoundOut o;
    finish_round_pose<PICP_FINISH_WAVE>(A, s_tot[f], round, pr, pt, chi_prev, o);
    if (tmo) o.done = 1;  // stop (the host reports the error and re-runs the batch)
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 9; ++i) s_pose[f][i] = pr[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) s_pose[f][9 + i] = pt[i];
      s_done[f] = o.done;
      if (o.done) store_state(&s_st[f], pr, pt, chi_prev, o, round);
      __hip_atomic_store(&s_gen[f], round, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    PSTAMPF(round, f, 4);
    last_round = round;
    done = o.done != 0;  // every lane computed the same o
  }
  // every partner read its base before publishing round 1, and has finished its last round
  if (split > 1 && lane == 0) tagbase[2 * blockIdx.x + f] = tbase + (unsigned)last_round;
  if (h == 0 && lane < 32 && 2 * g + f < n_problems)
    reinterpret_cast<int32_t*>(&st_out[2 * g + f])[lane] = reinterpret_cast<const int32_t*>(&s_st[f])[lane];
}

// ---------------------------------------------------------------------------------------------
// host side

static size_t pair_lds_bytes(int npt, int split, int max_n, int* lds_items_out) {
  const int per_block = (split > 1) ? ((((max_n + split - 1) / split) + 3) & ~3) : max_n;
  const int lds_items = (per_block > npt * PP_WORK) ? min(per_block - npt * PP_WORK, PP_LDS_ITEMS) : 0;
  if (lds_items_out) *lds_items_out = lds_items;
  return (size_t)2 * 5 * lds_items * sizeof(float);
}

template <int N>
static const void* pair_kernel_n(int var) {
  switch (var) {
    case PICP_V_PINHOLE: return (const void*)picp_pair_kernel<N, PICP_V_PINHOLE>;
    case PICP_V_PINHOLE_KEEP: return (const void*)picp_pair_kernel<N, PICP_V_PINHOLE_KEEP>;
    default: return (const void*)picp_pair_kernel<N, PICP_V_GENERAL>;
  }
}

static const void* pair_kernel_ptr(int npt, int var) {
  switch (npt) {
    case 1: return pair_kernel_n<1>(var);
    case 2: return pair_kernel_n<2>(var);
    case 4: return pair_kernel_n<4>(var);
    default: return nullptr;
  }
}

extern "C" int picp_pair_threads(void) { return PP_BS; }
extern "C" int picp_pair_npt_cap(void) { return 4; }

// grid of a pair launch: ceil(np / 2) pairs x split parts, padded to whole groups of 8 x split
extern "C" int picp_pair_grid(int n_problems, int split) {
  const int pairs = (n_problems + 1) / 2;
  return ((split * pairs + 8 * split - 1) / (8 * split)) * (8 * split);
}

// Pair blocks one CU holds at once (the smaller of the two pinhole variants).
extern "C" hipError_t picp_pair_occupancy(int npt, int split, int max_n, const float K[9], int* blocks_per_cu) {
  if (!blocks_per_cu || (split != 1 && split != 2 && split != 4)) return hipErrorInvalidValue;
  const size_t lds_bytes = pair_lds_bytes(npt, split, max_n, nullptr);
  int best = -1;
  for (int keep = 0; keep < 2; ++keep) {
    const void* fn = pair_kernel_ptr(npt, picp_variant(K, keep));
    if (!fn) return hipErrorInvalidValue;
    if (lds_bytes > 65536) {
      hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
      if (e != hipSuccess) return e;
    }
    int occ = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, PP_BS, lds_bytes);
    if (e != hipSuccess) return e;
    best = (best < 0 || occ < best) ? occ : best;
  }
  *blocks_per_cu = best;
  return hipSuccess;
}

// Uniform batches only (A.uniform).  xg = 2 x grid x 2 x 64 u64 granules, tagbase = 2 x grid u32
// (both zeroed once per layout), err the error word; every block of a split launch must be
// resident at once (the caller checks the grid against picp_pair_occupancy).
extern "C" hipError_t picp_launch_pair(hipStream_t stream, int n_problems, int npt, const float* X, const float* Y,
                                       const float* Z, const float* U, const float* V, const PicpArgs* args,
                                       const PicpState* st_in, PicpState* st_out, int max_n, int split,
                                       unsigned long long* xg, unsigned int* err, unsigned int* tagbase,
                                       unsigned long long timeout_ticks) {
  if (n_problems <= 0 || !args || !args->uniform || (split != 1 && split != 2 && split != 4) || !err)
    return hipErrorInvalidValue;
  if (split > 1 && (!xg || !tagbase)) return hipErrorInvalidValue;
  const void* fn = pair_kernel_ptr(npt, picp_variant(args->K, args->keep_outliers));
  if (!fn) return hipErrorInvalidValue;
  int lds_items = 0;
  const size_t lds_bytes = pair_lds_bytes(npt, split, max_n, &lds_items);
  if (lds_bytes > 65536) hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
  const int grid = picp_pair_grid(n_problems, split);
  void* kargs[] = {(void*)&X, (void*)&Y, (void*)&Z, (void*)&U, (void*)&V, (void*)args, (void*)&st_in, (void*)&st_out,
                   (void*)&lds_items, (void*)&split, (void*)&n_problems, (void*)&xg, (void*)&err, (void*)&tagbase,
                   (void*)&timeout_ticks};
  hipError_t e = hipLaunchKernel(fn, dim3(grid), dim3(PP_BS), kargs, lds_bytes, stream);
  return (e != hipSuccess) ? e : hipGetLastError();
}
