// picp_persistent.hip -- the whole exec/icp_test.cpp:88-107 loop in ONE launch, for batches whose
// blocks all fit on the chip at once (a single 100k-1M frame, a few frames).
//
// Why: with one launch per round the critical path of a round is launch gap + a chip-wide
// re-read of every block partial + the serial solve (tools/stamps.py).  Here each
// block loads its slice of the frame into REGISTERS once (never re-read from HBM), and each
// round costs one fan-in and one fan-out inside the launch:
//   1. every block linearizes its slice at the current pose and publishes its 32-float partial
//      as 32 granules {tag = round+1, value} (8-byte relaxed agent-scope atomic stores: the R2
//      hand-off of cdna_hip_programming.md Guideline 16 -- the data IS the flag, no fences);
//   2. the problem's solver blocks (its first PICP_PSOLVERS blocks, one per XCD under round-robin
//      placement) each sweep those granules until every tag matches, sum them in a FIXED order
//      (deterministic: every solver gets the same bits), solve the damped 6x6 system and apply
//      the update (picp_device.h: finish_round), then publish the new pose as 16 granules
//      {round+1, word} twice: kept in their XCD's L2 and agent-scope;
//   3. every other block polls its solver's 16 pose granules (one wave) -- the L2 copy once the
//      first round has shown that it runs on the solver's XCD -- then starts the next round.
// Correctness does not depend on placement or timing: only tags are trusted.  Blocks must be
// co-resident (the host caps the grid at the CU count with ~110 VGPRs / 10 KB LDS per block),
// every spin is bounded by a per-round s_memrealtime deadline (timeout -> error word, loop exits), and
// tags are offset by a per-problem round counter kept on the device (tagbase), so granules left
// by earlier launches never match and no memset runs between launches.
#include "picp_device.h"

using namespace picp;

typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) unsigned int gu32_t;
#define RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT
#define PICP_MAX_PBLK 256   // max blocks per problem in this mode (sweep registers)
#define PICP_PBLOCK 512     // the partition's unit: npt items per lane of a 512-thread block
// -DPICP_PWIDE=1 (A/B): npt 8 (4096 items per block, C3) as 1024 threads x 4 items, four waves
// per SIMD instead of two within 128 VGPRs.  Alone, that linearize is 11 % faster than 512 x 8
// (tools/ubench/lin_ubench.hip at 97 VGPRs); inside this kernel, squeezed to 128 VGPRs next to the
// hand-off code, the leader's linearize + publish took 3.9 instead of 3.5 us and C3 did not move
// (139-141k it/s both; profiles/r03/pwide/).
#ifndef PICP_PWIDE
#define PICP_PWIDE 0
#endif
// Followers' pose wait: two polls in flight this many s_sleep units (64 clocks) apart (0: one)
#ifndef PICP_POSE_STAGGER
#define PICP_POSE_STAGGER 8
#endif
// The solvers' sweep with two passes in flight, PICP_SWEEP_STAGGER x 64 clocks apart (0: one
// pass at a time).  Each pass loads every pending granule pair (the others point past the buffer's
// range: no memory access, a zero), so both passes' loads are unconditional and the waits count
// exactly one pass.  C3 150.5k -> 156.5k it/s (8 x 64 clocks; 16: 155k); with one item per lane
// (C2) -2 %, so it starts at PICP_SWEEP_MIN_NPT items (profiles/r05/sweep_stagger/).
#ifndef PICP_SWEEP_STAGGER
#define PICP_SWEEP_STAGGER 8
#endif
#ifndef PICP_SWEEP_MIN_NPT  // the staggered sweep from this many items per lane on
#define PICP_SWEEP_MIN_NPT 2
#endif
#ifndef PICP_POSE_NPOLL  // polls in flight in the followers' pose wait (2 or 3), when staggered
#define PICP_POSE_NPOLL 2
#endif
#define PICP_POSE_GRAN 16   // pose granules per set: R(9) t(3) done(1) solver XCC id(1) pad(2)
// Solver blocks per problem (-DPICP_PSOLVERS=1 for A/B: one leader, every follower polling its
// agent-scope pose).  Blocks kb and kb + 8j share an XCD under round-robin placement, so solver
// kb & 7 publishes where its followers' polls are L2 hits instead of fabric round trips: an
// agent-scope (sc1) store drops its line from the writer's L2 (MI355X_MICROARCH.md), a
// workgroup-scope (sc0) store keeps it there.  Placement is not guaranteed, so the solver also
// publishes agent-scope and carries its XCC id; a follower on another XCD polls that copy.
#ifndef PICP_PSOLVERS
#define PICP_PSOLVERS 8
#endif
// each solver owns two pose sets (its L2 copy and its agent-scope copy) of the problem's region
static_assert(2 * PICP_PSOLVERS <= PICP_POSE_SETS, "PICP_PSOLVERS needs 2 pose sets each (picp_internal.h)");
// (A timeout in one solver ends its followers' waits; the other solvers then wait out their own
// deadline before the error word forces the re-run.  Checking the error word every 32 passes of an
// incomplete sweep would end them sooner, but that check in the spin loops measured C2 -2.6 %,
// C3 -1.2 % on the normal path (profiles/r06/t4/ab.log), so timeouts keep the two-window cost.)
// raw buffer load aux: sc1 (bit 4: bypass L1, served by L2 / the fabric) | volatile (bit 31:
// never hoisted out of a spin loop)
#define PICP_AUX_SC1_VOLATILE ((int)(16u | 0x80000000u))
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Diagnostic build only (-DPICP_STAMPS): s_memrealtime per phase of rounds (epochs) 11 and 12.
#ifdef PICP_STAMPS
__device__ unsigned long long picp_pstamps[2][256][8];
#define PSTAMP(k)                                                                              \
  do {                                                                                         \
    if (threadIdx.x == 0 && (epoch == 11 || epoch == 12) && blockIdx.x < 256)                  \
      picp_pstamps[epoch - 11][blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();               \
  } while (0)
extern "C" hipError_t picp_debug_pstamps(unsigned long long* out, size_t n_words);
// the leader's sweep, thread 0 (wave 0): each pass's issue and return times, rounds 11 and 12
__device__ unsigned long long picp_sweepstamps[2][64];
#define SWSTAMP(k)                                                                             \
  do {                                                                                         \
    if (threadIdx.x == 0 && (epoch == 11 || epoch == 12) && (k) < 64)                          \
      picp_sweepstamps[epoch - 11][(k)] = __builtin_amdgcn_s_memrealtime();                     \
  } while (0)
extern "C" hipError_t picp_debug_sweepstamps(unsigned long long* out, size_t n_words);
#else
#define SWSTAMP(k) \
  do {             \
  } while (0)
#define PSTAMP(k) \
  do {            \
  } while (0)
#endif

__device__ __forceinline__ unsigned long long granule(unsigned epoch, float v) {
  return ((unsigned long long)epoch << 32) | (unsigned long long)__float_as_uint(v);
}

// hand-off polls run back to back: an s_sleep 1 (64 clocks) between polls measured C2 214-223k
// vs 222-225k it/s without it, bimodal vs steady (C3 unchanged; profiles/r02/e3/ab_spin.log).
// -DPICP_POLL_SLEEP restores the pause for A/B runs.
#ifdef PICP_POLL_SLEEP
#define PICP_POLL_PAUSE() __builtin_amdgcn_s_sleep(1)
#else
#define PICP_POLL_PAUSE() ((void)0)
#endif

__device__ __forceinline__ bool timed_out(unsigned long long deadline) {
  return __builtin_amdgcn_s_memrealtime() > deadline;
}

template <int NPT, int PH, int BS>
__global__ __launch_bounds__(BS) void picp_persistent_kernel(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const float* __restrict__ U, const float* __restrict__ V, const PicpArgs A,
    const PicpState* __restrict__ st_in, PicpState* __restrict__ st_out,
    unsigned long long* gpart, unsigned long long* gpose, unsigned int* err, unsigned int* tagbase,
    unsigned long long* arrive, unsigned long long timeout_ticks) {
  __shared__ double s_red[PICP_NPART][BS / 64];  // term-major: one row per combining lane
  __shared__ float s_tot[PICP_NPART];
  __shared__ float s_wave[BS / 64][PICP_NPART];
  __shared__ float s_pose[12];
  __shared__ int s_done;
  __shared__ int s_tmo;  // a wait of this block timed out (the error word is for the host)
  __shared__ int s_l2;   // a follower on its solver's XCD: poll the L2 copy of the pose

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nblk = A.nblk_u;
  const int p = (int)blockIdx.x / nblk;
  const int kb = (int)blockIdx.x - p * nblk;
  const int first = kb * A.ipb;
  const int count = max(0, min(A.ipb, A.n_u - first));
  const int64_t base = (int64_t)p * A.stride_u + first;
  const bool leader = (kb == 0);                 // keeps the loop state and the tag base
  const bool solver = (kb < PICP_PSOLVERS);      // sweeps, solves and publishes the pose
  const int sg = kb % PICP_PSOLVERS;             // this block's solver
  // partial granules are double-buffered by round parity, so correctness does not rest on the
  // leader having swept round r before any block publishes round r+1
  const size_t part_stride = (size_t)gridDim.x * PICP_NPART;
  gu64_t* my_part0 = ((gu64_t*)gpart) + (size_t)blockIdx.x * PICP_NPART;
  gu64_t* prob_part0 = ((gu64_t*)gpart) + (size_t)p * nblk * PICP_NPART;
  gu64_t* prob_pose = ((gu64_t*)gpose) + (size_t)p * PICP_POSE_SETS * PICP_POSE_GRAN;
  gu64_t* pose_l2 = prob_pose + (size_t)(2 * sg) * PICP_POSE_GRAN;      // kept in the XCD's L2
  gu64_t* pose_gl = prob_pose + (size_t)(2 * sg + 1) * PICP_POSE_GRAN;  // agent scope
  unsigned my_xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(my_xcc));
  gu32_t* errw = ((gu32_t*)err);
  // Granule tags are tbase + round.  tbase is the problem's count of rounds run by every earlier
  // launch on these buffers (its leader advances it after the last round), so tags never repeat
  // and no memset node has to clear the granules before each launch.
  gu32_t* tbase_p = ((gu32_t*)tagbase) + p;
  const unsigned tbase = __hip_atomic_load(tbase_p, RLX_AGENT);
#ifdef PICP_ARRIVAL
  // A/B: a per-problem count of block publishes, on a line of its own.  It
  // tracks tbase * nblk across launches (both zeroed together by the host), so round e is complete
  // at (tbase + e) * nblk.  The solvers wait on it before the sweep -- a hint only: the sweep
  // still checks every granule's tag, so a late or reordered count costs time, never a result.
  gu64_t* arrive_p = ((gu64_t*)arrive) + (size_t)p * 16;
#else
  (void)arrive;
#endif

  // this block's slice, loaded once into registers (coalesced: item = tid + k*BLOCK)
  float xs[NPT], ys[NPT], zs[NPT], us[NPT], vs[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = tid + k * BS;
    const int ic = min(i, max(count - 1, 0));
    xs[k] = X[base + ic];
    ys[k] = Y[base + ic];
    zs[k] = Z[base + ic];
    us[k] = U[base + ic];
    vs[k] = V[base + ic];
  }

  if (tid == 0) {  // initial state, as launch 0 of the multi-launch path
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
    s_l2 = 0;
    if (leader && s.done) st_out[p] = s;
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

  float chi_prev = FLT_MAX;  // the leader's loop state besides the pose (exec/icp_test.cpp:89)
  unsigned long long pose_sink = 0, pa = 0, pb = 0, pc = 0;  // the follower's pose polls (PICP_POSE_STAGGER)
  for (unsigned epoch = 1; !s_done; ++epoch) {
    // every wait of this round is bounded from the round's start (a whole solve may take far
    // longer than timeout_ticks at large max_rounds; one round never does)
    const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + timeout_ticks;
    // ---- 1. linearize the slice at the current pose, publish the block partial ----
    PSTAMP(0);
    Pose T;
    T.r00 = s_pose[0]; T.r10 = s_pose[1]; T.r20 = s_pose[2];
    T.r01 = s_pose[3]; T.r11 = s_pose[4]; T.r21 = s_pose[5];
    T.r02 = s_pose[6]; T.r12 = s_pose[7]; T.r22 = s_pose[8];
    T.t0 = s_pose[9]; T.t1 = s_pose[10]; T.t2 = s_pose[11];
    float v[PICP_NPART];
    Cnt nc = {0u, 0u};  // the wave's n_in / n_proj (scalar unit)
    if constexpr (NPT == 1) {  // one item per lane: the scalar path (latency-bound C2 frames)
      Acc a;
#pragma unroll
      for (int i = 0; i < 21; ++i) a.h[i] = 0.0f;
#pragma unroll
      for (int i = 0; i < 6; ++i) a.b[i] = 0.0f;
      a.chi_in = a.chi_out = 0.0f;
      accumulate<PH>(T, C, thr, inv_thr, keep, xs[0], ys[0], zs[0], us[0], vs[0], tid < count, a, nc);
#pragma unroll
      for (int i = 0; i < 21; ++i) v[PICP_P_H + i] = a.h[i];
#pragma unroll
      for (int i = 0; i < 6; ++i) v[PICP_P_B + i] = a.b[i];
      v[PICP_P_CHI_IN] = a.chi_in;
      v[PICP_P_CHI_OUT] = a.chi_out;
      v[PICP_P_N_IN] = 0.0f;
      v[PICP_P_N_PROJ] = 0.0f;
      v[31] = 0.0f;
    } else {  // NPT register-resident items per lane
      if constexpr (acc_pairs(NPT)) {
        Acc2 a;
        acc2_zero(a);
        accumulate_regs<PH, NPT>(T, C, thr, inv_thr, keep, xs, ys, zs, us, vs, tid, BS, count, a, nc);
        acc2_fold(a, v);
      } else {
        Acc a;
        acc_zero(a);
        accumulate_regs1<PH, NPT>(T, C, thr, inv_thr, keep, xs, ys, zs, us, vs, tid, BS, count, a, nc);
        acc_fold(a, v);
      }
    }
    const float wsum = wave_counts(wave_reduce32(v, lane), lane, nc);
    if ((lane & 1) == 0) s_wave[wave][lane >> 1] = wsum;
    __syncthreads();
    if (tid < PICP_NPART) {
      float sum = s_wave[0][tid];
#pragma unroll
      for (int w = 1; w < BS / 64; ++w) sum += s_wave[w][tid];
      __hip_atomic_store(my_part0 + (epoch & 1) * part_stride + tid, granule(tbase + epoch, sum), RLX_AGENT);
#ifdef PICP_ARRIVAL
      if (tid == 0) __hip_atomic_fetch_add(arrive_p, 1ull, RLX_AGENT);  // after wave 0's granule stores
#endif
    }
    PSTAMP(1);

    if (solver) {
#ifdef PICP_ARRIVAL
      {
        const unsigned long long target = (unsigned long long)(tbase + epoch) * (unsigned)nblk;
        while (__hip_atomic_load(arrive_p, RLX_AGENT) < target && !timed_out(deadline)) {
        }
      }
#endif
      // ---- 2. sweep the problem's partials: 16-B sc1 loads of granule pairs (2c, 2c+1) of
      //         blocks g + NG*i (c = tid&15, g = tid>>4); each 8-B half carries its own tag ----
      const int c = tid & 15, g = tid >> 4;
      constexpr int NG = BS / 16;  // block groups swept in parallel
      constexpr int MAXG = PICP_MAX_PBLK / NG;
      const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(prob_part0 + (epoch & 1) * part_stride), 0, nblk * PICP_NPART * 8, 0x00020000);
      u32x4 gv[MAXG];
      // re-poll only the pairs whose tags have not both matched yet: a full 50 KB sweep costs
      // ~0.5 us at one block's share of the fabric, a re-poll of the few late blocks far less
      // (a probe-first sweep -- only each block's last pair polled until it arrives -- measured
      // 17 % slower on C2: the pass is a round trip, not bandwidth, and the probe adds one)
      unsigned pending = 0;
#pragma unroll
      for (int i = 0; i < MAXG; ++i) {
        gv[i] = (u32x4){0u, 0u, 0u, 0u};
        if (g + NG * i < nblk) pending |= 1u << i;
      }
      [[maybe_unused]] int npass = 0;  // sweep passes (diagnostic stamps)
      constexpr int SWEEP_ST = (NPT >= PICP_SWEEP_MIN_NPT) ? PICP_SWEEP_STAGGER : 0;
      if constexpr (SWEEP_ST > 0) {
        u32x4 ga[MAXG], gb[MAXG];
        auto issue = [&](u32x4* gg, unsigned want) {
#pragma unroll
          for (int i = 0; i < MAXG; ++i)
            gg[i] = __builtin_amdgcn_raw_buffer_load_b128(
                rsrc, (want & (1u << i)) ? ((g + NG * i) * PICP_NPART + 2 * c) * 8 : 0x7ffffff0, 0,
                PICP_AUX_SC1_VOLATILE);
        };
        auto take = [&](const u32x4* gg, unsigned want) {
#pragma unroll
          for (int i = 0; i < MAXG; ++i)
            if ((want & pending & (1u << i)) && gg[i][1] == tbase + epoch && gg[i][3] == tbase + epoch) {
              gv[i] = gg[i];
              pending &= ~(1u << i);
            }
        };
        unsigned wa = pending, wb;
        issue(ga, wa);
        __builtin_amdgcn_s_sleep(SWEEP_ST);
        wb = pending;
        issue(gb, wb);
        for (;;) {
          take(ga, wa);
          if (!pending) break;
          wa = pending;
          issue(ga, wa);
          take(gb, wb);
          if (!pending) break;
          wb = pending;
          issue(gb, wb);
          if (timed_out(deadline)) {
            __hip_atomic_store(errw, 1u, RLX_AGENT);
            s_tmo = 1;
            break;
          }
        }
      } else {
        for (;;) {
          const unsigned want = pending;  // issue every pending load before checking any tag
          SWSTAMP(2 * npass);
#pragma unroll
          for (int i = 0; i < MAXG; ++i)
            if (want & (1u << i))
              gv[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, ((g + NG * i) * PICP_NPART + 2 * c) * 8, 0,
                                                             PICP_AUX_SC1_VOLATILE);
#pragma unroll
          for (int i = 0; i < MAXG; ++i)
            if ((want & (1u << i)) && gv[i][1] == tbase + epoch && gv[i][3] == tbase + epoch) pending &= ~(1u << i);
          SWSTAMP(2 * npass + 1);
          ++npass;
          if (!pending) break;
          if (timed_out(deadline)) {
            __hip_atomic_store(errw, 1u, RLX_AGENT);
            s_tmo = 1;
            break;
          }
          PICP_POLL_PAUSE();
        }
      }
      double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
      for (int i = 0; i < MAXG; ++i)
        if (g + NG * i < nblk) {
          acc0 += (double)__uint_as_float(gv[i][0]);
          acc1 += (double)__uint_as_float(gv[i][2]);
        }
      // the wave's four groups (lanes c, 16+c, 32+c, 48+c) first: every lane ends with the same
      // (a0+a1)+(a2+a3) (IEEE addition commutes), so the order stays fixed
      acc0 += __shfl_xor(acc0, 16);
      acc1 += __shfl_xor(acc1, 16);
      acc0 += __shfl_xor(acc0, 32);
      acc1 += __shfl_xor(acc1, 32);
      if (lane < 16) {
        s_red[2 * c][wave] = acc0;
        s_red[2 * c + 1][wave] = acc1;
      }
      __syncthreads();
      PSTAMP(2);
      // ---- finish the round in wave 0 only: lanes < 32 combine the groups (fixed order), then
      //      the wave finishes the round (every lane computes the same values) and
      //      lanes 0-15 each publish their pose word directly; the other waves meet wave 0 at
      //      the barrier below, off the publish path ----
      if (wave == 0) {
        // the pose: kept from the round start when the linearize leaves registers to spare (one
        // item per lane), else re-read here (three 16-B LDS loads, landing during the combine):
        // kept live through a register-bound linearize it spilled; s_pose changes only after the
        // finish
        float pr[9], pt[3];
        if constexpr (NPT == 1) {
          pr[0] = T.r00; pr[1] = T.r10; pr[2] = T.r20; pr[3] = T.r01; pr[4] = T.r11; pr[5] = T.r21;
          pr[6] = T.r02; pr[7] = T.r12; pr[8] = T.r22; pt[0] = T.t0; pt[1] = T.t1; pt[2] = T.t2;
        } else {
#pragma unroll
          for (int i = 0; i < 9; ++i) pr[i] = s_pose[i];
#pragma unroll
          for (int i = 0; i < 3; ++i) pt[i] = s_pose[9 + i];
        }
        if (lane < PICP_NPART) {
          double ws[BS / 64];  // every load issued before the first add
#pragma unroll
          for (int w = 0; w < BS / 64; ++w) ws[w] = s_red[lane][w];
          double t = ws[0];
#pragma unroll
          for (int w = 1; w < BS / 64; ++w) t += ws[w];
          s_tot[lane] = total_word(A, lane, t);  // lane e converts total e
        }
        __builtin_amdgcn_wave_barrier();
        {
          // the wave finishes the round (every lane the same values, loop state in registers)
          RoundOut o;
          PSTAMP(4);
          finish_round_pose<PICP_FINISH_WAVE>(A, s_tot, (int)epoch, pr, pt, chi_prev, o);
          PSTAMP(5);
          if (s_tmo) o.done = 1;  // a sweep timed out
          // ---- publish the new pose (and the done flag): lane l < 16 owns word l ----
          float w = 0.0f;
#pragma unroll
          for (int i = 0; i < 9; ++i) w = (lane == i) ? pr[i] : w;
#pragma unroll
          for (int i = 0; i < 3; ++i) w = (lane == 9 + i) ? pt[i] : w;
          w = (lane == 12) ? __int_as_float(o.done) : w;
          w = (lane == 13) ? __uint_as_float(my_xcc) : w;
          if (lane < PICP_POSE_GRAN) {
            const unsigned long long gw = granule(tbase + epoch, w);
            if (PICP_PSOLVERS > 1)
              __hip_atomic_store(pose_l2 + lane, gw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(pose_gl + lane, gw, RLX_AGENT);
          }
          if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 9; ++i) s_pose[i] = pr[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) s_pose[9 + i] = pt[i];
            s_done = o.done;
            if (o.done && leader) {
              store_state(st_out + p, pr, pt, chi_prev, o, (int)epoch);
              // every block of the problem read tbase before publishing round 1, and this is
              // after its last round: the next launch's tags start past this one's
              __hip_atomic_store(tbase_p, tbase + epoch, RLX_AGENT);
            }
          }
        }
      }
      __syncthreads();
      PSTAMP(3);
    } else {
      // ---- 3. wait for the leader's pose of this round (one wave, 16 lanes) ----
      if (wave == 0) {
        unsigned long long gp = 0;
#if PICP_POSE_STAGGER > 0
        // Two polls in flight, PICP_POSE_STAGGER x 64 clocks apart: each poll is re-issued as soon
        // as it has been checked, so the pair keeps its offset and the pose is seen within about
        // half a round trip of landing instead of a whole one (two polls issued together, checked
        // in turn, measured no gain in round 2: they stay together).  Every lane loads (lanes >= 16
        // repeat granule 15), so the waits count exactly one poll; the poll still in flight at the
        // exit keeps its registers until the next round's wait consumes them (pose_sink), so
        // nothing waits on it.
        const int gl = lane < PICP_POSE_GRAN ? lane : PICP_POSE_GRAN - 1;
        // sc1 loads either way: past the L1, served by the L2 (the L2 copy's line stays there)
        const gu64_t* src = (PICP_PSOLVERS > 1 && s_l2) ? pose_l2 : pose_gl;
        auto poll = [&]() -> unsigned long long { return __hip_atomic_load(src + gl, RLX_AGENT); };
        auto good = [&](unsigned long long v) { return __all((unsigned)(v >> 32) == tbase + epoch); };
        pose_sink ^= pa ^ pb ^ pc;  // last round's polls: long complete
        bool tmo = false;
        pa = poll();
        __builtin_amdgcn_s_sleep(PICP_POSE_STAGGER);
        if constexpr (PICP_POSE_NPOLL >= 3) {
          pb = poll();
          __builtin_amdgcn_s_sleep(PICP_POSE_STAGGER);
          for (;;) {
            pc = poll();
            if (good(pa)) { gp = pa; break; }
            pa = poll();
            if (good(pb)) { gp = pb; break; }
            pb = poll();
            if (good(pc)) { gp = pc; break; }
            if (timed_out(deadline)) { tmo = true; break; }
          }
        } else {
          for (;;) {
            pb = poll();
            if (good(pa)) { gp = pa; break; }
            pa = poll();
            if (good(pb)) { gp = pb; break; }
            if (timed_out(deadline)) { tmo = true; break; }
          }
        }
        if (tmo) {
          if (lane == 0) __hip_atomic_store(errw, 2u, RLX_AGENT);
          gp = lane == 12 ? 1u : 0u;  // force done
          if (lane < 12) gp = __float_as_uint(s_pose[lane]);
        }
#else
        const gu64_t* src = (PICP_PSOLVERS > 1 && s_l2) ? pose_l2 : pose_gl;
        for (;;) {
          bool ok = true;
          if (lane < PICP_POSE_GRAN) {
            gp = __hip_atomic_load(src + lane, RLX_AGENT);
            ok = (unsigned)(gp >> 32) == tbase + epoch;
          }
          if (__all(ok)) break;
          if (timed_out(deadline)) {
            if (lane == 0) __hip_atomic_store(errw, 2u, RLX_AGENT);
            gp = lane == 12 ? 1u : 0u;  // force done
            if (lane < 12) gp = __float_as_uint(s_pose[lane]);
            break;
          }
          PICP_POLL_PAUSE();
        }
#endif
        if (lane < 12) s_pose[lane] = __uint_as_float((unsigned)gp);
        if (lane == 12) s_done = (int)(unsigned)gp;
        // the solver's XCC id: from the next round on, poll the L2 copy when it is this XCD's
        if (PICP_PSOLVERS > 1 && lane == 13) s_l2 = ((unsigned)gp == my_xcc) ? 1 : 0;
      }
      __syncthreads();
      PSTAMP(2);
    }
  }
  // an opaque never-true test keeps the follower's last in-flight poll alive to here
  if (timeout_ticks == ~0ull && (pose_sink ^ pa ^ pb ^ pc) == 1ull) s_pose[0] = 0.0f;
}

#ifdef PICP_STAMPS
extern "C" hipError_t picp_debug_pstamps(unsigned long long* out, size_t n_words) {
  const size_t cap = sizeof(picp_pstamps) / sizeof(unsigned long long);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(picp_pstamps), (n_words < cap ? n_words : cap) * 8, 0,
                             hipMemcpyDeviceToHost);
}
extern "C" hipError_t picp_debug_sweepstamps(unsigned long long* out, size_t n_words) {
  const size_t cap = sizeof(picp_sweepstamps) / sizeof(unsigned long long);
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(picp_sweepstamps), (n_words < cap ? n_words : cap) * 8, 0,
                                     hipMemcpyDeviceToHost);
  if (e == hipSuccess) {  // clear for the next run (a shorter sweep leaves no stale passes)
    static const unsigned long long zero[2 * 64] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(picp_sweepstamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
  }
  return e;
}
#endif

// ------------------------------- host launch wrapper -------------------------------
extern "C" int picp_persistent_block(void) { return PICP_PBLOCK; }

// npt (items per lane of a 512-thread block) -> the kernel's items per lane and block size
template <int N>
struct PShape {
  static constexpr int npt = (PICP_PWIDE && N == 8) ? 4 : N;
  static constexpr int bs = (PICP_PWIDE && N == 8) ? 1024 : PICP_PBLOCK;
};

template <int N>
static const void* persistent_kernel_n(int var) {
  constexpr int T = PShape<N>::npt, B = PShape<N>::bs;
  switch (var) {
    case PICP_V_PINHOLE: return (const void*)picp_persistent_kernel<T, PICP_V_PINHOLE, B>;
    case PICP_V_PINHOLE_KEEP: return (const void*)picp_persistent_kernel<T, PICP_V_PINHOLE_KEEP, B>;
    default: return (const void*)picp_persistent_kernel<T, PICP_V_GENERAL, B>;
  }
}

// Blocks of the persistent variant for (npt, K) one CU holds at once (registers, LDS, waves).
// Its blocks hand rounds to each other, so the host launches it only when grid <= this x CUs.
extern "C" hipError_t picp_persistent_occupancy(int npt, const float K[9], int* blocks_per_cu) {
  if (!blocks_per_cu) return hipErrorInvalidValue;
  // the smaller of the two pinhole variants: keep_outliers is a per-solve argument
  int best = -1;
  for (int keep = 0; keep < 2; ++keep) {
    const void* fn = nullptr;
    switch (npt) {
      case 1: fn = persistent_kernel_n<1>(picp_variant(K, keep)); break;
      case 2: fn = persistent_kernel_n<2>(picp_variant(K, keep)); break;
      case 4: fn = persistent_kernel_n<4>(picp_variant(K, keep)); break;
      case 8: fn = persistent_kernel_n<8>(picp_variant(K, keep)); break;
      default: return hipErrorInvalidValue;
    }
    int occ = 0;
    const hipError_t e =
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, npt == 8 ? PShape<8>::bs : PICP_PBLOCK, 0);
    if (e != hipSuccess) return e;
    best = (best < 0 || occ < best) ? occ : best;
  }
  *blocks_per_cu = best;
  return hipSuccess;
}

extern "C" hipError_t picp_launch_persistent(hipStream_t stream, int grid, int npt, const float* X,
                                             const float* Y, const float* Z, const float* U,
                                             const float* V, const PicpArgs* args,
                                             const PicpState* st_in, PicpState* st_out,
                                             unsigned long long* gpart, unsigned long long* gpose,
                                             unsigned int* err, unsigned int* tagbase,
                                             unsigned long long* arrive, unsigned long long timeout_ticks) {
  if (grid <= 0 || !args || !args->uniform || args->nblk_u > PICP_MAX_PBLK) return hipErrorInvalidValue;
  const int var = picp_variant(args->K, args->keep_outliers);
#define PICP_LAUNCH_PV(N, PV)                                                                      \
  hipLaunchKernelGGL((picp_persistent_kernel<PShape<N>::npt, PV, PShape<N>::bs>), dim3(grid),      \
                     dim3(PShape<N>::bs), 0, stream, X, Y, Z, U, V, *args, st_in, st_out, gpart, gpose, \
                     err, tagbase, arrive, timeout_ticks)
#define PICP_LAUNCH_P(N)                                                            \
  if (var == PICP_V_PINHOLE) PICP_LAUNCH_PV(N, PICP_V_PINHOLE);                     \
  else if (var == PICP_V_PINHOLE_KEEP) PICP_LAUNCH_PV(N, PICP_V_PINHOLE_KEEP);      \
  else PICP_LAUNCH_PV(N, PICP_V_GENERAL)
  switch (npt) {
    case 1: PICP_LAUNCH_P(1); break;
    case 2: PICP_LAUNCH_P(2); break;
    case 4: PICP_LAUNCH_P(4); break;
    case 8: PICP_LAUNCH_P(8); break;
    default: return hipErrorInvalidValue;
  }
#undef PICP_LAUNCH_P
#undef PICP_LAUNCH_PV
  return hipGetLastError();
}
