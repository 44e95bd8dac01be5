// picp_kernels.hip -- hand-written gfx950 (MI355X / CDNA4) kernels of the PICP hot path.
//
//   picp_round_kernel   one Gauss-Newton round of a batch of PICP problems:
//                       body      = linearize: one lane per correspondence, float4 SoA loads,
//                                   projection + 2x6 Jacobian + chi2 gate in registers,
//                                   halving-butterfly wave64 reduction of the 31 normal-equation
//                                   terms, LDS cross-wave sum, one 128 B partial per block
//                                   published write-through + an arrival ticket;
//                       last arriver = finish the round (deterministic double reduce of the
//                                   block partials, damped 6x6 LDL^T solve, v2tEuler
//                                   left-update, icp_test convergence test).
//   picp_gather_kernel  IntPairVector gather (image idx, world idx) -> SoA planes.
//   picp_triangulate_kernel  batched two-view DLT (cv::triangulatePoints replacement).
//
// Reference semantics: src/picp_solver.cpp:26-105, src/camera.h:24-36, src/defs.h:100-145,
// exec/icp_test.cpp:88-107, src/cam.cpp:94-140 (paths relative to the reference root).
// Memory-bound (20 algorithmic B and ~160 FP32 flop per correspondence-round): no MFMA.
#include <hip/hip_runtime.h>

#include <float.h>
#include <stdint.h>
#include <stdlib.h>

#include "picp_internal.h"

// Diagnostic build only (-DPICP_STAMPS, lib/libpicp_amd_stamps.so): thread 0 of each block
// records s_memrealtime (100 MHz) at phase boundaries of launches j = 10 and 11 into a buffer
// nothing else reads.  The shipped library compiles these to nothing.
#ifdef PICP_STAMPS
#define PICP_STAMP_BLOCKS 4096
__device__ unsigned long long picp_stamps[2][PICP_STAMP_BLOCKS][8];
#define STAMP(k)                                                                         \
  do {                                                                                   \
    if (threadIdx.x == 0 && (j == 10 || j == 11) && blockIdx.x < PICP_STAMP_BLOCKS) \
      picp_stamps[j - 10][blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();              \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#endif

#include "picp_device.h"


using namespace picp;

// Last-arriver reduction of one problem's published partials (the guide's in-launch split-K
// combine, cdna_hip_programming.md §6 Guideline 16): every partial word was stored write-through
// (sc1) and drained before its block took the ticket, so EVERY load here is an sc1 load
// (relaxed agent-scope atomic), which no CU's L1 can serve stale, on any XCD.  Thread t sums
// column (t & 15) -- two floats of the 32 -- over rows (t >> 4) + 16k in double, then a
// fixed-order LDS combine: deterministic for a given block partition.  Result in s_tot[0..31].
#define PICP_RED_UNROLL 32  // 16 x 32 = 512 partials per sweep: one load latency for <= 512 blocks
__device__ __forceinline__ void reduce_published(const unsigned long long* __restrict__ part, int blk0,
                                                 int nblk, double (*s_red)[PICP_NPART + 1],
                                                 double* s_tot) {
  const int tid = threadIdx.x;
  const int c = tid & 15, r = tid >> 4;  // 16 row groups x 16 u64 columns
  double lo = 0.0, hi = 0.0;
  const unsigned long long* col = part + (size_t)blk0 * (PICP_NPART / 2) + c;
  for (int base = 0; base < nblk; base += 16 * PICP_RED_UNROLL) {
    unsigned long long w[PICP_RED_UNROLL];
#pragma unroll
    for (int u = 0; u < PICP_RED_UNROLL; ++u) {
      const int bb = min(base + u * 16 + r, nblk - 1);
      w[u] = __hip_atomic_load(col + (size_t)bb * (PICP_NPART / 2), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int u = 0; u < PICP_RED_UNROLL; ++u) {
      const bool ok = base + u * 16 + r < nblk;
      lo += ok ? (double)__uint_as_float((unsigned)(w[u] & 0xffffffffull)) : 0.0;
      hi += ok ? (double)__uint_as_float((unsigned)(w[u] >> 32)) : 0.0;
    }
  }
  s_red[r][2 * c] = lo;
  s_red[r][2 * c + 1] = hi;
  __syncthreads();
  if (tid < PICP_NPART) {
    double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0;
#pragma unroll
    for (int k = 0; k < 16; k += 4) {
      t0 += s_red[k + 0][tid];
      t1 += s_red[k + 1][tid];
      t2 += s_red[k + 2][tid];
      t3 += s_red[k + 3][tid];
    }
    s_tot[tid] = (t0 + t1) + (t2 + t3);
  }
  __syncthreads();
}

// Launch j (0 <= j < R) of the fused R-round solve: every block of a live problem linearizes
// round j+1 over its slice at the pose in st_in, reduces it (wave64 permlane/DPP + LDS), and
// publishes its 32-float partial write-through; the LAST block of the problem to take the
// arrival ticket reduces all of them (deterministic order), runs finish_round (damping, LDL^T,
// Rx*Ry*Rz update, icp_test convergence) and writes st_out.  One state read per block per
// round instead of a sweep of every partial: the launch boundary is the only other hand-off.
// Finished problems propagate their state through the ping-pong.  VEC = correspondences per
// lane per chunk (4: float4 loads, for large batches; 1: one per lane, to spread a single frame
// over every SIMD).  tickets[p] are zeroed by a memset node before launch 0 and re-zeroed by
// each last arriver.
template <int VEC, int PH>
__global__ __launch_bounds__(PICP_BLOCK) void picp_round_kernel(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const float* __restrict__ U, const float* __restrict__ V, const PicpArgs A,
    const PicpProblem* __restrict__ probs, const int4* __restrict__ blkinfo,
    const PicpState* __restrict__ st_in, PicpState* __restrict__ st_out,
    unsigned long long* __restrict__ part, unsigned int* __restrict__ tickets, int j, int rev_sweep) {
  __shared__ double s_red[16][PICP_NPART + 1];
  __shared__ double s_tot[PICP_NPART];
  __shared__ float s_wave[PICP_BLOCK / 64][PICP_NPART];
  __shared__ int32_t s_state[32];
  __shared__ int s_last;

  const int tid = threadIdx.x;
  STAMP(0);
#ifdef PICP_STAMPS
  if (threadIdx.x == 0 && (j == 10 || j == 11) && blockIdx.x < PICP_STAMP_BLOCKS) {
    unsigned xcc, hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    picp_stamps[j - 10][blockIdx.x][6] = xcc;
    picp_stamps[j - 10][blockIdx.x][7] = hwid;
  }
#endif
  int p, first = 0, count = 0, blk0, nblk;
  int64_t base;
  if (A.uniform) {
    p = (int)blockIdx.x / A.nblk_u;
    const int kb = (int)blockIdx.x - p * A.nblk_u;
    first = kb * A.ipb;
    count = max(0, min(A.ipb, A.n_u - first));
    blk0 = p * A.nblk_u;
    nblk = A.nblk_u;
    base = (int64_t)p * A.stride_u + first;
  } else {
    const int4 bi = blkinfo[blockIdx.x];
    p = bi.x;
    first = bi.y;
    count = bi.z;
    const PicpProblem P = probs[p];
    blk0 = P.blk0;
    nblk = P.nblk;
    base = P.offset + first;
  }
  const bool leader = (int)blockIdx.x == blk0;

  // Items per lane per step: VEC = 4 -> a float4 of 4 consecutive items; VEC = 1 -> items c and
  // c + PICP_BLOCK (coalesced across the block).  Processed in pairs (accumulate2).
  constexpr int NI = (VEC == 4) ? 4 : 2;
  constexpr int ISTRIDE = (VEC == 4) ? 1 : PICP_BLOCK;  // distance between a lane's items
  constexpr int STEP = PICP_BLOCK * NI;
  const int c0 = tid * VEC;
  // load the step at c < count.  VEC = 4: the float4 at c stays inside the problem's padded
  // range (offsets and block ranges are multiples of 4); VEC = 1: an item past `count` reads a
  // clamped valid item.  Items past `count` are masked by accumulate2.
  auto load_step = [&](int c, float* lx, float* ly, float* lz, float* lu, float* lv) {
    if constexpr (VEC == 4) {
      const float4 x4 = *reinterpret_cast<const float4*>(X + base + c);
      const float4 y4 = *reinterpret_cast<const float4*>(Y + base + c);
      const float4 z4 = *reinterpret_cast<const float4*>(Z + base + c);
      const float4 u4 = *reinterpret_cast<const float4*>(U + base + c);
      const float4 v4 = *reinterpret_cast<const float4*>(V + base + c);
      lx[0] = x4.x; lx[1] = x4.y; lx[2] = x4.z; lx[3] = x4.w;
      ly[0] = y4.x; ly[1] = y4.y; ly[2] = y4.z; ly[3] = y4.w;
      lz[0] = z4.x; lz[1] = z4.y; lz[2] = z4.z; lz[3] = z4.w;
      lu[0] = u4.x; lu[1] = u4.y; lu[2] = u4.z; lu[3] = u4.w;
      lv[0] = v4.x; lv[1] = v4.y; lv[2] = v4.z; lv[3] = v4.w;
    } else {
#pragma unroll
      for (int k = 0; k < NI; ++k) {
        const int ck = min(c + k * ISTRIDE, max(count - 1, 0));
        lx[k] = X[base + ck];
        ly[k] = Y[base + ck];
        lz[k] = Z[base + ck];
        lu[k] = U[base + ck];
        lv[k] = V[base + ck];
      }
    }
  };
  // Streaming (VEC = 4): a ring of RING register slots, slot s holding the step at
  // c + s*STEP; each slot's next step is loaded as soon as the slot has been consumed, so every
  // wave keeps RING-1 steps of HBM reads in flight while it computes (memory-level parallelism
  // beyond the 2 resident waves per SIMD).  Single frames (VEC = 1) are latency-bound: one slot.
  constexpr int RING = (VEC == 4) ? 3 : 1;
  float bx[RING][NI], by[RING][NI], bz[RING][NI], bu[RING][NI], bv[RING][NI];
  // Odd rounds sweep the slice backwards (VEC = 4: float4 position c -> cnt4 - 4 - c, still one
  // contiguous run per wave): a round then starts on the lines the previous round touched last,
  // which the 256 MiB Infinity Cache still holds when the planes outgrow it (16M: 305 MiB).  The
  // per-lane summation order is fixed by (j, rev_sweep), so replays are deterministic.
  const int cnt4 = (count + 3) & ~3;
  const bool rev = (VEC == 4) && rev_sweep;
  auto phys = [&](int c) { return rev ? cnt4 - 4 - c : c; };
  // The state (the pose) is loaded FIRST: loads return in order, so a state load issued behind
  // the ring's 15 prefetches would wait for all of them (stamps: ~4.5 us at 16M).  The first
  // steps do not depend on the pose, so their latency overlaps the state's.
  int32_t st_word = 0;
  if (tid < 32) st_word = reinterpret_cast<const int32_t*>(st_in + p)[tid];
#pragma unroll
  for (int sl = 0; sl < RING; ++sl)
    if (c0 + sl * STEP < count) load_step(phys(c0 + sl * STEP), bx[sl], by[sl], bz[sl], bu[sl], bv[sl]);

  if (tid < 32) s_state[tid] = st_word;
  __syncthreads();
  if (j == 0 && tid == 0) {  // the icp_test loop state at entry (exec/icp_test.cpp:89)
    PicpState& s = *reinterpret_cast<PicpState*>(s_state);
    s.chi_prev = FLT_MAX;
    s.chi_in = s.chi_out = 0.0f;
    s.n_in = s.n_proj = 0;
    s.rounds = 0;
    s.done = (A.max_rounds <= 0) ? 1 : 0;
    s.ok = 1;
    s.converged = 0;
  }
  __syncthreads();
  STAMP(1);
  const PicpState& s_in = *reinterpret_cast<const PicpState*>(s_state);
  if (s_in.done) {  // finished earlier: propagate the state through the ping-pong
    if (leader && tid < 32) reinterpret_cast<int32_t*>(&st_out[p])[tid] = s_state[tid];
    return;
  }

  // ---------------- linearize (src/picp_solver.cpp:56-91) ----------------
  Pose T;
  T.r00 = s_in.R[0]; T.r10 = s_in.R[1]; T.r20 = s_in.R[2];
  T.r01 = s_in.R[3]; T.r11 = s_in.R[4]; T.r21 = s_in.R[5];
  T.r02 = s_in.R[6]; T.r12 = s_in.R[7]; T.r22 = s_in.R[8];
  T.t0 = s_in.t[0]; T.t1 = s_in.t[1]; T.t2 = s_in.t[2];
  Cam C;
  C.k00 = A.K[0]; C.k10 = A.K[1]; C.k20 = A.K[2];
  C.k01 = A.K[3]; C.k11 = A.K[4]; C.k21 = A.K[5];
  C.k02 = A.K[6]; C.k12 = A.K[7]; C.k22 = A.K[8];
  C.maxx = A.maxx;
  C.maxy = A.maxy;
  const float thr = A.threshold;
  const float inv_thr = 1.0f / thr;
  const bool keep = A.keep_outliers != 0;

  Acc2 a;
  acc2_zero(a);
  Cnt nc = {0u, 0u};  // the wave's counts; the loop is divergent at the tail: lane 0's copy is the total
  for (int c = c0; c < count; c += RING * STEP) {
#pragma unroll
    for (int sl = 0; sl < RING; ++sl) {
      const int cs = c + sl * STEP;
      if (cs < count) {
        const int ps = phys(cs);
#pragma unroll
        for (int k = 0; k < NI; k += 2)
          accumulate2<PH>(T, C, thr, inv_thr, keep, (f2){bx[sl][k], bx[sl][k + 1]},
                          (f2){by[sl][k], by[sl][k + 1]}, (f2){bz[sl][k], bz[sl][k + 1]},
                          (f2){bu[sl][k], bu[sl][k + 1]}, (f2){bv[sl][k], bv[sl][k + 1]},
                          ps + k * ISTRIDE < count, ps + (k + 1) * ISTRIDE < count, a, nc);
        const int cn = cs + RING * STEP;
        if (cn < count) load_step(phys(cn), bx[sl], by[sl], bz[sl], bu[sl], bv[sl]);
      }
    }
  }

  STAMP(2);
  float v[PICP_NPART];
  acc2_fold(a, v);
  const int lane = tid & 63, wave = tid >> 6;
  const float wsum = wave_counts(wave_reduce32(v, lane), lane, nc);
  if ((lane & 1) == 0) s_wave[wave][lane >> 1] = wsum;
  __syncthreads();
  // publish: lane t < 16 of wave 0 stores partial floats (2t, 2t+1) as one write-through
  // 8-byte word, the wave drains its stores, then lane 0 takes the problem's ticket
  if (tid < 16) {
    float e0 = s_wave[0][2 * tid], e1 = s_wave[0][2 * tid + 1];
#pragma unroll
    for (int w = 1; w < PICP_BLOCK / 64; ++w) {
      e0 += s_wave[w][2 * tid];
      e1 += s_wave[w][2 * tid + 1];
    }
    const unsigned long long word = ((unsigned long long)__float_as_uint(e1) << 32) | __float_as_uint(e0);
    __hip_atomic_store(part + (size_t)blockIdx.x * (PICP_NPART / 2) + tid, word, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  if (wave == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) {
      const unsigned int old = __hip_atomic_fetch_add(tickets + p, 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
      s_last = (old == (unsigned)(nblk - 1)) ? 1 : 0;
    }
  }
  __syncthreads();
  STAMP(3);
  if (!s_last) return;

  // ---------------- the last arriver finishes the round (src/picp_solver.cpp:93-105) -------
  reduce_published(part, blk0, nblk, s_red, s_tot);
  STAMP(4);
  if (tid == 0) {
    double tot[PICP_NPART];
#pragma unroll
    for (int i = 0; i < PICP_NPART; ++i) tot[i] = s_tot[i];
    PicpState ns;
    finish_round(A, s_in, tot, j + 1, ns);
    st_out[p] = ns;
    __hip_atomic_store(tickets + p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  STAMP(5);
}

#ifdef PICP_STAMPS
extern "C" hipError_t picp_debug_stamps(unsigned long long* out, size_t n_words) {
  const size_t cap = sizeof(picp_stamps) / sizeof(unsigned long long);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(picp_stamps), (n_words < cap ? n_words : cap) * 8, 0,
                             hipMemcpyDeviceToHost);
}
#endif

// IntPairVector gather: pairs[k] = (image idx, world idx) (src/picp_solver.cpp:65-66).
extern "C" __global__ void picp_gather_kernel(const float* __restrict__ world,
                                              const float* __restrict__ image,
                                              const int2* __restrict__ pairs, int64_t m,
                                              float* __restrict__ X, float* __restrict__ Y,
                                              float* __restrict__ Z, float* __restrict__ U,
                                              float* __restrict__ V, int64_t off) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const int2 pr = pairs[i];
  X[off + i] = world[3 * (int64_t)pr.y + 0];
  Y[off + i] = world[3 * (int64_t)pr.y + 1];
  Z[off + i] = world[3 * (int64_t)pr.y + 2];
  U[off + i] = image[2 * (int64_t)pr.x + 0];
  V[off + i] = image[2 * (int64_t)pr.x + 1];
}

// Batched two-view DLT (cv::triangulatePoints as called from src/cam.cpp:115, then
// convertPointsFromHomogeneous :118).  One lane per point; A (4x4) in double, right singular
// vector of the smallest singular value by one-sided (Hestenes) Jacobi with a fixed sweep
// count, all indices compile-time so A and V live in registers.
extern "C" __global__ void picp_triangulate_kernel(const float* __restrict__ P1,
                                                   const float* __restrict__ P2,
                                                   const float2* __restrict__ uv1,
                                                   const float2* __restrict__ uv2, int64_t q,
                                                   float* __restrict__ xyz) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= q) return;
  float o[3];
  triangulate_dlt(P1, P2, uv1[i], uv2[i], o);
  xyz[3 * i + 0] = o[0];
  xyz[3 * i + 1] = o[1];
  xyz[3 * i + 2] = o[2];
}

// ------------------------------- host launch wrappers -------------------------------
// (called by picp_runtime.cpp; every shape/grid assumption is checked there first)
extern "C" hipError_t picp_launch_round(hipStream_t stream, int grid, int vec, const float* X,
                                        const float* Y, const float* Z, const float* U,
                                        const float* V, const PicpArgs* args,
                                        const PicpProblem* probs, const int4* blkinfo,
                                        const PicpState* st_in, PicpState* st_out,
                                        unsigned long long* part, unsigned int* tickets, int j) {
  if (grid <= 0 || !args || !part || !tickets) return hipErrorInvalidValue;
  // odd rounds sweep backwards (Infinity-Cache reuse); PICP_SWEEP_FORWARD=1 disables (A/B)
  const char* fwd = getenv("PICP_SWEEP_FORWARD");  // read per launch: graphs capture it
  const bool forward_only = fwd && atoi(fwd) != 0;
  const int rev = (!forward_only && (j & 1)) ? 1 : 0;
  const int var = picp_variant(args->K, args->keep_outliers);
#define PICP_LAUNCH_R(VEC, PH)                                                                        \
  hipLaunchKernelGGL((picp_round_kernel<VEC, PH>), dim3(grid), dim3(PICP_BLOCK), 0, stream, X, Y, Z, U, \
                     V, *args, probs, blkinfo, st_in, st_out, part, tickets, j, rev)
#define PICP_LAUNCH_RV(VEC)                                                        \
  if (var == PICP_V_PINHOLE) PICP_LAUNCH_R(VEC, PICP_V_PINHOLE);                   \
  else if (var == PICP_V_PINHOLE_KEEP) PICP_LAUNCH_R(VEC, PICP_V_PINHOLE_KEEP);    \
  else PICP_LAUNCH_R(VEC, PICP_V_GENERAL)
  if (vec == 4) {
    PICP_LAUNCH_RV(4);
  } else if (vec == 1) {
    PICP_LAUNCH_RV(1);
  } else {
    return hipErrorInvalidValue;
  }
#undef PICP_LAUNCH_RV
#undef PICP_LAUNCH_R
  return hipGetLastError();
}

extern "C" hipError_t picp_launch_gather(hipStream_t stream, const float* world,
                                         const float* image, const int2* pairs, int64_t m,
                                         float* X, float* Y, float* Z, float* U, float* V,
                                         int64_t off) {
  if (m <= 0) return hipSuccess;
  const int threads = 256;
  const int64_t grid = (m + threads - 1) / threads;
  hipLaunchKernelGGL(picp_gather_kernel, dim3((unsigned)grid), dim3(threads), 0, stream, world,
                     image, pairs, m, X, Y, Z, U, V, off);
  return hipGetLastError();
}

extern "C" hipError_t picp_launch_triangulate(hipStream_t stream, const float* P1,
                                              const float* P2, const float2* uv1,
                                              const float2* uv2, int64_t q, float* xyz) {
  if (q <= 0) return hipSuccess;
  const int threads = 128;
  const int64_t grid = (q + threads - 1) / threads;
  hipLaunchKernelGGL(picp_triangulate_kernel, dim3((unsigned)grid), dim3(threads), 0, stream,
                     P1, P2, uv1, uv2, q, xyz);
  return hipGetLastError();
}

// ------------------------------- self-test of rcp_rn ----------------------------------
// Counts the floats x = 2^e * (1 + k 2^-23), e in [e_lo, e_hi), k in [0, 2^23), of both signs
// for which rcp_rn(x) and the IEEE division 1.0f / x differ in any bit.
extern "C" __global__ void picp_rcp_check_kernel(int e_lo, int e_hi, unsigned long long* bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)1 << 24;  // 2^23 mantissas x 2 signs per binade
  if (i >= (int64_t)(e_hi - e_lo) * per) return;
  const int e = e_lo + (int)(i / per);
  const unsigned rem = (unsigned)(i % per);
  const unsigned bits = ((rem >> 23) << 31) | ((unsigned)(e + 127) << 23) | (rem & 0x7fffffu);
  const float x = __uint_as_float(bits);
  if (__float_as_uint(rcp_rn(x)) != __float_as_uint(1.0f / x)) atomicAdd(bad, 1ull);
}
