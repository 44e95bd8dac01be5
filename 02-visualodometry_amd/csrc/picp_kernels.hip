// picp_kernels.hip -- hand-written gfx950 (MI355X / CDNA4) kernels of the PICP hot path.
//
//   picp_round_kernel   one Gauss-Newton round of a batch of PICP problems:
//                       prologue  = finish the previous round (deterministic double reduce of
//                                   the block partials, damped 6x6 LDL^T solve, v2tEuler
//                                   left-update, icp_test convergence test);
//                       body      = linearize: one lane per correspondence, float4 SoA loads,
//                                   projection + 2x6 Jacobian + chi2 gate in registers,
//                                   halving-butterfly wave64 reduction of the 31 normal-equation
//                                   terms, LDS cross-wave sum, one 128 B partial per block.
//   picp_gather_kernel  IntPairVector gather (image idx, world idx) -> SoA planes.
//   picp_triangulate_kernel  batched two-view DLT (cv::triangulatePoints replacement).
//
// Reference semantics: src/picp_solver.cpp:26-105, src/camera.h:24-36, src/defs.h:100-145,
// exec/icp_test.cpp:88-107, src/cam.cpp:94-140 (paths relative to the reference root).
// Memory-bound (20 algorithmic B and ~160 FP32 flop per correspondence-round): no MFMA.
#include <hip/hip_runtime.h>

#include <float.h>
#include <stdint.h>

#include "picp_internal.h"

// Diagnostic build only (-DPICP_STAMPS, lib/libpicp_amd_stamps.so): thread 0 of each block
// records s_memrealtime (100 MHz) at phase boundaries of launches j = 10 and 11 into a buffer
// nothing else reads.  The shipped library compiles these to nothing.
#ifdef PICP_STAMPS
#define PICP_STAMP_BLOCKS 4096
__device__ unsigned long long picp_stamps[2][PICP_STAMP_BLOCKS][8];
#define STAMP(k)                                                                         \
  do {                                                                                   \
    if (threadIdx.x == 0 && !finalize && (j == 10 || j == 11) && blockIdx.x < PICP_STAMP_BLOCKS) \
      picp_stamps[j - 10][blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();              \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#endif

#include "picp_device.h"


using namespace picp;

// Deterministic sum of a problem's block partials (nblk x 32 floats) in double.  Lane t reads
// float4 quad (t & 7) of blocks (t >> 3) + 32*u: all PICP_RED_UNROLL loads of a sweep are
// issued before the first add (out-of-range slots re-read the last block and are masked, so
// no load sits behind a branch), i.e. one memory latency per 32*PICP_RED_UNROLL blocks.  Then a
// fixed-order LDS combine.  Result in s_tot[0..31]; all threads call; ends with a barrier.
#define PICP_RED_UNROLL 16
__device__ __forceinline__ void reduce_partials(const float* __restrict__ part, int blk0, int nblk,
                                                double (*s_red)[PICP_NPART + 1], double* s_tot,
                                                int32_t* st_slot, int32_t st_word) {
  const int tid = threadIdx.x;
  const int q = tid & 7, r = tid >> 3;  // PICP_BLOCK/8 = 32 block slots per sweep
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  const float4* p4 = reinterpret_cast<const float4*>(part + (size_t)blk0 * PICP_NPART) + q;
  for (int base = 0; base < nblk; base += 32 * PICP_RED_UNROLL) {
    float4 v[PICP_RED_UNROLL];
#pragma unroll
    for (int u = 0; u < PICP_RED_UNROLL; ++u) {
      const int bb = min(base + u * 32 + r, nblk - 1);
      v[u] = p4[(size_t)bb * (PICP_NPART / 4)];
    }
#pragma unroll
    for (int u = 0; u < PICP_RED_UNROLL; ++u) {
      const bool ok = base + u * 32 + r < nblk;
      a0 += ok ? (double)v[u].x : 0.0;
      a1 += ok ? (double)v[u].y : 0.0;
      a2 += ok ? (double)v[u].z : 0.0;
      a3 += ok ? (double)v[u].w : 0.0;
    }
  }
  s_red[r][4 * q + 0] = a0;
  s_red[r][4 * q + 1] = a1;
  s_red[r][4 * q + 2] = a2;
  s_red[r][4 * q + 3] = a3;
  if (st_slot) *st_slot = st_word;
  __syncthreads();
  if (tid < PICP_NPART) {
    double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0;
#pragma unroll
    for (int k = 0; k < 32; k += 4) {
      t0 += s_red[k + 0][tid];
      t1 += s_red[k + 1][tid];
      t2 += s_red[k + 2][tid];
      t3 += s_red[k + 3][tid];
    }
    s_tot[tid] = (t0 + t1) + (t2 + t3);
  }
  __syncthreads();
}

// Launch j (0 <= j <= R) of the fused R-round solve.  Launch j finishes round j-1 (j>0) and,
// unless the problem is done, linearizes round j.  With finalize=1 only the finishing part
// runs, one block per problem.  State and partials ping-pong between launches, so no
// inter-workgroup synchronisation is ever needed inside a launch: the kernel boundary is the
// only hand-off.  VEC = correspondences per lane per chunk (4: float4 loads, for large
// batches; 1: one per lane, to spread a single frame over every SIMD).
template <int VEC>
__global__ __launch_bounds__(PICP_BLOCK) void picp_round_kernel(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const float* __restrict__ U, const float* __restrict__ V, const PicpArgs A,
    const PicpProblem* __restrict__ probs, const int4* __restrict__ blkinfo,
    const PicpState* __restrict__ st_in, PicpState* __restrict__ st_out,
    const float* __restrict__ part_in, float* __restrict__ part_out, int j, int finalize) {
  __shared__ double s_red[32][PICP_NPART + 1];
  __shared__ double s_tot[PICP_NPART];
  __shared__ float s_wave[PICP_BLOCK / 64][PICP_NPART];
  __shared__ float s_pose[12];
  __shared__ int32_t s_state[32];
  __shared__ int s_go;

  const int tid = threadIdx.x;
  STAMP(0);
  int p, first = 0, count = 0, blk0, nblk;
  int64_t base;
  if (A.uniform) {
    p = finalize ? (int)blockIdx.x : (int)blockIdx.x / A.nblk_u;
    const int kb = (int)blockIdx.x - p * A.nblk_u;
    first = kb * A.ipb;
    count = max(0, min(A.ipb, A.n_u - first));
    blk0 = p * A.nblk_u;
    nblk = A.nblk_u;
    base = (int64_t)p * A.stride_u + first;
  } else {
    if (finalize) {
      p = blockIdx.x;
    } else {
      const int4 bi = blkinfo[blockIdx.x];
      p = bi.x;
      first = bi.y;
      count = bi.z;
    }
    const PicpProblem P = probs[p];
    blk0 = P.blk0;
    nblk = P.nblk;
    base = P.offset + first;
  }
  const bool leader = finalize || ((int)blockIdx.x == blk0);

  // Prefetch this lane's first chunk of every plane: the loads do not depend on the pose, so
  // their latency overlaps the prologue below.
  float xs[VEC], ys[VEC], zs[VEC], us[VEC], vs[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) xs[k] = ys[k] = zs[k] = us[k] = vs[k] = 0.0f;
  const int c0 = tid * VEC;
  if (!finalize && c0 < count) {
    if constexpr (VEC == 4) {
      const float4 x4 = *reinterpret_cast<const float4*>(X + base + c0);
      const float4 y4 = *reinterpret_cast<const float4*>(Y + base + c0);
      const float4 z4 = *reinterpret_cast<const float4*>(Z + base + c0);
      const float4 u4 = *reinterpret_cast<const float4*>(U + base + c0);
      const float4 v4 = *reinterpret_cast<const float4*>(V + base + c0);
      xs[0] = x4.x; xs[1] = x4.y; xs[2] = x4.z; xs[3] = x4.w;
      ys[0] = y4.x; ys[1] = y4.y; ys[2] = y4.z; ys[3] = y4.w;
      zs[0] = z4.x; zs[1] = z4.y; zs[2] = z4.z; zs[3] = z4.w;
      us[0] = u4.x; us[1] = u4.y; us[2] = u4.z; us[3] = u4.w;
      vs[0] = v4.x; vs[1] = v4.y; vs[2] = v4.z; vs[3] = v4.w;
    } else {
      xs[0] = X[base + c0];
      ys[0] = Y[base + c0];
      zs[0] = Z[base + c0];
      us[0] = U[base + c0];
      vs[0] = V[base + c0];
    }
  }

  if (j == 0) {
    if (tid < 12) s_pose[tid] = (tid < 9) ? st_in[p].R[tid] : st_in[p].t[tid - 9];
    if (tid == 0) {
      PicpState s = st_in[p];
      s.chi_prev = FLT_MAX;  // exec/icp_test.cpp:89
      s.chi_in = s.chi_out = 0.0f;
      s.n_in = s.n_proj = 0;
      s.rounds = 0;
      s.done = (A.max_rounds <= 0) ? 1 : 0;
      s.ok = 1;
      s.converged = 0;
      if (leader) st_out[p] = s;
      s_go = !s.done;
    }
  } else {
    // The state (128 B -> LDS) and the previous round's partials are independent loads: issue
    // both before waiting on either.  The partials of a finished problem are stale but unused.
    int32_t st_word = 0;
    if (tid < 32) st_word = reinterpret_cast<const int32_t*>(st_in + p)[tid];
    STAMP(1);
    reduce_partials(part_in, blk0, nblk, s_red, s_tot, tid < 32 ? &s_state[tid] : nullptr, st_word);
    STAMP(2);
    const PicpState& s_in = *reinterpret_cast<const PicpState*>(s_state);
    if (s_in.done) {  // finished earlier: propagate the state through the ping-pong
      if (leader && tid < 32) reinterpret_cast<int32_t*>(&st_out[p])[tid] = s_state[tid];
      return;
    }
    if (tid == 0) {
      double tot[PICP_NPART];
#pragma unroll
      for (int i = 0; i < PICP_NPART; ++i) tot[i] = s_tot[i];
      PicpState ns;
      finish_round(A, s_in, tot, j, ns);
      STAMP(6);
#pragma unroll
      for (int i = 0; i < 9; ++i) s_pose[i] = ns.R[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) s_pose[9 + i] = ns.t[i];
      s_go = !ns.done;
      if (leader) st_out[p] = ns;
    }
  }
  __syncthreads();
  STAMP(3);
  if (finalize || !s_go) return;

  // ---------------- linearize (src/picp_solver.cpp:56-91) ----------------
  Pose T;
  T.r00 = s_pose[0]; T.r10 = s_pose[1]; T.r20 = s_pose[2];
  T.r01 = s_pose[3]; T.r11 = s_pose[4]; T.r21 = s_pose[5];
  T.r02 = s_pose[6]; T.r12 = s_pose[7]; T.r22 = s_pose[8];
  T.t0 = s_pose[9]; T.t1 = s_pose[10]; T.t2 = s_pose[11];
  Cam C;
  C.k00 = A.K[0]; C.k10 = A.K[1]; C.k20 = A.K[2];
  C.k01 = A.K[3]; C.k11 = A.K[4]; C.k21 = A.K[5];
  C.k02 = A.K[6]; C.k12 = A.K[7]; C.k22 = A.K[8];
  C.maxx = A.maxx;
  C.maxy = A.maxy;
  const float thr = A.threshold;
  const bool keep = A.keep_outliers != 0;

  Acc a;
#pragma unroll
  for (int i = 0; i < 21; ++i) a.h[i] = 0.0f;
#pragma unroll
  for (int i = 0; i < 6; ++i) a.b[i] = 0.0f;
  a.chi_in = a.chi_out = a.n_in = a.n_proj = 0.0f;

  for (int c = c0; c < count; c += PICP_BLOCK * VEC) {
    if (c != c0) {  // chunks after the prefetched one
      if constexpr (VEC == 4) {
        const float4 x4 = *reinterpret_cast<const float4*>(X + base + c);
        const float4 y4 = *reinterpret_cast<const float4*>(Y + base + c);
        const float4 z4 = *reinterpret_cast<const float4*>(Z + base + c);
        const float4 u4 = *reinterpret_cast<const float4*>(U + base + c);
        const float4 v4 = *reinterpret_cast<const float4*>(V + base + c);
        xs[0] = x4.x; xs[1] = x4.y; xs[2] = x4.z; xs[3] = x4.w;
        ys[0] = y4.x; ys[1] = y4.y; ys[2] = y4.z; ys[3] = y4.w;
        zs[0] = z4.x; zs[1] = z4.y; zs[2] = z4.z; zs[3] = z4.w;
        us[0] = u4.x; us[1] = u4.y; us[2] = u4.z; us[3] = u4.w;
        vs[0] = v4.x; vs[1] = v4.y; vs[2] = v4.z; vs[3] = v4.w;
      } else {
        xs[0] = X[base + c];
        ys[0] = Y[base + c];
        zs[0] = Z[base + c];
        us[0] = U[base + c];
        vs[0] = V[base + c];
      }
    }
    const int rem = count - c;
#pragma unroll
    for (int k = 0; k < VEC; ++k) accumulate_one(T, C, thr, keep, xs[k], ys[k], zs[k], us[k], vs[k], rem > k, a);
  }

  STAMP(4);
  float v[PICP_NPART];
#pragma unroll
  for (int i = 0; i < 21; ++i) v[PICP_P_H + i] = a.h[i];
#pragma unroll
  for (int i = 0; i < 6; ++i) v[PICP_P_B + i] = a.b[i];
  v[PICP_P_CHI_IN] = a.chi_in;
  v[PICP_P_CHI_OUT] = a.chi_out;
  v[PICP_P_N_IN] = a.n_in;
  v[PICP_P_N_PROJ] = a.n_proj;
  v[31] = 0.0f;
  const int lane = tid & 63, wave = tid >> 6;
  const float wsum = wave_reduce32(v, lane);
  if ((lane & 1) == 0) s_wave[wave][lane >> 1] = wsum;
  __syncthreads();
  if (tid < PICP_NPART) {
    float sum = s_wave[0][tid];
#pragma unroll
    for (int w = 1; w < PICP_BLOCK / 64; ++w) sum += s_wave[w][tid];
    part_out[(size_t)blockIdx.x * PICP_NPART + tid] = sum;
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
                                        const float* part_in, float* part_out, int j,
                                        int finalize) {
  if (grid <= 0 || !args) return hipErrorInvalidValue;
  if (vec == 4)
    hipLaunchKernelGGL(picp_round_kernel<4>, dim3(grid), dim3(PICP_BLOCK), 0, stream, X, Y, Z, U,
                       V, *args, probs, blkinfo, st_in, st_out, part_in, part_out, j, finalize);
  else if (vec == 1)
    hipLaunchKernelGGL(picp_round_kernel<1>, dim3(grid), dim3(PICP_BLOCK), 0, stream, X, Y, Z, U,
                       V, *args, probs, blkinfo, st_in, st_out, part_in, part_out, j, finalize);
  else
    return hipErrorInvalidValue;
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
