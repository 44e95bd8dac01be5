// picp_block.hip -- batched independent frames: ONE block per problem runs the whole
// exec/icp_test.cpp:88-107 loop.
//
// The first NPT*PICP_BBLOCK correspondences of a problem are loaded once into registers (NPT
// per lane); any remainder is re-read every round (two per lane per step, L2/MALL-resident
// after the first round).  Every round is: linearize in registers -> wave64 reduction (permlane/DPP) -> LDS
// combine of the 8 waves -> one lane finishes the round (fp32 LDL^T, Rx*Ry*Rz update,
// convergence; picp_device.h) -> barrier.  No inter-workgroup communication at all, no launch
// per round and no HBM re-read per round: a batch of frames is bound by VALU issue, not by
// hand-off latency or HBM.  Ragged batches read (offset, n) from the problem
// table.
#include "picp_device.h"

using namespace picp;

#define PICP_BBLOCK 512  // 8 waves: 2 per SIMD at <= 256 VGPRs
#define PICP_BLDS_ITEMS 7680  // items staged in LDS: 5 x 4 B x 7680 = 150 KB of the 160 KB per CU

template <int NPT, int PH>
__global__ __launch_bounds__(PICP_BBLOCK) void picp_block_kernel(
    const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
    const float* __restrict__ U, const float* __restrict__ V, const PicpArgs A,
    const PicpProblem* __restrict__ probs, const PicpState* __restrict__ st_in,
    PicpState* __restrict__ st_out, int lds_items) {
  extern __shared__ float s_lds[];  // [5][lds_items]: the problem's items past the registers
  __shared__ float s_wave[PICP_BBLOCK / 64][PICP_NPART];
  __shared__ double s_tot[PICP_NPART];
  __shared__ float s_pose[12];
  __shared__ int s_done;
  __shared__ PicpState s_st;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int p = blockIdx.x;
  int64_t base;
  int n;
  if (A.uniform) {
    base = (int64_t)p * A.stride_u;
    n = A.n_u;
  } else {
    const PicpProblem P = probs[p];
    base = P.offset;
    n = P.n;
  }

  // the problem, loaded once into registers (coalesced: item = tid + k*BLOCK)
  float xs[NPT], ys[NPT], zs[NPT], us[NPT], vs[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int ic = min(tid + k * PICP_BBLOCK, max(n - 1, 0));
    xs[k] = X[base + ic];
    ys[k] = Y[base + ic];
    zs[k] = Z[base + ic];
    us[k] = U[base + ic];
    vs[k] = V[base + ic];
  }

  // items NPT*BLOCK .. NPT*BLOCK + n_lds - 1 are staged in LDS once (read every round at LDS
  // latency); any beyond that are streamed from L2/MALL every round
  const int r0 = NPT * PICP_BBLOCK;
  const int n_lds = max(0, min(n - r0, lds_items));
  float* lx = s_lds;
  float* ly = s_lds + lds_items;
  float* lz = s_lds + 2 * lds_items;
  float* lu = s_lds + 3 * lds_items;
  float* lv = s_lds + 4 * lds_items;
  for (int i = tid; i < n_lds; i += PICP_BBLOCK) {
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

  for (int round = 1; !s_done; ++round) {
    Pose T;
    T.r00 = s_pose[0]; T.r10 = s_pose[1]; T.r20 = s_pose[2];
    T.r01 = s_pose[3]; T.r11 = s_pose[4]; T.r21 = s_pose[5];
    T.r02 = s_pose[6]; T.r12 = s_pose[7]; T.r22 = s_pose[8];
    T.t0 = s_pose[9]; T.t1 = s_pose[10]; T.t2 = s_pose[11];
    Acc2 a;
    acc2_zero(a);
#pragma unroll
    for (int k = 0; k < NPT; k += 2) {  // pairs (k, k+1); NPT == 1: slot B repeats item 0, masked
      const int k1 = (k + 1 < NPT) ? k + 1 : k;
      accumulate2<PH>(T, C, thr, inv_thr, keep, (f2){xs[k], xs[k1]}, (f2){ys[k], ys[k1]},
                      (f2){zs[k], zs[k1]}, (f2){us[k], us[k1]}, (f2){vs[k], vs[k1]},
                      tid + k * PICP_BBLOCK < n, k + 1 < NPT && tid + (k + 1) * PICP_BBLOCK < n, a);
    }
    for (int i = tid; i < n_lds; i += 2 * PICP_BBLOCK) {  // LDS-staged items, in pairs
      const int i2 = min(i + PICP_BBLOCK, n_lds - 1);
      accumulate2<PH>(T, C, thr, inv_thr, keep, (f2){lx[i], lx[i2]}, (f2){ly[i], ly[i2]}, (f2){lz[i], lz[i2]},
                      (f2){lu[i], lu[i2]}, (f2){lv[i], lv[i2]}, true, i + PICP_BBLOCK < n_lds, a);
    }
    for (int i = r0 + n_lds + tid; i < n; i += 2 * PICP_BBLOCK) {  // streamed remainder
      const int i2 = min(i + PICP_BBLOCK, n - 1);
      const float x0 = X[base + i], y0 = Y[base + i], z0 = Z[base + i], u0 = U[base + i], v0 = V[base + i];
      const float x1 = X[base + i2], y1 = Y[base + i2], z1 = Z[base + i2], u1 = U[base + i2], v1 = V[base + i2];
      accumulate2<PH>(T, C, thr, inv_thr, keep, (f2){x0, x1}, (f2){y0, y1}, (f2){z0, z1}, (f2){u0, u1},
                      (f2){v0, v1}, true, i + PICP_BBLOCK < n, a);
    }
    float v[PICP_NPART];
    acc2_fold(a, v);
    const float wsum = wave_reduce32(v, lane);
    if ((lane & 1) == 0) s_wave[wave][lane >> 1] = wsum;
    __syncthreads();
    if (tid < PICP_NPART) {  // fixed-order combine of the 8 waves, one lane per term
      double t = 0.0;
#pragma unroll
      for (int w = 0; w < PICP_BBLOCK / 64; ++w) t += (double)s_wave[w][tid];
      s_tot[tid] = t;
    }
    __syncthreads();
    if (tid == 0) {
      double tot[PICP_NPART];
#pragma unroll
      for (int i = 0; i < PICP_NPART; ++i) tot[i] = s_tot[i];
      PicpState ns;
      finish_round(A, s_st, tot, round, ns);
      s_st = ns;
#pragma unroll
      for (int i = 0; i < 9; ++i) s_pose[i] = ns.R[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) s_pose[9 + i] = ns.t[i];
      s_done = ns.done;
    }
    __syncthreads();
  }
  if (tid < 32) reinterpret_cast<int32_t*>(&st_out[p])[tid] = reinterpret_cast<const int32_t*>(&s_st)[tid];
}

extern "C" int picp_block_max_items(void) { return 8 * PICP_BBLOCK; }  // register-resident part

// max_n: the largest problem of the launch (sizes the LDS stage: max_n - npt*512 items, capped)
extern "C" hipError_t picp_launch_block(hipStream_t stream, int grid, int npt, const float* X,
                                        const float* Y, const float* Z, const float* U,
                                        const float* V, const PicpArgs* args,
                                        const PicpProblem* probs, const PicpState* st_in,
                                        PicpState* st_out, int max_n) {
  if (grid <= 0 || !args) return hipErrorInvalidValue;
  const bool ph = picp_use_pinhole(args->K);
  const int lds_items = (max_n > npt * PICP_BBLOCK) ? min(max_n - npt * PICP_BBLOCK, PICP_BLDS_ITEMS) : 0;
  const size_t lds_bytes = (size_t)5 * lds_items * sizeof(float);
#define PICP_LAUNCH_B(N)                                                                                  \
  if (ph) {                                                                                               \
    if (lds_bytes > 65536)                                                                                \
      hipFuncSetAttribute((const void*)picp_block_kernel<N, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                          (int)lds_bytes);                                                                \
    hipLaunchKernelGGL((picp_block_kernel<N, 1>), dim3(grid), dim3(PICP_BBLOCK), lds_bytes, stream, X, Y, \
                       Z, U, V, *args, probs, st_in, st_out, lds_items);                                  \
  } else {                                                                                                \
    if (lds_bytes > 65536)                                                                                \
      hipFuncSetAttribute((const void*)picp_block_kernel<N, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                          (int)lds_bytes);                                                                \
    hipLaunchKernelGGL((picp_block_kernel<N, 0>), dim3(grid), dim3(PICP_BBLOCK), lds_bytes, stream, X, Y, \
                       Z, U, V, *args, probs, st_in, st_out, lds_items);                                  \
  }
  switch (npt) {
    case 1: PICP_LAUNCH_B(1); break;
    case 2: PICP_LAUNCH_B(2); break;
    case 4: PICP_LAUNCH_B(4); break;
    case 8: PICP_LAUNCH_B(8); break;
    default: return hipErrorInvalidValue;
  }
#undef PICP_LAUNCH_B
  return hipGetLastError();
}
