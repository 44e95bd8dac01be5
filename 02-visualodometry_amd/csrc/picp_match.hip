// picp_match.hip -- descriptor matching (reference: match_points, src/my_utilities.h:70-120),
// the producer of the PICP correspondences.
//
// For every descriptor of set 1: the nearest descriptor of set 2 by squared L2 distance and the
// second-nearest distance, updated with strict '<' in set-2 index order exactly as the
// reference loop does; accepted iff best < dist_thr (0.2) and best/second < ratio_thr (0.8)
// (src/my_utilities.h:44-46,100-103).  The distance is summed over the dims in order with FP
// contraction off, so indices, distances and accept flags are bit-identical to the CPU oracle.
//
// Two queries per lane, their descriptors in registers as float2 pairs, so the subtract, square
// and in-order accumulation of both run as packed fp32 (v_pk_add_f32 / v_pk_mul_f32: two exact
// IEEE ops per lane per instruction -- FMA contraction is off, so the bits equal the oracle's);
// set 2 is streamed through LDS in tiles shared by the 512 queries of a block, one broadcast LDS
// read feeding both queries.  Batched: blockIdx.y = problem (ragged sets).
#include <hip/hip_runtime.h>

#include <float.h>
#include <stdint.h>

#include "picp_internal.h"

#define PICP_MATCH_BLOCK 256
#define PICP_MATCH_QPL 2  // queries per lane: (query A, query B) packed in one float2
#define PICP_MATCH_QPB (PICP_MATCH_BLOCK * PICP_MATCH_QPL)
#define PICP_MATCH_TILE 256
#define PICP_MATCH_MAXD 32

typedef float f2 __attribute__((ext_vector_type(2)));

// The reference's update (src/my_utilities.h:91-97), in index order,
//   if (d < best) { second = best; best = d; bi = j; } else if (d < second) second = d;
// branch-free for finite d >= 0 (best <= second always holds):
//   second' = med3(best, d, second)   (d < best: best; best <= d < second: d; else second;
//                                       d == best: best == d, as the reference's else-branch)
//   best'   = d < best ? d : best
//   bi'     = d < best ? j : bi       (strict: the first index of the minimum wins)
__device__ inline void match_update(float d, int32_t j, float& best, float& second, int32_t& bi) {
  const bool lt = d < best;
  second = __builtin_amdgcn_fmed3f(best, d, second);
  best = lt ? d : best;
  bi = lt ? j : bi;
}

template <int D>  // D > 0: compile-time dim; D == 0: runtime dim <= PICP_MATCH_MAXD
__global__ __launch_bounds__(PICP_MATCH_BLOCK) void picp_match_kernel(
    const float* __restrict__ q_desc, const float* __restrict__ r_desc,
    const MatchProblem* __restrict__ probs, int dim_rt, float dist_thr, float ratio_thr,
    int32_t* __restrict__ best_idx, float* __restrict__ best_dist,
    float* __restrict__ second_dist, int32_t* __restrict__ accepted) {
  constexpr int DM = D > 0 ? D : PICP_MATCH_MAXD;
  const int dim = D > 0 ? D : dim_rt;
  constexpr int TILE = DM <= 16 ? PICP_MATCH_TILE : PICP_MATCH_TILE / 2;
  __shared__ f2 tile[TILE * DM];  // each value duplicated: one LDS read = both lanes of a pk op
  const MatchProblem P = probs[blockIdx.y];
  const int64_t q0 = (int64_t)blockIdx.x * PICP_MATCH_QPB;
  if (q0 >= P.nq) return;  // whole block past this problem
  const int64_t qa = q0 + threadIdx.x, qb = qa + PICP_MATCH_BLOCK;
  const bool va = qa < P.nq, vb = qb < P.nq;
  f2 q[DM];
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    q[k].x = (va && k < dim) ? q_desc[(P.q_off + qa) * dim + k] : 0.0f;
    q[k].y = (vb && k < dim) ? q_desc[(P.q_off + qb) * dim + k] : 0.0f;
  }
  float best_a = FLT_MAX, second_a = FLT_MAX, best_b = FLT_MAX, second_b = FLT_MAX;  // :78-79
  int32_t bi_a = -1, bi_b = -1;
  for (int64_t t0 = 0; t0 < P.nr; t0 += TILE) {
    const int nt = (int)((P.nr - t0) < TILE ? (P.nr - t0) : TILE);
    __syncthreads();
    for (int e = threadIdx.x; e < nt * dim; e += PICP_MATCH_BLOCK) {
      const float r = r_desc[(P.r_off + t0) * dim + e];
      tile[e] = (f2){r, r};
    }
    __syncthreads();
    if (va) {
      for (int j = 0; j < nt; ++j) {
        f2 d = {0.0f, 0.0f};
        {
#pragma clang fp contract(off)
#pragma unroll
          for (int k = 0; k < DM; ++k) {
            if (k < dim) {  // (a - r)^2 summed over the dims in order, per query
              const f2 t = q[k] - tile[j * dim + k];
              d = d + t * t;
            }
          }
        }
        const int32_t jj = (int32_t)(t0 + j);
        match_update(d.x, jj, best_a, second_a, bi_a);
        match_update(d.y, jj, best_b, second_b, bi_b);
      }
    }
  }
  // accepted iff best < DISTANCE_THRESHOLD and best/second < RATIO_THRESHOLD (:100-103)
  if (va) {
    const int64_t o = P.q_off + qa;
    best_idx[o] = bi_a;
    best_dist[o] = best_a;
    second_dist[o] = second_a;
    accepted[o] = (bi_a != -1 && best_a < dist_thr && best_a / second_a < ratio_thr) ? 1 : 0;
  }
  if (vb) {
    const int64_t o = P.q_off + qb;
    best_idx[o] = bi_b;
    best_dist[o] = best_b;
    second_dist[o] = second_b;
    accepted[o] = (bi_b != -1 && best_b < dist_thr && best_b / second_b < ratio_thr) ? 1 : 0;
  }
}

extern "C" hipError_t picp_launch_match(hipStream_t stream, int n_problems, int64_t max_nq,
                                        const float* q_desc, const float* r_desc,
                                        const MatchProblem* probs, int dim, float dist_thr,
                                        float ratio_thr, int32_t* best_idx, float* best_dist,
                                        float* second_dist, int32_t* accepted) {
  if (n_problems <= 0 || max_nq <= 0) return hipSuccess;
  if (dim < 1 || dim > PICP_MATCH_MAXD || n_problems > 65535) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((max_nq + PICP_MATCH_QPB - 1) / PICP_MATCH_QPB), (unsigned)n_problems);
  if (dim == 10)
    hipLaunchKernelGGL(picp_match_kernel<10>, grid, dim3(PICP_MATCH_BLOCK), 0, stream, q_desc, r_desc,
                       probs, dim, dist_thr, ratio_thr, best_idx, best_dist, second_dist, accepted);
  else
    hipLaunchKernelGGL(picp_match_kernel<0>, grid, dim3(PICP_MATCH_BLOCK), 0, stream, q_desc, r_desc,
                       probs, dim, dist_thr, ratio_thr, best_idx, best_dist, second_dist, accepted);
  return hipGetLastError();
}
