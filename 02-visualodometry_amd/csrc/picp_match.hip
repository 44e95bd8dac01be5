// picp_match.hip -- descriptor matching (reference: match_points, src/my_utilities.h:70-120),
// the producer of the PICP correspondences.
//
// For every descriptor of set 1: the nearest descriptor of set 2 by squared L2 distance and the
// second-nearest distance, updated with strict '<' in set-2 index order exactly as the
// reference loop does; accepted iff best < dist_thr (0.2) and best/second < ratio_thr (0.8)
// (src/my_utilities.h:44-46,100-103).  The distance is summed over the dims in order with FP
// contraction off, so indices, distances and accept flags are bit-identical to the CPU oracle.
//
// One lane per query, the query's descriptor in registers; set 2 is streamed through LDS in
// tiles shared by the 256 queries of a block.  Batched: blockIdx.y = problem (ragged sets).
#include <hip/hip_runtime.h>

#include <float.h>
#include <stdint.h>

#include "picp_internal.h"

#define PICP_MATCH_BLOCK 256
#define PICP_MATCH_TILE 256
#define PICP_MATCH_MAXD 32


template <int D>  // D > 0: compile-time dim; D == 0: runtime dim <= PICP_MATCH_MAXD
__global__ __launch_bounds__(PICP_MATCH_BLOCK) void picp_match_kernel(
    const float* __restrict__ q_desc, const float* __restrict__ r_desc,
    const MatchProblem* __restrict__ probs, int dim_rt, float dist_thr, float ratio_thr,
    int32_t* __restrict__ best_idx, float* __restrict__ best_dist,
    float* __restrict__ second_dist, int32_t* __restrict__ accepted) {
  constexpr int DM = D > 0 ? D : PICP_MATCH_MAXD;
  const int dim = D > 0 ? D : dim_rt;
  __shared__ float tile[PICP_MATCH_TILE * DM];
  const MatchProblem P = probs[blockIdx.y];
  const int64_t qi = (int64_t)blockIdx.x * PICP_MATCH_BLOCK + threadIdx.x;
  if ((int64_t)blockIdx.x * PICP_MATCH_BLOCK >= P.nq) return;  // whole block past this problem
  const bool active = qi < P.nq;
  float q[DM];
#pragma unroll
  for (int k = 0; k < DM; ++k) q[k] = (active && k < dim) ? q_desc[(P.q_off + qi) * dim + k] : 0.0f;
  float best = FLT_MAX, second = FLT_MAX;  // src/my_utilities.h:78-79
  int32_t bi = -1;
  for (int64_t t0 = 0; t0 < P.nr; t0 += PICP_MATCH_TILE) {
    const int nt = (int)((P.nr - t0) < PICP_MATCH_TILE ? (P.nr - t0) : PICP_MATCH_TILE);
    __syncthreads();
    for (int e = threadIdx.x; e < nt * dim; e += PICP_MATCH_BLOCK)
      tile[e] = r_desc[(P.r_off + t0) * dim + e];
    __syncthreads();
    if (active) {
      for (int j = 0; j < nt; ++j) {
        float d = 0.0f;
        {
#pragma clang fp contract(off)
#pragma unroll
          for (int k = 0; k < DM; ++k) {
            if (k < dim) {
              const float t = q[k] - tile[j * dim + k];
              d = d + t * t;
            }
          }
        }
        if (d < best) {  // :91-97
          second = best;
          best = d;
          bi = (int32_t)(t0 + j);
        } else if (d < second) {
          second = d;
        }
      }
    }
  }
  if (active) {
    const int64_t o = P.q_off + qi;
    best_idx[o] = bi;
    best_dist[o] = best;
    second_dist[o] = second;
    accepted[o] = (bi != -1 && best < dist_thr && best / second < ratio_thr) ? 1 : 0;  // :100-103
  }
}

extern "C" hipError_t picp_launch_match(hipStream_t stream, int n_problems, int64_t max_nq,
                                        const float* q_desc, const float* r_desc,
                                        const MatchProblem* probs, int dim, float dist_thr,
                                        float ratio_thr, int32_t* best_idx, float* best_dist,
                                        float* second_dist, int32_t* accepted) {
  if (n_problems <= 0 || max_nq <= 0) return hipSuccess;
  if (dim < 1 || dim > PICP_MATCH_MAXD || n_problems > 65535) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((max_nq + PICP_MATCH_BLOCK - 1) / PICP_MATCH_BLOCK), (unsigned)n_problems);
  if (dim == 10)
    hipLaunchKernelGGL(picp_match_kernel<10>, grid, dim3(PICP_MATCH_BLOCK), 0, stream, q_desc, r_desc,
                       probs, dim, dist_thr, ratio_thr, best_idx, best_dist, second_dist, accepted);
  else
    hipLaunchKernelGGL(picp_match_kernel<0>, grid, dim3(PICP_MATCH_BLOCK), 0, stream, q_desc, r_desc,
                       probs, dim, dist_thr, ratio_thr, best_idx, best_dist, second_dist, accepted);
  return hipGetLastError();
}
