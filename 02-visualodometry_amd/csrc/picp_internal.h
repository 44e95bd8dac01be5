// picp_internal.h -- device-visible data layout shared by the HIP kernels and the host
// runtime of libpicp_amd.so.  Not part of the public C-ABI (include/picp_c.h).
//
// HBM layout of a PICP batch (DESIGN.md §Data layout):
//   planes X,Y,Z,U,V : float32 SoA, one plane each, problem p occupies
//                      [prob.offset, prob.offset + prob.n) of every plane; offsets are
//                      multiples of 4 floats so every block streams float4 (dwordx4) loads.
//   PicpArgs         : batch-wide camera/gate/loop parameters, by-value kernel argument.
//   PicpProblem[np]  : ragged batches only: per-problem partition.
//   int4 blkinfo[nb] : ragged batches only: block -> (problem, first item, item count).
//   PicpState[2][np] : ping-pong per-problem solver state (pose + icp_test loop state).
//   float part[2][nb][32] : ping-pong per-block partial sums of the normal equations.
#pragma once
#include <stdint.h>

#define PICP_BLOCK 256            // threads per linearize block (4 waves of 64)
#define PICP_NPART 32             // floats per block partial (31 used)
// persistent mode: pose granule sets per problem -- solver g (g < 8) publishes an L2-kept copy
// (set 2g) and an agent-scope copy (set 2g + 1), 16 granules (one 128-B line) each
#define PICP_POSE_SETS 16
// partial slot layout
#define PICP_P_H 0                // 21 upper-triangle entries of H (row-major upper)
#define PICP_P_B 21               // 6 entries of b
#define PICP_P_CHI_IN 27
#define PICP_P_CHI_OUT 28
#define PICP_P_N_IN 29
#define PICP_P_N_PROJ 30

// Ragged batches only: per-problem partition (uniform batches compute it from blockIdx).
struct PicpProblem {
  int64_t offset;      // first item in the SoA planes (multiple of 4)
  int32_t n;           // number of correspondences
  int32_t blk0;        // first linearize block (index into partials) of this problem
  int32_t nblk;        // number of linearize blocks (>= 1)
  int32_t pad;
};

// Batch-wide launch arguments, passed BY VALUE (kernel-argument SGPRs: no memory hop).
struct PicpArgs {
  float K[9];            // camera matrix, column-major (src/camera.h:45)
  float maxx, maxy;      // cols-1, rows-1 (src/camera.h:31,33)
  float threshold;       // kernel threshold (src/picp_solver.h:72)
  float damping;         // src/picp_solver.h:73
  float conv_eps;        // exec/icp_test.cpp:91 (negative: never converge)
  int32_t min_inliers;   // src/picp_solver.h:74
  int32_t keep_outliers; // oneRound's keep_outliers
  int32_t max_rounds;    // exec/icp_test.cpp:88
  int32_t uniform;       // 1: problem p = block / nblk_u, items at p*stride_u (no tables)
  int32_t n_u;           // uniform: correspondences per problem
  int32_t nblk_u;        // uniform: blocks per problem
  int32_t ipb;           // items per linearize block
  int64_t stride_u;      // uniform: plane stride between problems (multiple of 4)
};

// 128-byte per-problem solver state
struct PicpState {
  float R[9];          // world-in-camera rotation, column-major
  float t[3];          // world-in-camera translation
  float chi_prev;      // icp_test's prevError (exec/icp_test.cpp:89,106)
  float chi_in;        // stats of the last linearization (chiInliers)
  float chi_out;       // chiOutliers
  int32_t n_in;        // numInliers
  int32_t n_proj;      // correspondences that passed projectPoint
  int32_t rounds;      // oneRound calls executed
  int32_t done;        // loop finished (converged, failed or max_rounds)
  int32_t ok;          // return value of the last oneRound
  int32_t converged;   // icp_test's convergenceReached
  int32_t pad[11];
};

static_assert(sizeof(PicpState) == 128, "PicpState must be 128 B");
static_assert(sizeof(PicpProblem) % 8 == 0, "PicpProblem alignment");

// ---------------------------------------------------------------------------------------
// descriptor matching (picp_match.hip): query rows [q_off, q_off + nq) of the query
// descriptors against reference rows [r_off, r_off + nr); best_idx is relative to r_off.
// Every PICP device translation unit is compiled WITHOUT packed-FP32 VALU instructions
// (v_pk_fma/mul/add_f32): hipcc_nopk.sh passes -target-feature -packed-fp32-ops to the whole
// device compile.  On MI355X (gfx950, ROCm 7.2) the compiler's packed code for apply_update gave
// lanes 48-63 of a wave results that differ from lanes 0-47 on identical inputs whenever an MFMA
// kernel ran on the same CU (tools/ubench/permlane_stress.hip victim 9 beside an MFMA kernel; none
// alone or beside LDS / FP32 / FP64 / transcendental / DPP / permlane load; the scalar build of the
// same function, victim 23, none).  In the VO sequence that made the PICP poses depend on whether
// the matcher ran beside the block kernel.  The flag is TU-wide on purpose: a
// per-kernel target("no-packed-fp32-ops") attribute stops HIP's header functions (__syncthreads,
// ...) from inlining into the kernel, and the calls cost C2 18 % and C5 80 % (round-3 pass).
// `make PK=1` restores packed code (-DPICP_ALLOW_PK) for A/B builds.

// The finishing wave's 6x6 solve: 0 = one lane (ldl6_solve), 1 = over each 16-lane row by DPP
// row_newbcast (picp_device.h ldl6_solve_wave).  The two give the same bits on every workload
// (tools/pose_dump.py); the row form is faster alone (624-680 vs 708-732 cycles) but not in the
// kernels: C2 210.5-217.0k vs 218.7-220.3k it/s, C5 625.5-627.0k vs 630.3-633.2k frames/s
// (profiles/r03/finish/).  A/B builds: -DPICP_FINISH_WAVE=1.
#ifndef PICP_FINISH_WAVE
#define PICP_FINISH_WAVE 0
#endif


struct MatchProblem {
  int64_t q_off, nq, r_off, nr;
  // the index of reference r_off in the caller's numbering (0: indices relative to r_off): a
  // problem over a later part of a reference set reports indices in the whole set's numbering
  int64_t idx0;
};

// ---------------------------------------------------------------------------------------
// essential-matrix bootstrap (picp_essential.hip; src/cam.cpp:37-91), by value
struct EssArgs {
  int32_t n_problems;
  int32_t max_iters;   // findEssentialMat maxIters (RANSAC hypotheses scored per problem)
  double fx, fy, cx, cy;
  double prob;         // findEssentialMat prob
  double threshold;    // findEssentialMat threshold (pixels)
  double dist;         // recoverPose distanceThresh
};

// ---------------------------------------------------------------------------------------
// device-resident VO sequence (picp_vo.hip): exec/icp_test.cpp:36-136 per segment
struct VoSegment {
  int64_t f0;       // first frame of the segment (bootstrap pair = f0, f0+1)
  int64_t map_off;  // first map slot of the segment
  int64_t slot0;    // first pose / step-record slot (steps + 1 slots)
  int32_t steps;    // PICP steps (frames f0+1 .. f0+steps are estimated)
  int32_t pad;
};

struct VoStep {     // per pose slot; slot 0 of a segment = the bootstrap
  int32_t n_corr;   // map correspondences of the frame (PICP input size)
  int32_t n_in;     // inliers of the last PICP round
  int32_t rounds;   // oneRound calls
  int32_t n_new;    // points triangulated and appended after this frame
  float chi_in;
  float chi_out;
  int32_t converged;
  int32_t n_proj;
};

struct VoArgs {     // by value; every pointer is device memory
  float K[9];
  int32_t dim;
  int32_t n_seg;             // segments of this launch: seg0 .. seg0 + n_seg - 1
  int32_t seg0;
  const int64_t* frame_off;  // n_frames + 1
  const float2* uv;          // per observation
  const float* desc;         // per observation, dim floats
  const VoSegment* segs;
  const float* boot;         // per segment: camera-in-world poses of f0 and f0+1 (2 x 16)
  const int32_t* pm_bi;      // frame f -> f+1 matches, indexed by f's observation
  const int32_t* pm_acc;
  const int32_t* wm_bi;      // next frame -> map matches, indexed by the frame's observation
  const int32_t* wm_acc;
  float* map_xyz;            // 3 per slot
  float* map_desc;           // dim per slot
  int64_t* map_n;            // per segment
  float* X;                  // PICP SoA planes, segment s at s * cap_c
  float* Y;
  float* Z;
  float* U;
  float* V;
  int64_t cap_c;
  PicpProblem* probs;
  PicpState* st_in;
  const PicpState* st_out;
  MatchProblem* wprobs;      // next step's world-match problem of each segment
  // the world match split by map age (split != 0; picp_vo_runtime.cpp): the append of step t
  // writes the LATE part of step t + 1 (the points it added) and the EARLY part of step t + 2
  // (the map as it leaves it), the latter double-buffered by step parity:
  // eprobs[(step & 1) * seg_all + s]
  MatchProblem* lprobs;
  MatchProblem* eprobs;
  int32_t split;
  int32_t seg_all;           // segments of the handle (eprobs' parity stride)
  float* poses;              // 16 per slot, camera-in-world, column-major
  VoStep* steps;
  int2* pairs;               // append scratch: segment s at s * cap_c
  // matcher prep (picp_match.hip): fp16 rows of dp = 16*kch halves + two guard norms
  int32_t dp;
  const _Float16* obs_h;
  const float* obs_n1;
  const float* obs_n2;
  _Float16* map_h;
  float* map_n1;
  float* map_n2;
};
