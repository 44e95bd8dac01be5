// picp_device.h -- device-side math shared by the PICP kernels (picp_kernels.hip, multi-launch
// rounds; picp_persistent.hip, single-launch rounds): per-correspondence projection/Jacobian/gate
// (src/camera.h:24-36, src/picp_solver.cpp:26-91), the wave64 normal-equation reduction, the
// damped 6x6 LDL^T solve and the v2tEuler left update (src/picp_solver.cpp:93-105,
// src/defs.h:100-136), and the icp_test convergence rule (exec/icp_test.cpp:99-106).
#pragma once
#include <hip/hip_runtime.h>

#include <float.h>
#include <stdlib.h>
#include <stdint.h>

#include <type_traits>

#include "picp_internal.h"

namespace picp {

struct Pose {
  float r00, r01, r02, r10, r11, r12, r20, r21, r22;
  float t0, t1, t2;
};

struct Cam {
  float k00, k01, k02, k10, k11, k12, k20, k21, k22;
  float maxx, maxy;  // cols-1, rows-1 (src/camera.h:31,33)
};

// Per-item math variant, fixed at launch (picp_variant): any K with the kernel weight chosen at
// run time; the reference's pinhole K with outliers rejected (keep_outliers = false, as
// icp_test runs it: every used item has weight exactly 1, so the weighted Jacobian IS the
// Jacobian and no weight is formed); pinhole K with outliers kept (robust weight per item).
#define PICP_V_GENERAL 0
#define PICP_V_PINHOLE 1
#define PICP_V_PINHOLE_KEEP 2

struct Acc {
  float h[21];  // upper triangle of H, row-major (i<=j)
  float b[6];
  float chi_in, chi_out;
};

// n_in / n_proj of a wave, counted on the SCALAR unit: each item's inlier and projectable
// predicates are already lane masks (v_cmp results), so a count is s_bcnt1 + s_add per mask,
// issued beside the VALU work instead of as selects and adds in it.  Inside a divergent loop the
// compiler keeps the counter per lane; a lane's copy then counts the items of every iteration
// that lane ran, and lane 0 of a wave runs every iteration any lane of it runs (its items come
// first), so wave_counts reads lane 0.
struct Cnt {
  unsigned n_in, n_proj;
};

__device__ __forceinline__ void cnt_add(Cnt& c, bool inl, bool valid) {
  c.n_in += (unsigned)__builtin_popcountll(__builtin_amdgcn_ballot_w64(inl));
  c.n_proj += (unsigned)__builtin_popcountll(__builtin_amdgcn_ballot_w64(valid));
}

// After wave_reduce32 (lane l holds the wave total of value l >> 1): the wave's counts, as the
// float words of PICP_P_N_IN / PICP_P_N_PROJ (exact: a wave counts far fewer than 2^24 items).
__device__ __forceinline__ float wave_counts(float wsum, int lane, const Cnt& c) {
  const unsigned n_in = __builtin_amdgcn_readlane(c.n_in, 0);
  const unsigned n_proj = __builtin_amdgcn_readlane(c.n_proj, 0);
  wsum = ((lane >> 1) == PICP_P_N_IN) ? (float)n_in : wsum;
  return ((lane >> 1) == PICP_P_N_PROJ) ? (float)n_proj : wsum;
}

typedef float f2 __attribute__((ext_vector_type(2)));

// Two accumulation slots per lane: correspondences are processed in PAIRS, item A in .x and
// item B in .y of every value (written as float2 math: packed-FP32 instructions until the device
// code was built without them, picp_internal.h; now two scalar chains); the slots are folded
// once per thread at the end.
struct Acc2 {
  f2 h[21];
  f2 b[6];
  f2 chi_in, chi_out;
};

__device__ __forceinline__ void acc2_zero(Acc2& a) {
#pragma unroll
  for (int i = 0; i < 21; ++i) a.h[i] = (f2){0.0f, 0.0f};
#pragma unroll
  for (int i = 0; i < 6; ++i) a.b[i] = (f2){0.0f, 0.0f};
  a.chi_in = a.chi_out = (f2){0.0f, 0.0f};
}

// fold the two slots into the 32-term partial layout (picp_internal.h PICP_P_*); the counts
// are wave-level (Cnt, wave_counts)
__device__ __forceinline__ void acc2_fold(const Acc2& a, float v[PICP_NPART]) {
#pragma unroll
  for (int i = 0; i < 21; ++i) v[PICP_P_H + i] = a.h[i].x + a.h[i].y;
#pragma unroll
  for (int i = 0; i < 6; ++i) v[PICP_P_B + i] = a.b[i].x + a.b[i].y;
  v[PICP_P_CHI_IN] = a.chi_in.x + a.chi_in.y;
  v[PICP_P_CHI_OUT] = a.chi_out.x + a.chi_out.y;
  v[PICP_P_N_IN] = 0.0f;
  v[PICP_P_N_PROJ] = 0.0f;
  v[31] = 0.0f;
}

// Correctly rounded 1/x in 3 instructions: v_rcp_f32 (about 1 ulp) and one FMA Newton step.
// Verified bit-identical to the IEEE division 1.0f/x for EVERY float x in [2^-8, 2^8) by
// picp_selftest_rcp (tests/test_gpu_parity.py); both operations are exact under power-of-two
// scaling inside the normal range, so that covers every x with 2^-100 <= |x| <= 2^100
// (rcp_safe).  Outside it (and for 0, inf, NaN) callers use the IEEE division.
__device__ __forceinline__ float rcp_rn(float x) {
  const float r = __builtin_amdgcn_rcpf(x);
  const float e = fmaf(-x, r, 1.0f);
  return fmaf(e, r, r);
}

__device__ __forceinline__ bool rcp_safe(float x) {
  const float a = fabsf(x);
  return (a >= 7.8886091e-31f) & (a <= 1.2676506e30f);  // [2^-100, 2^100]; NaN -> false
}

// ---------------------------------------------------------------------------------------
// Per-correspondence math.  The block that decides projectability and the chi2 gate is
// compiled with FP contraction OFF and evaluates every sum left to right, exactly like the
// CPU oracle (oracle/picp_oracle.c), so inlier/outlier/skip decisions are bit-identical to
// the oracle at the same pose.  The Jacobian and accumulation are free to use FMA.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void accumulate_one(const Pose& T, const Cam& C, float thr,
                                               bool keep, float x, float y, float z, float u,
                                               float v, bool in_range, Acc& a, Cnt& n) {
  float pc0, pc1, pc2, ph0, ph1, ph2, iz, e0, e1, chi;
  bool valid;
  {
#pragma clang fp contract(off)
    // src/camera.h:26  pc = R*p + t
    pc0 = ((T.r00 * x + T.r01 * y) + T.r02 * z) + T.t0;
    pc1 = ((T.r10 * x + T.r11 * y) + T.r12 * z) + T.t1;
    pc2 = ((T.r20 * x + T.r21 * y) + T.r22 * z) + T.t2;
    // src/camera.h:29  ph = K*pc
    ph0 = (C.k00 * pc0 + C.k01 * pc1) + C.k02 * pc2;
    ph1 = (C.k10 * pc0 + C.k11 * pc1) + C.k12 * pc2;
    ph2 = (C.k20 * pc0 + C.k21 * pc1) + C.k22 * pc2;
    // src/camera.h:30 / picp_solver.cpp:44: (float)(1.0/(double)z) == correctly rounded
    // 1.0f/z (double rounding is innocuous for division at 53 >= 2*24+2); hipcc's default
    // fp32 division is correctly rounded.
    iz = 1.0f / ph2;
    const float ix = ph0 * iz;
    const float iy = ph1 * iz;
    // src/camera.h:27-28 (z<=0 rejects; NaN passes as in the reference) and :31-34
    // bitwise, not short-circuit: the same predicate without per-item exec-mask branches
    valid = in_range & !(pc2 <= 0.0f) & !((ix < 0.0f) | (ix > C.maxx) | (iy < 0.0f) | (iy > C.maxy));
    e0 = ix - u;  // src/picp_solver.cpp:34
    e1 = iy - v;
    chi = e0 * e0 + e1 * e1;  // src/picp_solver.cpp:74
  }
  // src/picp_solver.cpp:75-89: strict gate, sqrt kernel weight, outliers only with keep
  const bool outlier = chi > thr;
  const bool inl = valid & !outlier;
  const bool use = inl | (valid & keep);
  const float lambda = outlier ? sqrtf(thr / chi) : 1.0f;
  const float w = inl ? 1.0f : lambda;
  a.chi_in += inl ? chi : 0.0f;
  a.chi_out += (valid && outlier) ? chi : 0.0f;
  cnt_add(n, inl, valid);
  // unused terms are zeroed by select before the Jacobian, so a skipped point (possibly
  // with an infinite iz) can never inject inf/NaN into H or b
  iz = use ? iz : 0.0f;
  pc0 = use ? pc0 : 0.0f;
  pc1 = use ? pc1 : 0.0f;
  pc2 = use ? pc2 : 0.0f;
  ph0 = use ? ph0 : 0.0f;
  ph1 = use ? ph1 : 0.0f;
  e0 = use ? e0 : 0.0f;
  e1 = use ? e1 : 0.0f;
  // src/picp_solver.cpp:38-52: J = Jp * K * [I | skew(-pc)]
  const float iz2 = iz * iz;
  const float jp02 = -ph0 * iz2, jp12 = -ph1 * iz2;
  const float a00 = iz * C.k00 + jp02 * C.k20;  // (Jp*K)(0,c)
  const float a01 = iz * C.k01 + jp02 * C.k21;
  const float a02 = iz * C.k02 + jp02 * C.k22;
  const float a10 = iz * C.k10 + jp12 * C.k20;  // (Jp*K)(1,c)
  const float a11 = iz * C.k11 + jp12 * C.k21;
  const float a12 = iz * C.k12 + jp12 * C.k22;
  float J0[6], J1[6];
  J0[0] = a00; J0[1] = a01; J0[2] = a02;
  J0[3] = a02 * pc1 - a01 * pc2;
  J0[4] = a00 * pc2 - a02 * pc0;
  J0[5] = a01 * pc0 - a00 * pc1;
  J1[0] = a10; J1[1] = a11; J1[2] = a12;
  J1[3] = a12 * pc1 - a11 * pc2;
  J1[4] = a10 * pc2 - a12 * pc0;
  J1[5] = a11 * pc0 - a10 * pc1;
  float W0[6], W1[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    W0[i] = w * J0[i];
    W1[i] = w * J1[i];
  }
  int k = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
#pragma unroll
    for (int j = i; j < 6; ++j) {
      a.h[k] = fmaf(W0[i], J0[j], fmaf(W1[i], J1[j], a.h[k]));
      ++k;
    }
    a.b[i] = fmaf(W0[i], e0, fmaf(W1[i], e1, a.b[i]));
  }
}

// The reciprocal of the depth (ph2 == pc2 exactly): RCP_CHECK decides per pair by a wave vote;
// RCP_FAST: the caller's vote found every depth of the section inside rcp_safe's range (rcp_rn,
// exhaustively verified); RCP_DIV: the IEEE division.
#define RCP_CHECK 0
#define RCP_FAST 1
#define RCP_DIV 2

// Pinhole camera K = [fx 0 cx; 0 fy cy; 0 0 1] (the reference's K, src/cam.cpp:11-16; the
// runtime selects this path only when K has exactly that structure).  Every term the general
// form multiplies by one of K's zeros is an exact +-0 and K(2,2) = 1 makes ph2 == pc2, so with
// those terms dropped the projection, bounds test, error and chi -- the gate -- AND the
// Jacobian, evaluated in the oracle's operation order with contraction off
// (oracle/picp_oracle.c or_error_and_jacobian: (Jp*K)*[I | skew(-pc)]), are bit-identical to
// the reference arithmetic for finite inputs (a sign of zero can differ only where pc2 == 0,
// which is rejected):
//   a00 = fx/z, a02 = cx/z - ph0/z^2, a11 = fy/z, a12 = cy/z - ph1/z^2
//   J0 = [a00, 0, a02, a02 pc1, a00 pc2 - a02 pc0, -a00 pc1]
//   J1 = [0, a11, a12, a12 pc1 - a11 pc2, -a12 pc0, a11 pc0]
// The structural zeros drop 12 of the 54 multiply-adds of H and b, and lambda = sqrt(thr/chi)
// comes from v_rsq (it only weighs kept outliers, within the H/b tolerance): ~1/3 fewer VALU
// instructions per correspondence than the general path.  KEEP (keep_outliers, compile time):
// without it every used item has weight 1 and every other item has J = e = 0 (zeroed inputs),
// so H and b take J itself -- bit-identical to multiplying by w in {0, 1}, 10 multiplies fewer.
// The camera-frame depth of one item in accumulate_pinhole's exact operation order (so the
// compiler shares it with the item's projection).
__device__ __forceinline__ float item_depth(const Pose& T, float x, float y, float z) {
#pragma clang fp contract(off)
  return ((T.r20 * x + T.r21 * y) + T.r22 * z) + T.t2;  // src/camera.h:26, row 2
}

// RCP: RCP_DIV (the IEEE division) or RCP_FAST (rcp_rn: the caller's wave vote found the depth
// inside rcp_safe's range; the same bits).
template <bool KEEP, int RCP = RCP_DIV>
__device__ __forceinline__ void accumulate_pinhole(const Pose& T, const Cam& C, float thr,
                                                   float inv_thr, float x, float y,
                                                   float z, float u, float v, bool in_range,
                                                   Acc& a, Cnt& n) {
  float pc0, pc1, pc2, ph0, ph1, iz, e0, e1, chi;
  bool valid, proj;
  {
#pragma clang fp contract(off)
    pc0 = ((T.r00 * x + T.r01 * y) + T.r02 * z) + T.t0;  // src/camera.h:26
    pc1 = ((T.r10 * x + T.r11 * y) + T.r12 * z) + T.t1;
    pc2 = ((T.r20 * x + T.r21 * y) + T.r22 * z) + T.t2;
    ph0 = C.k00 * pc0 + C.k02 * pc2;  // src/camera.h:29 without the zero terms
    ph1 = C.k11 * pc1 + C.k12 * pc2;
    iz = (RCP == RCP_FAST) ? rcp_rn(pc2) : 1.0f / pc2;  // ph2 == pc2 exactly
    const float ix = ph0 * iz;
    const float iy = ph1 * iz;
    // bitwise, not short-circuit: the same predicate without per-item exec-mask branches
    proj = !(pc2 <= 0.0f) & !((ix < 0.0f) | (ix > C.maxx) | (iy < 0.0f) | (iy > C.maxy));
    valid = in_range & proj;
    e0 = ix - u;
    e1 = iy - v;
    chi = e0 * e0 + e1 * e1;
  }
  const bool outlier = chi > thr;
  const bool inl = valid & !outlier;
  const bool use = inl | (valid & KEEP);
  // the robust weight only when outliers are kept
  const float w = KEEP ? (use ? (inl ? 1.0f : __builtin_amdgcn_rsqf(chi * inv_thr)) : 0.0f) : 1.0f;
  a.chi_in += inl ? chi : 0.0f;
  a.chi_out += (valid && outlier) ? chi : 0.0f;
  cnt_add(n, inl, valid);
  // A skipped point gets weight 0 and zeroed inputs, so it can never inject 0 * inf.  The
  // zeroing only matters for points whose J could be non-finite: ones that do not project, or
  // project from a depth under 1e-12.  A skipped point that projects from a larger depth
  // (an outlier, a padding lane's copy) has finite pc, ph and, with a finite chi, finite e: its
  // J is exactly 0 once iz alone is zeroed, and fma(+-0, finite, h) == h exactly (the sums start
  // at +0 and never become -0), so waves without a dangerous skipped point zero only iz, with
  // bit-identical H and b.
  if (__all(use | (proj & (pc2 >= 1e-12f) & (chi <= FLT_MAX)))) {
    iz = use ? iz : 0.0f;
  } else {
    iz = use ? iz : 0.0f;
    pc0 = use ? pc0 : 0.0f;
    pc1 = use ? pc1 : 0.0f;
    pc2 = use ? pc2 : 0.0f;
    ph0 = use ? ph0 : 0.0f;
    ph1 = use ? ph1 : 0.0f;
    e0 = use ? e0 : 0.0f;
    e1 = use ? e1 : 0.0f;
  }
  float J0[6], J1[6];
  {
#pragma clang fp contract(off)
    const float iz2 = iz * iz;  // src/picp_solver.cpp:45-50
    const float jp0 = -(ph0 * iz2), jp1 = -(ph1 * iz2);
    const float a00 = iz * C.k00, a02 = iz * C.k02 + jp0;
    const float a11 = iz * C.k11, a12 = iz * C.k12 + jp1;
    J0[0] = a00; J0[1] = 0.0f; J0[2] = a02;
    J0[3] = a02 * pc1;
    J0[4] = a00 * pc2 - a02 * pc0;
    J0[5] = -(a00 * pc1);
    J1[0] = 0.0f; J1[1] = a11; J1[2] = a12;
    J1[3] = -(a11 * pc2) + a12 * pc1;
    J1[4] = -(a12 * pc0);
    J1[5] = a11 * pc0;
  }
  float W0[6], W1[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    W0[i] = KEEP ? w * J0[i] : J0[i];
    W1[i] = KEEP ? w * J1[i] : J1[i];
  }
  int k = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
#pragma unroll
    for (int j = i; j < 6; ++j) {
      float h = a.h[k];
      if (i != 0 && j != 0) h = fmaf(W1[i], J1[j], h);  // J1[0] == 0
      if (i != 1 && j != 1) h = fmaf(W0[i], J0[j], h);  // J0[1] == 0
      a.h[k] = h;
      ++k;
    }
    float bb = a.b[i];
    if (i != 0) bb = fmaf(W1[i], e1, bb);
    if (i != 1) bb = fmaf(W0[i], e0, bb);
    a.b[i] = bb;
  }
}

// The general-K per-item math of accumulate_one up to the weighted Jacobian (for the packed
// pair accumulation): outputs are zeroed for an unused item, w is its kernel weight.
struct Item {
  float J0[6], J1[6], e0, e1, w, chi;
  bool inl, valid;
};

__device__ __forceinline__ void item_general(const Pose& T, const Cam& C, float thr, bool keep,
                                             float x, float y, float z, float u, float v,
                                             bool in_range, Item& o) {
  float pc0, pc1, pc2, ph0, ph1, ph2, iz, e0, e1, chi;
  bool valid;
  {
#pragma clang fp contract(off)
    pc0 = ((T.r00 * x + T.r01 * y) + T.r02 * z) + T.t0;
    pc1 = ((T.r10 * x + T.r11 * y) + T.r12 * z) + T.t1;
    pc2 = ((T.r20 * x + T.r21 * y) + T.r22 * z) + T.t2;
    ph0 = (C.k00 * pc0 + C.k01 * pc1) + C.k02 * pc2;
    ph1 = (C.k10 * pc0 + C.k11 * pc1) + C.k12 * pc2;
    ph2 = (C.k20 * pc0 + C.k21 * pc1) + C.k22 * pc2;
    iz = 1.0f / ph2;
    const float ix = ph0 * iz;
    const float iy = ph1 * iz;
    // bitwise, not short-circuit: the same predicate without per-item exec-mask branches
    valid = in_range & !(pc2 <= 0.0f) & !((ix < 0.0f) | (ix > C.maxx) | (iy < 0.0f) | (iy > C.maxy));
    e0 = ix - u;
    e1 = iy - v;
    chi = e0 * e0 + e1 * e1;
  }
  const bool outlier = chi > thr;
  const bool inl = valid & !outlier;
  const bool use = inl | (valid & keep);
  const float lambda = outlier ? sqrtf(thr / chi) : 1.0f;
  o.w = use ? (inl ? 1.0f : lambda) : 0.0f;
  o.chi = chi;
  o.inl = inl;
  o.valid = valid;
  iz = use ? iz : 0.0f;
  pc0 = use ? pc0 : 0.0f;
  pc1 = use ? pc1 : 0.0f;
  pc2 = use ? pc2 : 0.0f;
  ph0 = use ? ph0 : 0.0f;
  ph1 = use ? ph1 : 0.0f;
  o.e0 = use ? e0 : 0.0f;
  o.e1 = use ? e1 : 0.0f;
  const float iz2 = iz * iz;
  const float jp02 = -ph0 * iz2, jp12 = -ph1 * iz2;
  const float a00 = iz * C.k00 + jp02 * C.k20;
  const float a01 = iz * C.k01 + jp02 * C.k21;
  const float a02 = iz * C.k02 + jp02 * C.k22;
  const float a10 = iz * C.k10 + jp12 * C.k20;
  const float a11 = iz * C.k11 + jp12 * C.k21;
  const float a12 = iz * C.k12 + jp12 * C.k22;
  o.J0[0] = a00; o.J0[1] = a01; o.J0[2] = a02;
  o.J0[3] = a02 * pc1 - a01 * pc2;
  o.J0[4] = a00 * pc2 - a02 * pc0;
  o.J0[5] = a01 * pc0 - a00 * pc1;
  o.J1[0] = a10; o.J1[1] = a11; o.J1[2] = a12;
  o.J1[3] = a12 * pc1 - a11 * pc2;
  o.J1[4] = a10 * pc2 - a12 * pc0;
  o.J1[5] = a11 * pc0 - a10 * pc1;
}

// H += w (J0^T J0 + J1^T J1), b += w (J0^T e0 + J1^T e1) for both slots; SPARSE skips the
// pinhole Jacobian's structural zeros J0[1] = J1[0] = 0; !WEIGHTED: w is 1 for every item whose
// J is not zero (outliers rejected), so w is not applied
template <bool SPARSE, bool WEIGHTED>
__device__ __forceinline__ void acc2_normal(const f2 J0[6], const f2 J1[6], f2 e0, f2 e1, f2 w,
                                            Acc2& a) {
  f2 W0[6], W1[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    W0[i] = WEIGHTED ? w * J0[i] : J0[i];
    W1[i] = WEIGHTED ? w * J1[i] : J1[i];
  }
  int k = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
#pragma unroll
    for (int j = i; j < 6; ++j) {
      f2 h = a.h[k];
      if (!SPARSE || (i != 0 && j != 0)) h = __builtin_elementwise_fma(W1[i], J1[j], h);
      if (!SPARSE || (i != 1 && j != 1)) h = __builtin_elementwise_fma(W0[i], J0[j], h);
      a.h[k] = h;
      ++k;
    }
    f2 bb = a.b[i];
    if (!SPARSE || i != 0) bb = __builtin_elementwise_fma(W1[i], e1, bb);
    if (!SPARSE || i != 1) bb = __builtin_elementwise_fma(W0[i], e0, bb);
    a.b[i] = bb;
  }
}

__device__ __forceinline__ void acc2_stats(f2 chi, bool inlA, bool inlB, bool validA, bool validB,
                                           Acc2& a, Cnt& n) {
  a.chi_in += (f2){inlA ? chi.x : 0.0f, inlB ? chi.y : 0.0f};
  a.chi_out += (f2){(validA & !inlA) ? chi.x : 0.0f, (validB & !inlB) ? chi.y : 0.0f};
  cnt_add(n, inlA, validA);
  cnt_add(n, inlB, validB);
}

// A pair of correspondences, pinhole K: accumulate_pinhole's exact arithmetic with every
// elementwise step written on float2 (A in .x, B in .y).  Only the correctly rounded reciprocal, the
// compares and the selects stay per item.  Contraction is off exactly where the oracle has it
// off (gate and Jacobian), so both items are bit-identical to the scalar path.
// The camera-frame depth of a pair, in the exact operation order of accumulate_pinhole2 (so the
// compiler shares it): callers check a whole section of pairs for the fast reciprocal at once.
__device__ __forceinline__ f2 pair_depth(const Pose& T, f2 x, f2 y, f2 z) {
#pragma clang fp contract(off)
  return ((T.r20 * x + T.r21 * y) + T.r22 * z) + T.t2;  // src/camera.h:26, row 2
}

__device__ __forceinline__ bool pair_rcp_safe(const Pose& T, f2 x, f2 y, f2 z) {
  const f2 d = pair_depth(T, x, y, z);
  return rcp_safe(d.x) & rcp_safe(d.y);
}

template <bool KEEP, int RCP = RCP_CHECK>
__device__ __forceinline__ void accumulate_pinhole2(const Pose& T, const Cam& C, float thr,
                                                    float inv_thr, f2 x, f2 y, f2 z,
                                                    f2 u, f2 v, bool inA, bool inB, Acc2& a, Cnt& n) {
  f2 pc0, pc1, pc2, ph0, ph1, iz, e0, e1, chi;
  bool validA, validB;
  {
#pragma clang fp contract(off)
    pc0 = ((T.r00 * x + T.r01 * y) + T.r02 * z) + T.t0;  // src/camera.h:26
    pc1 = ((T.r10 * x + T.r11 * y) + T.r12 * z) + T.t1;
    pc2 = pair_depth(T, x, y, z);
    ph0 = C.k00 * pc0 + C.k02 * pc2;  // src/camera.h:29 without the zero terms
    ph1 = C.k11 * pc1 + C.k12 * pc2;
    // ph2 == pc2 exactly; the correctly rounded reciprocal per item (rcp_rn, exhaustively
    // verified), the IEEE division only when a lane of the wave holds an extreme value
    if (RCP == RCP_FAST || (RCP == RCP_CHECK && __all(rcp_safe(pc2.x) & rcp_safe(pc2.y)))) {
      iz.x = rcp_rn(pc2.x);
      iz.y = rcp_rn(pc2.y);
    } else {
      iz.x = 1.0f / pc2.x;
      iz.y = 1.0f / pc2.y;
    }
    const f2 ix = ph0 * iz;
    const f2 iy = ph1 * iz;
    // bitwise, not short-circuit: the same predicate without per-item exec-mask branches
    validA = inA & !(pc2.x <= 0.0f) &
             !((ix.x < 0.0f) | (ix.x > C.maxx) | (iy.x < 0.0f) | (iy.x > C.maxy));
    validB = inB & !(pc2.y <= 0.0f) &
             !((ix.y < 0.0f) | (ix.y > C.maxx) | (iy.y < 0.0f) | (iy.y > C.maxy));
    e0 = ix - u;
    e1 = iy - v;
    chi = e0 * e0 + e1 * e1;
  }
  const bool outA = chi.x > thr, outB = chi.y > thr;
  const bool inlA = validA & !outA, inlB = validB & !outB;
  const bool useA = inlA | (validA & KEEP), useB = inlB | (validB & KEEP);
  f2 w = {1.0f, 1.0f};
  if constexpr (KEEP) {  // the robust weight only when outliers are kept
    const f2 q = chi * inv_thr;
    w = (f2){useA ? (inlA ? 1.0f : __builtin_amdgcn_rsqf(q.x)) : 0.0f,
             useB ? (inlB ? 1.0f : __builtin_amdgcn_rsqf(q.y)) : 0.0f};
  }
  acc2_stats(chi, inlA, inlB, validA, validB, a, n);
  // a skipped item gets weight 0 and finite inputs, so it can never inject inf/NaN.  (Skipping
  // these selects for waves of projectable items, as accumulate_pinhole does, measured 1-4 %
  // slower here: the branches split the unrolled pairs' straight-line schedule.)
#define PICP_Z2(val) val = (f2){useA ? val.x : 0.0f, useB ? val.y : 0.0f}
  PICP_Z2(iz); PICP_Z2(pc0); PICP_Z2(pc1); PICP_Z2(pc2); PICP_Z2(ph0); PICP_Z2(ph1); PICP_Z2(e0); PICP_Z2(e1);
#undef PICP_Z2
  f2 J0[6], J1[6];
  {
#pragma clang fp contract(off)
    const f2 iz2 = iz * iz;  // src/picp_solver.cpp:45-52, the oracle's operation order
    const f2 jp0 = -(ph0 * iz2), jp1 = -(ph1 * iz2);
    const f2 a00 = iz * C.k00, a02 = iz * C.k02 + jp0;
    const f2 a11 = iz * C.k11, a12 = iz * C.k12 + jp1;
    const f2 zero = {0.0f, 0.0f};
    J0[0] = a00; J0[1] = zero; J0[2] = a02;
    J0[3] = a02 * pc1;
    J0[4] = a00 * pc2 - a02 * pc0;
    J0[5] = -(a00 * pc1);
    J1[0] = zero; J1[1] = a11; J1[2] = a12;
    J1[3] = -(a11 * pc2) + a12 * pc1;
    J1[4] = -(a12 * pc0);
    J1[5] = a11 * pc0;
  }
  acc2_normal<true, KEEP>(J0, J1, e0, e1, w, a);
}

// A pair of correspondences, pinhole K, into ONE accumulation slot: accumulate_pinhole2's math on
// float2 (two independent dependency chains through the projection, the gate and the Jacobian:
// the instruction-level parallelism the two-slot form buys), then item A's terms and item B's
// terms added into the same sums in that order -- exactly accumulate_pinhole(A) followed by
// accumulate_pinhole(B), so the sums are the one-slot form's bits.  A skipped item's J and e are
// zeroed (exact zeros: fma(+-0, x, h) == h, the sums never being -0), as accumulate_pinhole's
// zeroing path does.
template <bool KEEP, int RCP = RCP_CHECK>
__device__ __forceinline__ void accumulate_pinhole_p1(const Pose& T, const Cam& C, float thr, float inv_thr,
                                                      f2 x, f2 y, f2 z, f2 u, f2 v, bool inA, bool inB, Acc& a,
                                                      Cnt& n) {
  f2 pc0, pc1, pc2, ph0, ph1, iz, e0, e1, chi;
  bool validA, validB;
  {
#pragma clang fp contract(off)
    pc0 = ((T.r00 * x + T.r01 * y) + T.r02 * z) + T.t0;  // src/camera.h:26
    pc1 = ((T.r10 * x + T.r11 * y) + T.r12 * z) + T.t1;
    pc2 = pair_depth(T, x, y, z);
    ph0 = C.k00 * pc0 + C.k02 * pc2;  // src/camera.h:29 without the zero terms
    ph1 = C.k11 * pc1 + C.k12 * pc2;
    if (RCP == RCP_FAST || (RCP == RCP_CHECK && __all(rcp_safe(pc2.x) & rcp_safe(pc2.y)))) {
      iz.x = rcp_rn(pc2.x);
      iz.y = rcp_rn(pc2.y);
    } else {
      iz.x = 1.0f / pc2.x;
      iz.y = 1.0f / pc2.y;
    }
    const f2 ix = ph0 * iz;
    const f2 iy = ph1 * iz;
    validA = inA & !(pc2.x <= 0.0f) & !((ix.x < 0.0f) | (ix.x > C.maxx) | (iy.x < 0.0f) | (iy.x > C.maxy));
    validB = inB & !(pc2.y <= 0.0f) & !((ix.y < 0.0f) | (ix.y > C.maxx) | (iy.y < 0.0f) | (iy.y > C.maxy));
    e0 = ix - u;
    e1 = iy - v;
    chi = e0 * e0 + e1 * e1;
  }
  const bool outA = chi.x > thr, outB = chi.y > thr;
  const bool inlA = validA & !outA, inlB = validB & !outB;
  const bool useA = inlA | (validA & KEEP), useB = inlB | (validB & KEEP);
  f2 w = {1.0f, 1.0f};
  if constexpr (KEEP) {
    const f2 q = chi * inv_thr;
    w = (f2){useA ? (inlA ? 1.0f : __builtin_amdgcn_rsqf(q.x)) : 0.0f,
             useB ? (inlB ? 1.0f : __builtin_amdgcn_rsqf(q.y)) : 0.0f};
  }
  a.chi_in += inlA ? chi.x : 0.0f;  // item A, then item B: the one-slot order
  a.chi_out += (validA & outA) ? chi.x : 0.0f;
  a.chi_in += inlB ? chi.y : 0.0f;
  a.chi_out += (validB & outB) ? chi.y : 0.0f;
  cnt_add(n, inlA, validA);
  cnt_add(n, inlB, validB);
#define PICP_Z2(val) val = (f2){useA ? val.x : 0.0f, useB ? val.y : 0.0f}
  PICP_Z2(iz); PICP_Z2(pc0); PICP_Z2(pc1); PICP_Z2(pc2); PICP_Z2(ph0); PICP_Z2(ph1); PICP_Z2(e0); PICP_Z2(e1);
#undef PICP_Z2
  f2 J0[6], J1[6];
  {
#pragma clang fp contract(off)
    const f2 iz2 = iz * iz;  // src/picp_solver.cpp:45-52, the oracle's operation order
    const f2 jp0 = -(ph0 * iz2), jp1 = -(ph1 * iz2);
    const f2 a00 = iz * C.k00, a02 = iz * C.k02 + jp0;
    const f2 a11 = iz * C.k11, a12 = iz * C.k12 + jp1;
    const f2 zero = {0.0f, 0.0f};
    J0[0] = a00; J0[1] = zero; J0[2] = a02;
    J0[3] = a02 * pc1;
    J0[4] = a00 * pc2 - a02 * pc0;
    J0[5] = -(a00 * pc1);
    J1[0] = zero; J1[1] = a11; J1[2] = a12;
    J1[3] = -(a11 * pc2) + a12 * pc1;
    J1[4] = -(a12 * pc0);
    J1[5] = a11 * pc0;
  }
#pragma unroll
  for (int it = 0; it < 2; ++it) {  // item A's terms, then item B's (accumulate_pinhole's order)
    float W0[6], W1[6], K0[6], K1[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      K0[i] = it ? J0[i].y : J0[i].x;
      K1[i] = it ? J1[i].y : J1[i].x;
      const float wi = it ? w.y : w.x;
      W0[i] = KEEP ? wi * K0[i] : K0[i];
      W1[i] = KEEP ? wi * K1[i] : K1[i];
    }
    const float f0 = it ? e0.y : e0.x, f1 = it ? e1.y : e1.x;
    int k = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
#pragma unroll
      for (int j = i; j < 6; ++j) {
        float h = a.h[k];
        if (i != 0 && j != 0) h = fmaf(W1[i], K1[j], h);  // J1[0] == 0
        if (i != 1 && j != 1) h = fmaf(W0[i], K0[j], h);  // J0[1] == 0
        a.h[k] = h;
        ++k;
      }
      float bb = a.b[i];
      if (i != 0) bb = fmaf(W1[i], f1, bb);
      if (i != 1) bb = fmaf(W0[i], f0, bb);
      a.b[i] = bb;
    }
  }
}

// A pair of correspondences, general K: per-item math (item_general), paired accumulation.
__device__ __forceinline__ void accumulate_general2(const Pose& T, const Cam& C, float thr, bool keep,
                                                    f2 x, f2 y, f2 z, f2 u, f2 v, bool inA,
                                                    bool inB, Acc2& a, Cnt& n) {
  Item A, B;
  item_general(T, C, thr, keep, x.x, y.x, z.x, u.x, v.x, inA, A);
  item_general(T, C, thr, keep, x.y, y.y, z.y, u.y, v.y, inB, B);
  acc2_stats((f2){A.chi, B.chi}, A.inl, B.inl, A.valid, B.valid, a, n);
  f2 J0[6], J1[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    J0[i] = (f2){A.J0[i], B.J0[i]};
    J1[i] = (f2){A.J1[i], B.J1[i]};
  }
  acc2_normal<false, true>(J0, J1, (f2){A.e0, B.e0}, (f2){A.e1, B.e1}, (f2){A.w, B.w}, a);
}

// PH: the per-item variant (PICP_V_*); keep is read only by the general variant; RCP: how the
// pinhole variants take the reciprocal (RCP_*)
template <int PH, int RCP = RCP_CHECK>
__device__ __forceinline__ void accumulate2(const Pose& T, const Cam& C, float thr, float inv_thr,
                                            bool keep, f2 x, f2 y, f2 z, f2 u, f2 v, bool inA,
                                            bool inB, Acc2& a, Cnt& n) {
  if constexpr (PH == PICP_V_GENERAL)
    accumulate_general2(T, C, thr, keep, x, y, z, u, v, inA, inB, a, n);
  else
    accumulate_pinhole2<PH == PICP_V_PINHOLE_KEEP, RCP>(T, C, thr, inv_thr, x, y, z, u, v, inA, inB, a, n);
}

// NPT register-resident items per lane (item k at lane + k * stride) as pairs (k, k + 1) (NPT == 1:
// slot B repeats item 0, masked), with ONE wave vote on the fast reciprocal for the whole set
// instead of one per pair: the pairs then run as one straight-line block (a vote per pair split
// them into blocks, so every per-item predicate crossing the block edge was kept as a 0/1 VGPR and
// compared again, and the masks' scalar registers spilled).
template <int PH, int NPT>
__device__ __forceinline__ void accumulate_regs(const Pose& T, const Cam& C, float thr, float inv_thr,
                                                bool keep, const float* xs, const float* ys,
                                                const float* zs, const float* us, const float* vs,
                                                int first, int stride, int n, Acc2& a, Cnt& cnt) {
  bool fast = true;
  if constexpr (PH != PICP_V_GENERAL) {
#pragma unroll
    for (int k = 0; k < NPT; k += 2) {
      const int k1 = (k + 1 < NPT) ? k + 1 : k;
      fast &= pair_rcp_safe(T, (f2){xs[k], xs[k1]}, (f2){ys[k], ys[k1]}, (f2){zs[k], zs[k1]});
    }
  }
  auto run = [&](auto rcp) {
#pragma unroll
    for (int k = 0; k < NPT; k += 2) {
      const int k1 = (k + 1 < NPT) ? k + 1 : k;
      accumulate2<PH, decltype(rcp)::value>(T, C, thr, inv_thr, keep, (f2){xs[k], xs[k1]}, (f2){ys[k], ys[k1]},
                                            (f2){zs[k], zs[k1]}, (f2){us[k], us[k1]}, (f2){vs[k], vs[k1]},
                                            first + k * stride < n, k + 1 < NPT && first + (k + 1) * stride < n,
                                            a, cnt);
    }
  };
  if (PH == PICP_V_GENERAL || __all(fast))
    run(std::integral_constant<int, RCP_FAST>());
  else
    run(std::integral_constant<int, RCP_DIV>());
}

// Which accumulation form a kernel with NPT register-resident items per lane uses.  Measured on
// MI355X with the unpacked build (profiles/r03/acc/): one slot is faster at small NPT (C5, NPT 4:
// +2.7 %), the two-slot pair form at NPT 8 (C3 +5-9 %, C4 +17 %: its two independent
// accumulation chains and its paired LDS/stream loops).  -DPICP_ACC_PAIRS / -DPICP_ACC_ONE force
// one form for A/B builds.
// One-slot accumulation with the per-item math in pairs (accumulate_pinhole_p1): the same bits
// as item by item.  -DPICP_P1=0 restores the item-by-item form for A/B builds.
#ifndef PICP_P1
#define PICP_P1 0
#endif

__host__ __device__ constexpr bool acc_pairs(int npt) {
#if defined(PICP_ACC_PAIRS)
  return true;
#elif defined(PICP_ACC_ONE)
  return false;
#else
  return npt >= 8;
#endif
}

// accumulate_regs with ONE accumulator slot, item by item (the default since the device code is
// built without packed FP32, hipcc_nopk.sh): the pair form's two slots only paid for themselves
// as packed instructions; unpacked, they double the accumulator registers (58 instead of 29 per
// lane) and every per-pair select.  The fast-reciprocal vote is taken once for the whole set.
// The sum runs over the items in order k = 0 .. NPT-1 (the pair form summed even and odd items in
// separate slots): the bits differ from it in the last place, within the H/b tolerance.
template <int PH, int NPT>
__device__ __forceinline__ void accumulate_regs1(const Pose& T, const Cam& C, float thr, float inv_thr,
                                                 bool keep, const float* xs, const float* ys,
                                                 const float* zs, const float* us, const float* vs,
                                                 int first, int stride, int n, Acc& a, Cnt& cnt) {
  if constexpr (PH == PICP_V_GENERAL) {
#pragma unroll
    for (int k = 0; k < NPT; ++k)
      accumulate_one(T, C, thr, keep, xs[k], ys[k], zs[k], us[k], vs[k], first + k * stride < n, a, cnt);
  } else {
    bool fast = true;
#pragma unroll
    for (int k = 0; k < NPT; ++k) fast &= rcp_safe(item_depth(T, xs[k], ys[k], zs[k]));
    auto run = [&](auto rcp) {
      constexpr bool KP = PH == PICP_V_PINHOLE_KEEP;
      constexpr int R = decltype(rcp)::value;
#if PICP_P1
      // items in pairs (k, k + 1) through accumulate_pinhole_p1: the same sums in the same order
      // as item by item, with two dependency chains through the per-item math
#pragma unroll
      for (int k = 0; k + 1 < NPT; k += 2) {
        const bool inA = first + k * stride < n, inB = first + (k + 1) * stride < n;
        if (k + 2 < NPT || __any(inB))  // the last slot only in waves that hold an item there
          accumulate_pinhole_p1<KP, R>(T, C, thr, inv_thr, (f2){xs[k], xs[k + 1]}, (f2){ys[k], ys[k + 1]},
                                       (f2){zs[k], zs[k + 1]}, (f2){us[k], us[k + 1]}, (f2){vs[k], vs[k + 1]}, inA,
                                       inB, a, cnt);
        else
          accumulate_pinhole<KP, R>(T, C, thr, inv_thr, xs[k], ys[k], zs[k], us[k], vs[k], inA, a, cnt);
      }
      if constexpr (NPT & 1)
        accumulate_pinhole<KP, R>(T, C, thr, inv_thr, xs[NPT - 1], ys[NPT - 1], zs[NPT - 1], us[NPT - 1],
                                  vs[NPT - 1], first + (NPT - 1) * stride < n, a, cnt);
#else
#pragma unroll
      for (int k = 0; k < NPT; ++k)
        // the last slot only in waves that hold an item there (a wave-uniform branch): a frame
        // that fills 3.5 of 4 slots leaves whole waves empty in it, and with waves dealt to the
        // SIMDs in turn every SIMD then issues one slot less when n <= (NPT - 1/2) x BS (C5's
        // ~1,750 correspondences on 2,048 slots).  A skipped item adds exact zeros: same bits.
        if (NPT < 2 || k + 1 < NPT || __any(first + k * stride < n))
          accumulate_pinhole<KP, R>(T, C, thr, inv_thr, xs[k], ys[k], zs[k], us[k], vs[k], first + k * stride < n, a,
                                    cnt);
#endif
    };
    if (__all(fast))
      run(std::integral_constant<int, RCP_FAST>());
    else
      run(std::integral_constant<int, RCP_DIV>());
  }
}

// One streamed (LDS or HBM) item, pinhole or general, the fast reciprocal by a vote of the lanes
// that run this item (the loops that call it are divergent).
template <int PH>
__device__ __forceinline__ void accumulate_item(const Pose& T, const Cam& C, float thr, float inv_thr,
                                                bool keep, float x, float y, float z, float u, float v,
                                                bool in_range, Acc& a, Cnt& n) {
  if constexpr (PH == PICP_V_GENERAL) {
    accumulate_one(T, C, thr, keep, x, y, z, u, v, in_range, a, n);
  } else {
    if (__all(rcp_safe(item_depth(T, x, y, z))))
      accumulate_pinhole<PH == PICP_V_PINHOLE_KEEP, RCP_FAST>(T, C, thr, inv_thr, x, y, z, u, v, in_range, a, n);
    else
      accumulate_pinhole<PH == PICP_V_PINHOLE_KEEP, RCP_DIV>(T, C, thr, inv_thr, x, y, z, u, v, in_range, a, n);
  }
}

// Streamed (LDS or HBM) items i, i + stride, i + 2 stride, ... (i = first) of one lane into one
// slot, in that order: pairs through accumulate_pinhole_p1 (the fast reciprocal by a vote of the
// lanes that run the pair), the general variant item by item.  get(i, x, y, z, u, v) loads item i.
template <int PH, typename Get>
__device__ __forceinline__ void accumulate_stream1(const Pose& T, const Cam& C, float thr, float inv_thr, bool keep,
                                                   int first, int stride, int count, Get get, Acc& a, Cnt& n) {
#if PICP_P1
  if constexpr (PH != PICP_V_GENERAL) {
    constexpr bool KP = PH == PICP_V_PINHOLE_KEEP;
    for (int i = first; i < count; i += 2 * stride) {
      const bool inB = i + stride < count;
      const int j = inB ? i + stride : i;
      float x0, y0, z0, u0, v0, x1, y1, z1, u1, v1;
      get(i, x0, y0, z0, u0, v0);
      get(j, x1, y1, z1, u1, v1);
      const f2 x = {x0, x1}, y = {y0, y1}, z = {z0, z1};
      if (__all(pair_rcp_safe(T, x, y, z)))
        accumulate_pinhole_p1<KP, RCP_FAST>(T, C, thr, inv_thr, x, y, z, (f2){u0, u1}, (f2){v0, v1}, true, inB, a, n);
      else
        accumulate_pinhole_p1<KP, RCP_DIV>(T, C, thr, inv_thr, x, y, z, (f2){u0, u1}, (f2){v0, v1}, true, inB, a, n);
    }
    return;
  }
#endif
  for (int i = first; i < count; i += stride) {
    float x, y, z, u, v;
    get(i, x, y, z, u, v);
    accumulate_item<PH>(T, C, thr, inv_thr, keep, x, y, z, u, v, true, a, n);
  }
}

__device__ __forceinline__ void acc_zero(Acc& a) {
#pragma unroll
  for (int i = 0; i < 21; ++i) a.h[i] = 0.0f;
#pragma unroll
  for (int i = 0; i < 6; ++i) a.b[i] = 0.0f;
  a.chi_in = a.chi_out = 0.0f;
}

__device__ __forceinline__ void acc_fold(const Acc& a, float v[PICP_NPART]) {
#pragma unroll
  for (int i = 0; i < 21; ++i) v[PICP_P_H + i] = a.h[i];
#pragma unroll
  for (int i = 0; i < 6; ++i) v[PICP_P_B + i] = a.b[i];
  v[PICP_P_CHI_IN] = a.chi_in;
  v[PICP_P_CHI_OUT] = a.chi_out;
  v[PICP_P_N_IN] = 0.0f;
  v[PICP_P_N_PROJ] = 0.0f;
  v[31] = 0.0f;
}

// one correspondence with the variant chosen at compile time
template <int PH>
__device__ __forceinline__ void accumulate(const Pose& T, const Cam& C, float thr, float inv_thr,
                                           bool keep, float x, float y, float z, float u,
                                           float v, bool in_range, Acc& a, Cnt& n) {
  if constexpr (PH == PICP_V_GENERAL)
    accumulate_one(T, C, thr, keep, x, y, z, u, v, in_range, a, n);
  else
    accumulate_pinhole<PH == PICP_V_PINHOLE_KEEP>(T, C, thr, inv_thr, x, y, z, u, v, in_range, a, n);
}

__host__ __device__ inline bool is_pinhole(const float K[9]) {  // column-major K
  return K[1] == 0.0f && K[2] == 0.0f && K[3] == 0.0f && K[5] == 0.0f && K[8] == 1.0f;
}

}  // namespace picp

// launch-time camera path: pinhole unless K is general or PICP_FORCE_GENERAL_K=1 (A/B checks)
inline bool picp_use_pinhole(const float K[9]) {
  static const bool force_general = [] {
    const char* e = getenv("PICP_FORCE_GENERAL_K");
    return e && atoi(e) != 0;
  }();
  return !force_general && picp::is_pinhole(K);
}

// launch-time per-item variant (PICP_V_*): the camera path, and for the pinhole path whether
// outliers are kept (a compile-time weight)
inline int picp_variant(const float K[9], int keep_outliers) {
  if (!picp_use_pinhole(K)) return PICP_V_GENERAL;
  return keep_outliers ? PICP_V_PINHOLE_KEEP : PICP_V_PINHOLE;
}

namespace picp {

// Cross-lane moves without the LDS crossbar.  gfx950 v_permlane32_swap / v_permlane16_swap
// exchange half-waves / odd-even 16-lane rows between two registers; DPP reads a partner
// lane inside a 16-lane row (row_mirror l^15, row_half_mirror l^7, quad_perm l^2, l^1).
// bound_ctrl on: a lane whose source lane is disabled in EXEC reads 0, so the result never depends
// on the destination's old contents (every call site runs with EXEC full, where no source lane is
// disabled).  Passing the source as DPP "old" instead (round 4) tied the destination to it and
// cost a register copy per move: C2/C3 1-2 % slower in interleaved A/B (profiles/r05/ab_regress/).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
#define DPP_ROW_MIRROR 0x140
#define DPP_ROW_HALF_MIRROR 0x141
#define DPP_QUAD_XOR2 0x4E  // quad_perm [2,3,0,1]
#define DPP_QUAD_XOR1 0xB1  // quad_perm [1,0,3,2]

// Halving-butterfly step inside a 16-lane row: lanes l and P(l) (P an involution that flips
// bit HB) exchange the half of the 2*HALF values the other keeps.
template <int CTRL, int HB, int HALF>
__device__ __forceinline__ void bfly_dpp(float* v, int lane) {
  const bool hi = (lane >> HB) & 1;
#pragma unroll
  for (int i = 0; i < HALF; ++i) {
    const float send = hi ? v[i] : v[i + HALF];
    const float keep = hi ? v[i + HALF] : v[i];
    v[i] = keep + dpp<CTRL>(send);
  }
}

// Sum 32 per-lane values over the 64 lanes of a wave (32 -> 16 -> 8 -> 4 -> 2 -> 1 values per
// lane).  The swap steps need no select: after v_permlane32_swap(a=v[i], b=v[i+16]) the low
// half holds (own v[i], partner v[i]) and the high half (partner v[i+16], own v[i+16]), so a+b
// is the pair sum of the half each lane keeps.  Returns, in every lane, the wave total of value
// index (lane >> 1).
__device__ __forceinline__ float wave_reduce32_bperm(float* v, int lane) {
  // the half-wave exchanges through ds_bpermute (bit-identical sums in the same order)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const bool hi = (lane & 32) != 0;
    const float send = hi ? v[i] : v[i + 16], keep = hi ? v[i + 16] : v[i];
    v[i] = keep + __shfl_xor(send, 32);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool hi = (lane & 16) != 0;
    const float send = hi ? v[i] : v[i + 8], keep = hi ? v[i + 8] : v[i];
    v[i] = keep + __shfl_xor(send, 16);
  }
  bfly_dpp<DPP_ROW_MIRROR, 3, 4>(v, lane);
  bfly_dpp<DPP_ROW_HALF_MIRROR, 2, 2>(v, lane);
  bfly_dpp<DPP_QUAD_XOR2, 1, 1>(v, lane);
  return v[0] + dpp<DPP_QUAD_XOR1>(v[0]);
}

__device__ __forceinline__ float wave_reduce32(float* v, int lane) {
#ifdef PICP_NO_PERMLANE_SWAP
  // the half-wave exchanges through ds_bpermute (bit-identical sums in the same order).  Results
  // of the v_permlane*_swap form below moved in the last bits when other kernels ran beside it on
  // MI355X; this form did not.  Costs C2 3 %, C4 15 %, C5 10 %.
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const bool hi = (lane & 32) != 0;
    const float send = hi ? v[i] : v[i + 16], keep = hi ? v[i + 16] : v[i];
    v[i] = keep + __shfl_xor(send, 32);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool hi = (lane & 16) != 0;
    const float send = hi ? v[i] : v[i + 8], keep = hi ? v[i + 8] : v[i];
    v[i] = keep + __shfl_xor(send, 16);
  }
#else
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 16]), false, false);
    v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 8]), false, false);
    v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#endif
  bfly_dpp<DPP_ROW_MIRROR, 3, 4>(v, lane);
  bfly_dpp<DPP_ROW_HALF_MIRROR, 2, 2>(v, lane);
  bfly_dpp<DPP_QUAD_XOR2, 1, 1>(v, lane);
  return v[0] + dpp<DPP_QUAD_XOR1>(v[0]);
}

// 1/d in float: hardware v_rcp_f32 estimate refined by one Newton step (<= 1 ulp for normal
// d); |d| <= FLT_MIN -> 0 (Eigen's LDLT zero-pivot rule for float, src/picp_solver.cpp:102).
__device__ __forceinline__ float rcp32(float d) {
  float r = __builtin_amdgcn_rcpf(d);
  r = fmaf(r, fmaf(-d, r, 1.0f), r);
  return (fabsf(d) > FLT_MIN) ? r : 0.0f;
}

// Damped normal equations -> dx, in float32, the precision the reference solves in
// (Matrix6f::ldlt, src/picp_solver.cpp:102); H and b arrive as exact double sums.  LDL^T without
// pivoting, by Gaussian elimination on the LOWER triangle (H + damping*I is SPD: Eigen's diagonal
// pivoting only changes rounding): step j scales column j by 1/d_j and updates the trailing
// lower triangle; the back substitution reads U = D L^T from the lower entries (symmetry).  Pivot
// reciprocals are the hardware v_rcp_f32 (<= 1 ulp).  A pivot with |d| <= FLT_MIN gives 1/d = 0,
// Eigen's zero-pivot rule for float; that test is kept off the pivot chain (a flag, and the rare
// flagged system is solved again with the guard in the chain).  One lane, registers only, every
// index compile-time: the per-round critical path of every kernel (tools/ubench/parts_ubench).
// Row r of the system is read from the converted totals tw (total_word: damping folded into the
// diagonal, -b), upper triangle row-major.
__device__ __forceinline__ int tri_index(int r, int c) {  // upper-triangle slot of (min, max)
  const int lo = r < c ? r : c, hi = r < c ? c : r;
  return PICP_P_H + lo * (11 - lo) / 2 + hi;
}

template <bool GUARD>
__device__ __forceinline__ bool ldl6_solve(const float* tw, float dx[6]) {
  float a[6][6], rhs[6], id[6];
  bool bad = false;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
#pragma unroll
    for (int c = 0; c <= i; ++c) a[i][c] = tw[tri_index(c, i)];
    rhs[i] = tw[PICP_P_B + i];
  }
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const float d = a[j][j];
    float inv = __builtin_amdgcn_rcpf(d);
    if (GUARD) inv = (fabsf(d) > FLT_MIN) ? inv : 0.0f;
    else bad |= !(fabsf(d) > FLT_MIN);
    id[j] = inv;
    float f[6];
#pragma unroll
    for (int i = j + 1; i < 6; ++i) f[i] = a[i][j] * inv;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
#pragma unroll
      for (int c = j + 1; c <= i; ++c) a[i][c] = fmaf(-f[i], a[c][j], a[i][c]);
      rhs[i] = fmaf(-f[i], rhs[j], rhs[i]);
    }
  }
#pragma unroll
  for (int k = 5; k >= 0; --k) {
    const float x = rhs[k] * id[k];
    dx[k] = x;
#pragma unroll
    for (int i = 0; i < k; ++i) rhs[i] = fmaf(-a[k][i], x, rhs[i]);
  }
  return bad;
}

__device__ __forceinline__ void ldl6_solve(const float* tw, float dx[6]) {
  if (ldl6_solve<false>(tw, dx)) ldl6_solve<true>(tw, dx);  // a (near-)zero pivot: rare
}

// DPP row_newbcast:N (gfx950): lane N of each 16-lane row, to every lane of that row.  bound_ctrl
// set: a lane whose source is invalid would get 0, never a stale register (no source is invalid
// here: every lane of a finishing wave is active), and no tied "old" copy is needed.
template <int N>
__device__ __forceinline__ float row_bcast(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + N, 0xF, 0xF, true));
}

// ldl6_solve with the elimination spread over the lanes of each 16-lane row: lane r (< 6) holds
// row r of the lower triangle (its entries right of the diagonal are never read), and step j's
// pivot, its rhs and column j (a[c][j], c > j) reach every lane by row_newbcast.  The same
// operations on the same operands in the same order as ldl6_solve -- a[i][c] -= f_i a[c][j],
// f_i = a[i][j] / d_j, rhs_i -= f_i rhs_j, the back substitution from the column values each step
// broadcast -- so the result is bit-identical; 27 DPP moves replace 15 of the 35 trailing-update
// FMAs' serial issue and the 21 loads of the one-lane form.  Every lane of the wave must be
// active; every lane returns the same dx (each row solves the system).
template <bool GUARD>
__device__ __forceinline__ bool ldl6_solve_wave(const float* tw, float dx[6]) {
  const int r0 = (int)(__lane_id() & 15);
  const int r = r0 < 6 ? r0 : 5;  // lanes 6-15 shadow row 5 (never broadcast from)
  float col[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) col[c] = tw[tri_index(c, r)];
  float rhs = tw[PICP_P_B + r];
  float id[6], rj[6], lc[6][6];
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    float d, bj;
    switch (j) {  // DPP controls are immediates
      case 0: d = row_bcast<0>(col[0]); bj = row_bcast<0>(rhs); break;
      case 1: d = row_bcast<1>(col[1]); bj = row_bcast<1>(rhs); break;
      case 2: d = row_bcast<2>(col[2]); bj = row_bcast<2>(rhs); break;
      case 3: d = row_bcast<3>(col[3]); bj = row_bcast<3>(rhs); break;
      case 4: d = row_bcast<4>(col[4]); bj = row_bcast<4>(rhs); break;
      default: d = row_bcast<5>(col[5]); bj = row_bcast<5>(rhs); break;
    }
    float inv = __builtin_amdgcn_rcpf(d);
    if (GUARD) inv = (fabsf(d) > FLT_MIN) ? inv : 0.0f;
    else bad |= !(fabsf(d) > FLT_MIN);
    id[j] = inv;
    rj[j] = bj;
    const float f = col[j] * inv;
#pragma unroll
    for (int c = j + 1; c < 6; ++c) {
      float b;
      switch (c) {
        case 1: b = row_bcast<1>(col[j]); break;
        case 2: b = row_bcast<2>(col[j]); break;
        case 3: b = row_bcast<3>(col[j]); break;
        case 4: b = row_bcast<4>(col[j]); break;
        default: b = row_bcast<5>(col[j]); break;
      }
      lc[c][j] = b;  // a[c][j] after steps < j: the back substitution's U[j][c]
      col[c] = fmaf(-f, b, col[c]);
    }
    rhs = fmaf(-f, bj, rhs);
  }
#pragma unroll
  for (int k = 5; k >= 0; --k) {
    const float x = rj[k] * id[k];
    dx[k] = x;
#pragma unroll
    for (int i = 0; i < k; ++i) rj[i] = fmaf(-lc[k][i], x, rj[i]);
  }
  return bad;
}

__device__ __forceinline__ void ldl6_solve_wave(const float* tw, float dx[6]) {
  if (ldl6_solve_wave<false>(tw, dx)) ldl6_solve_wave<true>(tw, dx);
}

// sin/cos of GN increment angles.  Increments are small, so the float Taylor series (exact to
// float rounding for |a| <= 1/16: next term a^9/9! < 1e-16) avoids sincosf's range reduction
// on the critical path; ONE test for the three angles keeps the common case straight-line (three
// independent polynomial chains); larger angles take the libm path.
__device__ __forceinline__ void taylor_sincos(float a, float* s, float* c) {
  const float a2 = a * a;
  *s = a * fmaf(a2, fmaf(a2, fmaf(a2, -1.0f / 5040.0f, 1.0f / 120.0f), -1.0f / 6.0f), 1.0f);
  *c = fmaf(a2, fmaf(a2, fmaf(a2, fmaf(a2, 1.0f / 40320.0f, -1.0f / 720.0f), 1.0f / 24.0f), -0.5f), 1.0f);
}

// src/defs.h:100-136 v2tEuler's rotation: Rd = Rx(a)*Ry(b)*Rz(c) (float) of dx[3..5].
__device__ __forceinline__ void update_rotation(const float dx[6], float Rd[3][3]) {
  float sa, ca, sb, cb, sc, cc;
  if (fabsf(dx[3]) <= 0.0625f && fabsf(dx[4]) <= 0.0625f && fabsf(dx[5]) <= 0.0625f) {
    taylor_sincos(dx[3], &sa, &ca);
    taylor_sincos(dx[4], &sb, &cb);
    taylor_sincos(dx[5], &sc, &cc);
  } else {
    sincosf(dx[3], &sa, &ca);
    sincosf(dx[4], &sb, &cb);
    sincosf(dx[5], &sc, &cc);
  }
  // Rd = Rx(a)*Ry(b)*Rz(c) in closed form: the same products and sums as the 3x3 products
  // of src/defs.h:133 with their structural zeros and ones folded away (x*1 = x, x+0 = x).
  const float sasb = sa * sb, casb = ca * sb;
  Rd[0][0] = cb * cc;
  Rd[0][1] = -(cb * sc);
  Rd[0][2] = sb;
  Rd[1][0] = sasb * cc + ca * sc;
  Rd[1][1] = ca * cc - sasb * sc;
  Rd[1][2] = -(sa * cb);
  Rd[2][0] = sa * sc - casb * cc;
  Rd[2][1] = casb * sc + sa * cc;
  Rd[2][2] = ca * cb;
}

// src/defs.h:100-136 v2tEuler: R = Rx(a)*Ry(b)*Rz(c) (float), t = v[0:3]; then
// src/picp_solver.cpp:103 T <- v2tEuler(dx) * T.
__device__ __forceinline__ void apply_update(const float dx[6], float R[9], float t[3]) {
  // (round 4 pinned the contractions here with fp contract(off) for a fused append that is gone;
  // it cost C2/C3 1-2 % -- profiles/r05/ab_regress/ -- and parity does not depend on it)
  float Rd[3][3];
  update_rotation(dx, Rd);
  float Rn[9], tn[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float s = Rd[i][0] * R[j * 3 + 0];
      s = s + Rd[i][1] * R[j * 3 + 1];
      s = s + Rd[i][2] * R[j * 3 + 2];
      Rn[j * 3 + i] = s;
    }
    float s = Rd[i][0] * t[0];
    s = s + Rd[i][1] * t[1];
    s = s + Rd[i][2] * t[2];
    tn[i] = s + dx[i];
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = Rn[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = tn[i];
}

// The 32 block-partial totals (double) -> the float words finish_round_f consumes, one word per
// total so lane e of a wave can convert total e: H entries with the damping added on the
// diagonal (src/picp_solver.cpp:96), -b, chi_in, chi_out as float, n_in and n_proj as int bits.
__device__ __forceinline__ float total_word(const PicpArgs& A, int e, double t) {
  const bool diag = (e == 0) | (e == 6) | (e == 11) | (e == 15) | (e == 18) | (e == 20);
  // straight-line selects (lane e converts total e: branches would serialise the wave)
  const double h = t + (diag ? (double)A.damping : 0.0);
  const double d = (e < PICP_P_B) ? h : ((e < PICP_P_CHI_IN) ? -t : t);
  const float f = (float)d;
  const float c = __int_as_float((int32_t)t);
  return (e < PICP_P_N_IN) ? f : ((e < 31) ? c : 0.0f);
}

// What a round leaves besides the pose: the state fields no later round reads.
struct RoundOut {
  float chi_in, chi_out;
  int32_t n_in, n_proj, ok, done, converged;
};

// Finish round j of a problem from its converted totals (total_word: damping already in): the
// min-inlier check, the 6x6 solve, the update and the icp_test loop rule.  The loop state a round
// reads -- the pose R (column-major) / t and chi_prev -- is carried in registers by the finishing
// wave (every lane computes the same values; no LDS state round trip on the critical path).
// tw may be LDS.
// WAVE: the caller is a whole wave with every lane active (the block and persistent kernels'
// finishing wave): the elimination runs over each 16-lane row (ldl6_solve_wave, bit-identical).
template <bool WAVE = false>
__device__ __forceinline__ void finish_round_pose(const PicpArgs& A, const float* tw, int j, float R[9],
                                                  float t[3], float& chi_prev, RoundOut& o) {
  o.chi_in = tw[PICP_P_CHI_IN];
  o.chi_out = tw[PICP_P_CHI_OUT];
  o.n_in = __float_as_int(tw[PICP_P_N_IN]);
  o.n_proj = __float_as_int(tw[PICP_P_N_PROJ]);
  o.converged = 0;  // a converged loop is done: no round runs after it
  if (o.n_in < A.min_inliers) {  // src/picp_solver.cpp:97-100
    o.ok = 0;
    o.done = 1;
    return;
  }
  float dx[6];
  if constexpr (WAVE)
    ldl6_solve_wave(tw, dx);  // :96 (damping folded in by total_word), :102
  else
    ldl6_solve(tw, dx);
  apply_update(dx, R, t);  // :103
  o.ok = 1;
  o.done = 0;
  // exec/icp_test.cpp:99-106
  const float prev = chi_prev, cur = o.chi_in;
  const float rel = (prev > 1e-10f) ? fabsf(prev - cur) / prev : 0.0f;
  if (rel < A.conv_eps) {
    o.converged = 1;
    o.done = 1;
  } else {
    chi_prev = cur;
  }
  if (j >= A.max_rounds) o.done = 1;
}

// The 128-byte state after round j, written field by field (padding zeroed): a whole-struct copy
// from a local goes through a scratch alloca (SROA cannot split the memcpy).  dst: LDS or global.
template <typename S>
__device__ __forceinline__ void store_state(S* dst, const float R[9], const float t[3], float chi_prev,
                                            const RoundOut& o, int j) {
#pragma unroll
  for (int i = 0; i < 9; ++i) dst->R[i] = R[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) dst->t[i] = t[i];
  dst->chi_prev = chi_prev;
  dst->chi_in = o.chi_in;
  dst->chi_out = o.chi_out;
  dst->n_in = o.n_in;
  dst->n_proj = o.n_proj;
  dst->rounds = j;
  dst->done = o.done;
  dst->ok = o.ok;
  dst->converged = o.converged;
#pragma unroll
  for (int i = 0; i < 11; ++i) dst->pad[i] = 0;
}

// finish_round_pose on a stored state (the multi-launch round kernel: one lane).
__device__ __forceinline__ void finish_round_f(const PicpArgs& A, const PicpState& s,
                                               const float* tw, int j, PicpState& ns) {
  float R[9], t[3];
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = s.R[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = s.t[i];
  float chi_prev = s.chi_prev;
  RoundOut o;
  finish_round_pose(A, tw, j, R, t, chi_prev, o);
  store_state(&ns, R, t, chi_prev, o, j);
}

// Finish round (j-1) of a problem from its block-partial totals (double): H, b, stats -> new
// state.  One lane.
__device__ __forceinline__ void finish_round(const PicpArgs& A, const PicpState& s,
                                             const double* tot, int j, PicpState& ns) {
  float tw[PICP_NPART];
#pragma unroll
  for (int e = 0; e < PICP_NPART; ++e) tw[e] = total_word(A, e, tot[e]);
  finish_round_f(A, s, tw, j, ns);
}


// Refined hardware reciprocal and reciprocal square root in double: the v_rcp_f64 / v_rsq_f64
// estimate and two Newton steps (full double precision), half the dependency chain of the IEEE
// division / sqrt sequences.
__device__ __forceinline__ double tri_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  return fma(r, fma(-x, r, 1.0), r);
}
__device__ __forceinline__ double tri_rsq(double x) {
  double y = __builtin_amdgcn_rsq(x);
  y = fma(0.5 * y, fma(-x * y, y, 1.0), y);
  return fma(0.5 * y, fma(-x * y, y, 1.0), y);
}

// Right singular vector of the smallest singular value of the 4x4 DLT system A, by one-sided
// (Hestenes) Jacobi, at most 10 sweeps, stopping after the first sweep that rotates nothing
// (every later sweep would be a no-op); all indices compile-time so A and V stay in registers.
// A is consumed.
__device__ __forceinline__ void tri_null_jacobi(double A[4][4], double v[4]) {
  double Vm[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) Vm[r][c] = (r == c) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 10; ++sweep) {
    bool rotated = false;  // a sweep that rotates nothing leaves A and V unchanged: stop there
#pragma unroll
    for (int pq = 0; pq < 6; ++pq) {
      const int p = (pq < 3) ? 0 : ((pq < 5) ? 1 : 2);
      const int qq = (pq < 3) ? pq + 1 : ((pq < 5) ? pq - 1 : 3);
      double alpha = 0.0, beta = 0.0, gamma = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        alpha += A[k][p] * A[k][p];
        beta += A[k][qq] * A[k][qq];
        gamma += A[k][p] * A[k][qq];
      }
      // Rotate unless the pair is orthogonal to 1e-12 relative (gamma^2 <= 1e-24 alpha beta): the
      // smaller rotations move the result below float precision.
      if (fabs(gamma) > 1e-300 && gamma * gamma > 1e-24 * (alpha * beta)) {
        rotated = true;
        const double zeta = (beta - alpha) * tri_rcp(2.0 * gamma);
        const double q = fma(zeta, zeta, 1.0);
        const double t = ((zeta >= 0.0) ? 1.0 : -1.0) * tri_rcp(fabs(zeta) + q * tri_rsq(q));  // 1/(|z| + sqrt(1+z^2))
        const double c = tri_rsq(fma(t, t, 1.0));
        const double s = c * t;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const double akp = A[k][p], akq = A[k][qq];
          A[k][p] = c * akp - s * akq;
          A[k][qq] = s * akp + c * akq;
          const double vkp = Vm[k][p], vkq = Vm[k][qq];
          Vm[k][p] = c * vkp - s * vkq;
          Vm[k][qq] = s * vkp + c * vkq;
        }
      }
    }
    if (!rotated) break;  // identical result to running all 10 sweeps
  }
  double nrm[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) nrm[c] = A[0][c] * A[0][c] + A[1][c] * A[1][c] + A[2][c] * A[2][c] + A[3][c] * A[3][c];
  double best = nrm[0];
  v[0] = Vm[0][0]; v[1] = Vm[1][0]; v[2] = Vm[2][0]; v[3] = Vm[3][0];
#pragma unroll
  for (int c = 1; c < 4; ++c) {
    const bool take = nrm[c] < best;
    best = take ? nrm[c] : best;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = take ? Vm[r][c] : v[r];
  }
}

// Two-view linear (DLT) triangulation of one point, cv::triangulatePoints as called from
// src/cam.cpp:115 then convertPointsFromHomogeneous :118.  P1, P2: 3x4 ROW-major float.
// A (4x4) in double; X_h = the right singular vector of A's smallest singular value, by the
// one-sided Jacobi above (tri_null_jacobi).
// -DPICP_TRI_INVIT (A/B, measured slower, not the default): the eigenvector of the smallest
// eigenvalue of M = A^T A by inverse iteration on M through its
// LDL^T (no pivoting: M is positive semi-definite and, for a finite point, its null direction has
// w != 0, so the near-zero pivot is the last): x1 = M^-1 e4 (back substitution alone), then
// x2 = M^-1 x1.  x2 is accepted when it moved less than ~1.4e-6 rad from x1 (1 - |cos| < 1e-12):
// the error left after the second step is then below ~1e-12, the SVD's own rounding level.  A
// point whose system is not that well separated (near-parallel rays, a point at infinity, a
// degenerate ray pair, |w| <= 1e-5) takes the Jacobi SVD.  On the VO sequence's pairs (sigma4 / sigma3 ~1e-7)
// every point takes the fast path, within 2.1e-11 of numpy's SVD.  Parity green (the long-segment
// rule included), but the append got slower, not faster: C5 805k -> 777k frames/s, the N = 8
// per-rank shape 161.4k -> 159.2k, 8e 42.7k -> 42.0k (profiles/r06/t1/ab_tri.log).
__device__ inline void triangulate_dlt(const float* P1, const float* P2, float2 a, float2 b,
                                       float out[3]) {
  double A[4][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    A[0][k] = (double)a.x * (double)P1[8 + k] - (double)P1[0 + k];
    A[1][k] = (double)a.y * (double)P1[8 + k] - (double)P1[4 + k];
    A[2][k] = (double)b.x * (double)P2[8 + k] - (double)P2[0 + k];
    A[3][k] = (double)b.y * (double)P2[8 + k] - (double)P2[4 + k];
  }
  double v[4];
#ifndef PICP_TRI_INVIT
  tri_null_jacobi(A, v);
#else
  {
    double M[4][4];  // upper triangle used
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = i; j < 4; ++j) M[i][j] = A[0][i] * A[0][j] + A[1][i] * A[1][j] + A[2][i] * A[2][j] + A[3][i] * A[3][j];
    const double r0 = tri_rcp(M[0][0]);
    const double l10 = M[0][1] * r0, l20 = M[0][2] * r0, l30 = M[0][3] * r0;
    const double d1 = M[1][1] - l10 * M[0][1];
    const double r1 = tri_rcp(d1);
    const double l21 = (M[1][2] - l20 * M[0][1]) * r1, l31 = (M[1][3] - l30 * M[0][1]) * r1;
    const double d2 = M[2][2] - l20 * M[0][2] - l21 * l21 * d1;
    const double r2 = tri_rcp(d2);
    const double l32 = (M[2][3] - l30 * M[0][2] - l31 * l21 * d1) * r2;
    double d3 = M[3][3] - l30 * M[0][3] - l31 * l31 * d1 - l32 * l32 * d2;
    d3 = (fabs(d3) > 1e-300) ? d3 : 1e-300;  // an exactly singular M: any tiny pivot gives its null vector
    const double r3 = tri_rcp(d3);
    // x1 = M^-1 e4 = L^-T (e4 / d3), normalised
    double x3 = r3, x2 = -l32 * x3, x1 = -l21 * x2 - l31 * x3, x0 = -l10 * x1 - l20 * x2 - l30 * x3;
    double s = tri_rsq(x0 * x0 + x1 * x1 + x2 * x2 + x3 * x3);
    x0 *= s; x1 *= s; x2 *= s; x3 *= s;
    // x2' = M^-1 x1: forward L y = x1, then L^T x = y / d
    const double y0 = x0, y1 = x1 - l10 * y0, y2 = x2 - l20 * y0 - l21 * y1,
                 y3 = x3 - l30 * y0 - l31 * y1 - l32 * y2;
    const double z3 = y3 * r3, z2 = y2 * r2 - l32 * z3, z1 = y1 * r1 - l21 * z2 - l31 * z3,
                 z0 = y0 * r0 - l10 * z1 - l20 * z2 - l30 * z3;
    s = tri_rsq(z0 * z0 + z1 * z1 + z2 * z2 + z3 * z3);
    v[0] = z0 * s; v[1] = z1 * s; v[2] = z2 * s; v[3] = z3 * s;
    const double c = fabs(v[0] * x0 + v[1] * x1 + v[2] * x2 + v[3] * x3);
    // (|w| well above FLT_EPSILON: the dehomogenisation below is then sign-independent)
    const bool ok = (c > 1.0 - 1e-12) && (c <= 1.0 + 1e-12) && (d1 > 0.0) && (d2 > 0.0) && (M[0][0] > 0.0) &&
                    (fabs(v[3]) > 1e-5);
    if (!ok) tri_null_jacobi(A, v);  // rare: the fallback runs with the lanes that need it
  }
#endif
  // points4D is float; convertPointsFromHomogeneous in float, scale 1 when |w| <= FLT_EPSILON
  const float X4 = (float)v[0], Y4 = (float)v[1], Z4 = (float)v[2], W4 = (float)v[3];
  const float scale = (fabsf(W4) > FLT_EPSILON) ? 1.0f / W4 : 1.0f;
  out[0] = X4 * scale;
  out[1] = Y4 * scale;
  out[2] = Z4 * scale;
}

}  // namespace picp
