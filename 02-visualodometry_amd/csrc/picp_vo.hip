// picp_vo.hip -- the device-resident VO step around PICP (C5).
//
// The reference runs exec/icp_test.cpp:61-136 frame by frame on the host:
//   corr   = match_points(next, map)                         (:72-73)
//   pose   = PICP from the previous pose                      (:76-113)
//   pairs  = match_points(curr, next)                         (:117-119)
//   new    = add_new_world_points(corr, pairs)                (src/my_utilities.cpp:413-434)
//   map   += triangulatePoints(prev pose, pose, new)          (src/cam.cpp:94-140)
// Here every frame of a segment is one STEP and all segments of a sequence advance together:
// one step = 3 launches over all segments (world match, picp_block_kernel with the gather fused
// in -- picp_block.hip vo_gather_items; 4 with PICP_VO_FUSE=0 -- and append),
// with every count (map size, correspondences, new points) living in device memory, so a
// whole sequence is enqueued (and hipGraph-captured) without a single host round trip.
//
//   vo_gather_kernel  : one block per segment compacts the accepted next->map matches, in
//                       observation order (the IntPairVector order), into the PICP SoA planes
//                       and writes the segment's PicpProblem.
//   vo_append_kernel  : one block per segment records the PICP result (pose, stats), selects
//                       the curr->next pairs whose next point has no map match, triangulates
//                       them with (previous pose, new pose) in pair order and appends
//                       (xyz, curr descriptor) to the segment's map; then writes the next step's
//                       world-match problem and the PICP initial state.  With t < 0 it is the
//                       bootstrap (exec/icp_test.cpp:40-58 with the pose pair given).
// Ordered compaction = wave ballot + popcount prefix + an LDS scan over the block's waves, so
// map order and correspondence order equal the reference's sequential push_back order.
#include "picp_device.h"

using namespace picp;

#define VO_BLOCK 256
#define VO_WAVES (VO_BLOCK / 64)
// chunks of VO_BLOCK observations whose global loads are all issued before the first ordered
// compaction step (frames of <= 4096 observations; a larger frame's tail runs the plain loop).
// One-block-per-segment kernels are latency-bound: loading chunk by chunk between the scan's
// barriers serialised two dependent global round trips per chunk.
#define VO_PF 16
// The append kernel triangulates with every lane of its block (FP64 Jacobi per new point): a
// wider block puts four waves on each SIMD instead of one, so the FP64 chains of different
// points overlap.  Its compaction covers VOA_PF chunks of VOA_BLOCK (4096 observations).
#ifndef VOA_BLOCK
#define VOA_BLOCK 512  // 2 waves per SIMD (152 VGPRs); 1024 spills (profiles/r01/vo_append_ab.log)
#endif
#define VOA_WAVES (VOA_BLOCK / 64)
#define VOA_PF (4096 / VOA_BLOCK)

// Eigen::Isometry3f::inverse() of a column-major 4x4 (oracle/picp_oracle.c or_iso_inverse order)
__device__ inline void vo_iso_inverse(const float* T, float* Ti) {
#pragma clang fp contract(off)
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) Ti[j * 4 + i] = T[i * 4 + j];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    float s = Ti[0 * 4 + i] * T[12 + 0];
    s = s + Ti[1 * 4 + i] * T[12 + 1];
    s = s + Ti[2 * 4 + i] * T[12 + 2];
    Ti[12 + i] = -s;
  }
  Ti[3] = Ti[7] = Ti[11] = 0.0f;
  Ti[15] = 1.0f;
}

// P = K * inverse(T_cw)(0:3, 0:4), row-major 3x4 (src/cam.cpp:109-112)
__device__ inline void vo_projection(const float* K, const float* Tcw, float* P) {
#pragma clang fp contract(off)
  float Ti[16];
  vo_iso_inverse(Tcw, Ti);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s = K[0 * 3 + i] * Ti[j * 4 + 0];
      s = s + K[1 * 3 + i] * Ti[j * 4 + 1];
      s = s + K[2 * 3 + i] * Ti[j * 4 + 2];
      P[i * 4 + j] = s;
    }
}

// ordered block compaction: returns this lane's rank among the flagged lanes of the chunk;
// *total = flagged lanes in the chunk.  Contains two barriers (all lanes must call).
template <int NW>
__device__ inline int vo_block_rank(bool flag, int* s_cnt, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long m = __ballot(flag);
  const int r = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) s_cnt[w] = __popcll(m);
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    pre += (k < w) ? s_cnt[k] : 0;
    tot += s_cnt[k];
  }
  __syncthreads();  // s_cnt is reused by the next chunk
  *total = tot;
  return pre + r;
}

__global__ __launch_bounds__(VO_BLOCK) void vo_gather_kernel(const VoArgs a, int t) {
  PICP_KFENCE_IN();
  const int s = a.seg0 + (int)blockIdx.x;
  const VoSegment G = a.segs[s];
  const int64_t base = (int64_t)s * a.cap_c;
  __shared__ int s_cnt[VO_WAVES];
  if (t >= G.steps) {  // segment finished: an empty problem (its result is never read)
    if (threadIdx.x == 0) a.probs[s] = PicpProblem{base, 0, 0, 1, 0};
    PICP_KFENCE_OUT();
    return;
  }
  const int64_t nf = G.f0 + t + 1;
  const int64_t on = a.frame_off[nf], nn = a.frame_off[nf + 1] - on;
  const int64_t moff = G.map_off;
  int64_t cnt = 0;
  // every chunk's loads first (accept flag, map index, pixel; then the map point), ...
  bool fl[VO_PF];
  float px[VO_PF], py[VO_PF], pz[VO_PF];
  float2 pu[VO_PF];
  int jb[VO_PF];
#pragma unroll
  for (int c = 0; c < VO_PF; ++c) {
    const int64_t i = (int64_t)c * VO_BLOCK + threadIdx.x;
    fl[c] = i < nn && a.wm_acc[on + i] != 0;
    jb[c] = (i < nn) ? a.wm_bi[on + i] : 0;
    pu[c] = (i < nn) ? a.uv[on + i] : make_float2(0.0f, 0.0f);
  }
#pragma unroll
  for (int c = 0; c < VO_PF; ++c) {
    const int64_t j = moff + (fl[c] ? jb[c] : 0);
    px[c] = fl[c] ? a.map_xyz[3 * j + 0] : 0.0f;
    py[c] = fl[c] ? a.map_xyz[3 * j + 1] : 0.0f;
    pz[c] = fl[c] ? a.map_xyz[3 * j + 2] : 0.0f;
  }
  // ... then the ordered compaction, chunk by chunk, from registers
#pragma unroll
  for (int c = 0; c < VO_PF; ++c) {
    if ((int64_t)c * VO_BLOCK >= nn) break;  // uniform
    int tot;
    const int r = vo_block_rank<VO_WAVES>(fl[c], s_cnt, &tot);
    if (fl[c]) {
      const int64_t o = base + cnt + r;
      a.X[o] = px[c];
      a.Y[o] = py[c];
      a.Z[o] = pz[c];
      a.U[o] = pu[c].x;
      a.V[o] = pu[c].y;
    }
    cnt += tot;
  }
  for (int64_t c0 = (int64_t)VO_PF * VO_BLOCK; c0 < nn; c0 += VO_BLOCK) {  // frames > 4096 obs
    const int64_t i = c0 + threadIdx.x;
    const bool flag = i < nn && a.wm_acc[on + i] != 0;
    int tot;
    const int r = vo_block_rank<VO_WAVES>(flag, s_cnt, &tot);
    if (flag) {
      const int64_t j = moff + a.wm_bi[on + i];
      const int64_t o = base + cnt + r;
      const float2 z = a.uv[on + i];
      a.X[o] = a.map_xyz[3 * j + 0];
      a.Y[o] = a.map_xyz[3 * j + 1];
      a.Z[o] = a.map_xyz[3 * j + 2];
      a.U[o] = z.x;
      a.V[o] = z.y;
    }
    cnt += tot;
  }
  if (threadIdx.x == 0) a.probs[s] = PicpProblem{base, (int32_t)cnt, 0, 1, 0};
  PICP_KFENCE_OUT();
}

__global__ __launch_bounds__(VOA_BLOCK) void vo_append_kernel(const VoArgs a, int t) {
  PICP_KFENCE_IN();
  const int s = a.seg0 + (int)blockIdx.x;
  const VoSegment G = a.segs[s];
  const bool boot = t < 0;
  if (!boot && t >= G.steps) return;
  __shared__ float sP[24];
  __shared__ float sTn[16];
  __shared__ int64_t s_base;
  __shared__ int s_cnt[VOA_WAVES];
  const int64_t cf = G.f0 + (boot ? 0 : t), nf = cf + 1;
  const int64_t oc = a.frame_off[cf], nc = a.frame_off[cf + 1] - oc;
  const int64_t on = a.frame_off[nf];
  const int64_t rec = G.slot0 + (boot ? 0 : t + 1);
  if (threadIdx.x == 0) {
    float Tp[16], Te[16];
    if (boot) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        Tp[k] = a.boot[32 * s + k];
        Te[k] = a.boot[32 * s + 16 + k];
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) a.poses[16 * G.slot0 + k] = Tp[k];  // poses = {T0}
      s_base = 0;
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) Tp[k] = a.poses[16 * (G.slot0 + t) + k];
      const PicpState st = a.st_out[s];
      float Twc[16];
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i) Twc[j * 4 + i] = st.R[j * 3 + i];
#pragma unroll
      for (int i = 0; i < 3; ++i) Twc[12 + i] = st.t[i];
      Twc[3] = Twc[7] = Twc[11] = 0.0f;
      Twc[15] = 1.0f;
      vo_iso_inverse(Twc, Te);  // estimated_pose = worldInCameraPose().inverse() (:113)
#pragma unroll
      for (int k = 0; k < 16; ++k) a.poses[16 * rec + k] = Te[k];
      VoStep r;
      r.n_corr = a.probs[s].n;
      r.n_in = st.n_in;
      r.rounds = st.rounds;
      r.n_new = 0;
      r.chi_in = st.chi_in;
      r.chi_out = st.chi_out;
      r.converged = st.converged;
      r.n_proj = st.n_proj;
      a.steps[rec] = r;
      s_base = a.map_n[s];
    }
    float Kl[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) Kl[k] = a.K[k];
    vo_projection(Kl, Tp, sP);
    vo_projection(Kl, Te, sP + 12);
    // the next PICP starts from poses.back() (:77-78): T0 after the bootstrap, else Te
#pragma unroll
    for (int k = 0; k < 16; ++k) sTn[k] = boot ? Tp[k] : Te[k];
  }
  __syncthreads();
  const int64_t mbase = G.map_off + s_base;
  const int dim = a.dim;
  int2* pairs = a.pairs + (int64_t)s * a.cap_c;
  // pass 1: the selected (curr, next) pairs in pair order (add_new_world_points)
  int64_t cnt = 0;
  // every chunk's loads first (accept flag and next index, then the next point's map match), ...
  bool fl[VOA_PF];
  int jb[VOA_PF];
#pragma unroll
  for (int c = 0; c < VOA_PF; ++c) {
    const int64_t i = (int64_t)c * VOA_BLOCK + threadIdx.x;
    fl[c] = i < nc && a.pm_acc[oc + i] != 0;
    jb[c] = (i < nc) ? a.pm_bi[oc + i] : 0;
  }
#pragma unroll
  for (int c = 0; c < VOA_PF; ++c)  // next point not among the map correspondences
    fl[c] = fl[c] && (boot || a.wm_acc[on + (fl[c] ? jb[c] : 0)] == 0);
  // ... then the ordered compaction from registers
#pragma unroll
  for (int c = 0; c < VOA_PF; ++c) {
    if ((int64_t)c * VOA_BLOCK >= nc) break;  // uniform
    int tot;
    const int r = vo_block_rank<VOA_WAVES>(fl[c], s_cnt, &tot);
    if (fl[c]) pairs[cnt + r] = make_int2(c * VOA_BLOCK + (int)threadIdx.x, jb[c]);
    cnt += tot;
  }
  for (int64_t c0 = (int64_t)VOA_PF * VOA_BLOCK; c0 < nc; c0 += VOA_BLOCK) {  // frames > 4096 obs
    const int64_t i = c0 + threadIdx.x;
    bool flag = false;
    int j = 0;
    if (i < nc && a.pm_acc[oc + i]) {
      j = a.pm_bi[oc + i];
      flag = boot || a.wm_acc[on + j] == 0;
    }
    int tot;
    const int r = vo_block_rank<VOA_WAVES>(flag, s_cnt, &tot);
    if (flag) pairs[cnt + r] = make_int2((int)i, j);
    cnt += tot;
  }
  __syncthreads();
  // pass 2: every lane triangulates (src/cam.cpp:115-139) and appends (xyz, curr descriptor)
  for (int64_t k = threadIdx.x; k < cnt; k += VOA_BLOCK) {
    const int2 pr = pairs[k];
    const int64_t slot = mbase + k;
    float o[3];
#ifdef VOA_DIAG_NOTRI  // diagnostic build only (wrong map points): no FP64 triangulation
    {
      const float2 ua = a.uv[oc + pr.x], ub = a.uv[on + pr.y];
      o[0] = ua.x * sP[0] + ub.x;
      o[1] = ua.y * sP[5] + ub.y;
      o[2] = 1.0f + sP[10];
    }
#else
    triangulate_dlt(sP, sP + 12, a.uv[oc + pr.x], a.uv[on + pr.y], o);
#endif
    // the descriptor row and the matcher's prepped row of it (fp16 + guard norms): every load
    // first, then the stores -- the compiler cannot rule out that a store aliases a later load,
    // so an interleaved element copy paid one global round trip per element
    const int64_t src = oc + pr.x;
    float dv[32];  // dim <= 32 (picp_vo_create)
#pragma unroll
    for (int d = 0; d < 32; ++d) dv[d] = (d < dim) ? a.desc[src * dim + d] : 0.0f;
    uint4 hv[4];  // dp = 16 or 32 halves: dp / 8 chunks of 16 B (rows 32-B aligned)
    const uint4* hs = reinterpret_cast<const uint4*>(a.obs_h + src * a.dp);
#pragma unroll
    for (int c = 0; c < 4; ++c) hv[c] = (c < a.dp / 8) ? hs[c] : make_uint4(0u, 0u, 0u, 0u);
    const float n1 = a.obs_n1[src], n2 = a.obs_n2[src];
    a.map_xyz[3 * slot + 0] = o[0];
    a.map_xyz[3 * slot + 1] = o[1];
    a.map_xyz[3 * slot + 2] = o[2];
#pragma unroll
    for (int d = 0; d < 32; ++d)
      if (d < dim) a.map_desc[slot * dim + d] = dv[d];
    uint4* hd = reinterpret_cast<uint4*>(a.map_h + slot * a.dp);
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < a.dp / 8) hd[c] = hv[c];
    a.map_n1[slot] = n1;
    a.map_n2[slot] = n2;
  }
  if (threadIdx.x == 0) {
    const int64_t mn = s_base + cnt;
    a.map_n[s] = mn;
    if (boot) {
      VoStep r = {};
      r.n_new = (int32_t)cnt;
      a.steps[rec] = r;
    } else {
      a.steps[rec].n_new = (int32_t)cnt;
    }
    const int tn = boot ? 0 : t + 1;
    MatchProblem wp{0, 0, G.map_off, mn};
    if (tn < G.steps) {
      const int64_t f = G.f0 + tn + 1;
      wp.q_off = a.frame_off[f];
      wp.nq = a.frame_off[f + 1] - wp.q_off;
    }
    a.wprobs[s] = wp;
    // PICP initial state: world-in-camera = previous_pose.inverse() (:78)
    float Twc[16];
    vo_iso_inverse(sTn, Twc);
    PicpState st = {};
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int i = 0; i < 3; ++i) st.R[j * 3 + i] = Twc[j * 4 + i];
#pragma unroll
    for (int i = 0; i < 3; ++i) st.t[i] = Twc[12 + i];
    a.st_in[s] = st;
  }
  PICP_KFENCE_OUT();
}

extern "C" hipError_t picp_launch_vo_gather(hipStream_t stream, const VoArgs* a, int t) {
  if (!a || a->n_seg <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(vo_gather_kernel, dim3(a->n_seg), dim3(VO_BLOCK), 0, stream, *a, t);
  return hipGetLastError();
}

extern "C" hipError_t picp_launch_vo_append(hipStream_t stream, const VoArgs* a, int t) {
  if (!a || a->n_seg <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(vo_append_kernel, dim3(a->n_seg), dim3(VOA_BLOCK), 0, stream, *a, t);
  return hipGetLastError();
}

// 1 when this library's device code was built with packed FP32 (make PK=1, A/B builds only): the
// VO runtime then defaults to the serial schedule
extern "C" int picp_build_packed_fp32(void) {
#ifdef PICP_ALLOW_PK
  return 1;
#else
  return 0;
#endif
}
