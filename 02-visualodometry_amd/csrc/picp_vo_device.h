// picp_vo_device.h -- device pieces of the VO step shared by the VO kernels (picp_vo.hip) and the
// PICP block kernel's fused VO gather (picp_block.hip): pose algebra, the ordered block
// compaction and the append (exec/icp_test.cpp:113-132, src/my_utilities.cpp:413-434, src/cam.cpp:94-140).
#pragma once
#include "picp_device.h"

namespace picp {

// Diagnostic build only (-DVOA_TSTAMP): s_memrealtime phase sums of the append (thread 0 of every
// block, steps t >= 0; 100 MHz ticks): [0] record + projections, [1] pass 1 (flags, compaction),
// [2] pass 2 (triangulate, append; every lane), [3] the next problem and state, [4] blocks
// (tools/r06/append_tstamp.py).
#ifdef VOA_TSTAMP
__device__ unsigned long long picp_voa_tstamp[5];
#define VOA_TS(v) v = __builtin_amdgcn_s_memrealtime()
#else
#define VOA_TS(v) (void)0
#endif

// Eigen::Isometry3f::inverse() of a column-major 4x4 (oracle/picp_oracle.c or_iso_inverse order)
__device__ __forceinline__ void vo_iso_inverse(const float* T, float* Ti) {
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
__device__ __forceinline__ void vo_projection(const float* K, const float* Tcw, float* P) {
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
__device__ __forceinline__ int vo_block_rank(bool flag, int* s_cnt, int* total) {
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


// The append of step t (t < 0: the bootstrap) for segment s by a whole block of NT threads:
// record the PICP result, select the curr->next pairs whose next point has no map match (pass 1,
// pair order), triangulate them with (previous pose, new pose) and append (xyz, curr descriptor)
// to the map (pass 2), then write the next step's world-match problem and PICP initial state.
// st_res: the PICP result (a.st_out[s]); n_corr: the PICP input size (a.probs[s].n).  Contains barriers: every thread calls.
template <int NT>
__device__ __forceinline__ void vo_append_body(const VoArgs& a, int t, int s, const PicpState* st_res, int n_corr) {
  constexpr int NW = NT / 64;
  constexpr int PF = 4096 / NT;
  const VoSegment G = a.segs[s];
  const bool boot = t < 0;
  if (!boot && t >= G.steps) return;  // uniform
  __shared__ float sP[24];
  __shared__ float sTn[16];
  __shared__ int64_t s_base;
  __shared__ int s_cnt[NW];
  const int64_t cf = G.f0 + (boot ? 0 : t), nf = cf + 1;
  const int64_t oc = a.frame_off[cf], nc = a.frame_off[cf + 1] - oc;
  const int64_t on = a.frame_off[nf];
  const int64_t rec = G.slot0 + (boot ? 0 : t + 1);
#ifdef VOA_TSTAMP
  unsigned long long vt0 = 0, vt1 = 0, vt2 = 0, vt3 = 0, vt4 = 0;
#endif
  VOA_TS(vt0);
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
      const PicpState st = *st_res;
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
      r.n_corr = n_corr;
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
  VOA_TS(vt1);
  const int64_t mbase = G.map_off + s_base;
  const int dim = a.dim;
  int2* pairs = a.pairs + (int64_t)s * a.cap_c;
  // pass 1: the selected (curr, next) pairs in pair order (add_new_world_points)
  int64_t cnt = 0;
  // every chunk's loads first (accept flag and next index, then the next point's map match), ...
  bool fl[PF];
  int jb[PF];
#pragma unroll
  for (int c = 0; c < PF; ++c) {
    const int64_t i = (int64_t)c * NT + threadIdx.x;
    fl[c] = i < nc && a.pm_acc[oc + i] != 0;
    jb[c] = (i < nc) ? a.pm_bi[oc + i] : 0;
  }
#pragma unroll
  for (int c = 0; c < PF; ++c)  // next point not among the map correspondences
    fl[c] = fl[c] && (boot || a.wm_acc[on + (fl[c] ? jb[c] : 0)] == 0);
  // ... then the ordered compaction of every chunk with ONE barrier (vo_gather_items' form): per
  // (chunk, wave) counts, then each flagged pair's index = flagged before its chunk + before its
  // wave + its lane rank -- the order of the per-chunk compaction (two barriers per chunk) it replaces
  // (the same bits; C5 within +-0.5 % at every shape, profiles/r06/t29/ab.log)
  {
    __shared__ int s_wc[PF][NW];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int rk[PF];
#pragma unroll
    for (int c = 0; c < PF; ++c) {
      const unsigned long long m = __ballot(fl[c]);
      rk[c] = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) s_wc[c][w] = __popcll(m);
    }
    __syncthreads();
    int n = 0;
#pragma unroll
    for (int c = 0; c < PF; ++c) {
      int pre = 0, tot = 0;
#pragma unroll
      for (int k = 0; k < NW; ++k) {
        pre += (k < w) ? s_wc[c][k] : 0;
        tot += s_wc[c][k];
      }
      if (fl[c]) pairs[n + pre + rk[c]] = make_int2(c * NT + (int)threadIdx.x, jb[c]);
      n += tot;
    }
    cnt = n;
  }
  for (int64_t c0 = (int64_t)PF * NT; c0 < nc; c0 += NT) {  // frames > 4096 obs
    const int64_t i = c0 + threadIdx.x;
    bool flag = false;
    int j = 0;
    if (i < nc && a.pm_acc[oc + i]) {
      j = a.pm_bi[oc + i];
      flag = boot || a.wm_acc[on + j] == 0;
    }
    int tot;
    const int r = vo_block_rank<NW>(flag, s_cnt, &tot);
    if (flag) pairs[cnt + r] = make_int2((int)i, j);
    cnt += tot;
  }
  __syncthreads();
  VOA_TS(vt2);
  // pass 2: every lane triangulates (src/cam.cpp:115-139) and appends (xyz, curr descriptor)
  for (int64_t k = threadIdx.x; k < cnt; k += NT) {
    const int2 pr = pairs[k];
    const int64_t slot = mbase + k;
    float o[3];
    triangulate_dlt(sP, sP + 12, a.uv[oc + pr.x], a.uv[on + pr.y], o);
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
#ifdef VOA_TSTAMP
  __syncthreads();
#endif
  VOA_TS(vt3);
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
    if (a.split) {
      // the late part of step tn: frame f0+tn+1 against the points this append added (indices in
      // the whole map's numbering) ...
      a.lprobs[s] = MatchProblem{wp.q_off, wp.nq, G.map_off + s_base, cnt, s_base};
      // ... and the early part of step tn + 1: frame f0+tn+2 against the map as it is now
      const int te = tn + 1;
      MatchProblem ep{0, 0, G.map_off, mn, 0};
      if (te < G.steps) {
        const int64_t f = G.f0 + te + 1;
        ep.q_off = a.frame_off[f];
        ep.nq = a.frame_off[f + 1] - ep.q_off;
      }
      a.eprobs[(int64_t)(te & 1) * a.seg_all + s] = ep;
    }
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
#ifdef VOA_TSTAMP
    VOA_TS(vt4);
    if (!boot) {
      atomicAdd(&picp_voa_tstamp[0], vt1 - vt0);
      atomicAdd(&picp_voa_tstamp[1], vt2 - vt1);
      atomicAdd(&picp_voa_tstamp[2], vt3 - vt2);
      atomicAdd(&picp_voa_tstamp[3], vt4 - vt3);
      atomicAdd(&picp_voa_tstamp[4], 1ull);
    }
#endif
  }
}

}  // namespace picp
