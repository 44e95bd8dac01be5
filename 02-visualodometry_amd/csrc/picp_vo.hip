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
#include "picp_vo_device.h"

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
// points overlap.  Its compaction covers 4096 / VOA_BLOCK chunks of VOA_BLOCK (4096 observations).
#ifndef VOA_BLOCK
#define VOA_BLOCK 512  // 2 waves per SIMD (152 VGPRs); 1024 spills (profiles/r01/vo_append_ab.log)
#endif

__global__ __launch_bounds__(VO_BLOCK) void vo_gather_kernel(const VoArgs a, int t) {
  const int s = a.seg0 + (int)blockIdx.x;
  const VoSegment G = a.segs[s];
  const int64_t base = (int64_t)s * a.cap_c;
  __shared__ int s_cnt[VO_WAVES];
  if (t >= G.steps) {  // segment finished: an empty problem (its result is never read)
    if (threadIdx.x == 0) a.probs[s] = PicpProblem{base, 0, 0, 1, 0};
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
}

__global__ __launch_bounds__(VOA_BLOCK) void vo_append_kernel(const VoArgs a, int t) {
  const int s = a.seg0 + (int)blockIdx.x;
  vo_append_body<VOA_BLOCK>(a, t, s, a.st_out + s, (t < 0) ? 0 : a.probs[s].n);
}

extern "C" hipError_t picp_launch_vo_gather(hipStream_t stream, const VoArgs* a, int t) {
  if (!a || a->n_seg <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(vo_gather_kernel, dim3(a->n_seg), dim3(VO_BLOCK), 0, stream, *a, t);
  return hipGetLastError();
}

#ifdef VOA_TSTAMP
extern "C" hipError_t picp_debug_voa_tstamp(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(picp_voa_tstamp), sizeof(picp_voa_tstamp), 0,
                                     hipMemcpyDeviceToHost);
  if (e == hipSuccess && reset) {
    const unsigned long long z[5] = {0, 0, 0, 0, 0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(picp_voa_tstamp), z, sizeof(z), 0, hipMemcpyHostToDevice);
  }
  return e;
}
#endif

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
