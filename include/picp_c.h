/*
 * picp_c.h -- C-ABI of libpicp_amd.so, the MI355X (gfx950) PICP hot path.
 *
 * This is the drop-in boundary for the reference's pr::PICPSolver / pr::Camera
 * (llepa/02-VisualOdometry; paths below are relative to the reference repo root).  Plain
 * pointers and sizes only; no C++ or framework types.  Every call returns an int status
 * (PICP_OK == 0); nothing throws across the ABI.  picp_last_error() returns a
 * thread-local description of the last failure.
 *
 * Memory layouts (identical to the reference's Eigen types):
 *   pose  T_wc[16] : 4x4 float COLUMN-major (Eigen::Isometry3f), the world-in-camera pose
 *                    (pr::Camera::worldInCameraPose, src/camera.h:51).
 *   K[9]           : 3x3 float column-major (Eigen::Matrix3f, src/camera.h:45).
 *   world xyz      : float[3*n] packed (Vector3fVector, src/defs.h:22).
 *   image uv       : float[2*n] packed (Vector2fVector, src/defs.h:23).
 *   pairs          : int32[2*m] (first = image index, second = world index)
 *                    (IntPairVector, src/defs.h:209-211; src/picp_solver.cpp:65-66).
 *   P[12]          : 3x4 float ROW-major projection matrix (cv::Mat, src/cam.cpp:111-112).
 *
 * Threading: a handle is bound to one HIP device and owns one HIP stream; a handle must
 * not be used from two threads at once (the reference solver is single-threaded too).
 */
#ifndef PICP_C_H
#define PICP_C_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PICP_ABI_VERSION 3

/* status codes */
#define PICP_OK 0
#define PICP_ERR_ARG -1      /* null pointer / bad size / bad parameter           */
#define PICP_ERR_DEVICE -2   /* HIP runtime error (see picp_last_error)           */
#define PICP_ERR_RANGE -3    /* a correspondence index is out of range            */
#define PICP_ERR_STATE -4    /* call order violated (e.g. round before set_points)*/
#define PICP_ERR_NOMEM -5    /* device allocation failed                          */
#define PICP_TOO_FEW_INLIERS 1 /* oneRound returned false: n_in < min_inliers
                                  (src/picp_solver.cpp:97-100); pose not updated   */

typedef struct picp_handle picp_t;
typedef struct picp_batch picp_batch_t;

/* Solver statistics, the reference's accessors plus the icp_test loop outcome. */
typedef struct picp_stats {
  float chi_in;       /* PICPSolver::chiInliers  (src/picp_solver.h:47)  */
  float chi_out;      /* PICPSolver::chiOutliers (src/picp_solver.h:50)  */
  int32_t n_in;       /* PICPSolver::numInliers  (src/picp_solver.h:53)  */
  int32_t ok;         /* return value of the last oneRound               */
  int32_t rounds;     /* oneRound calls executed                          */
  int32_t converged;  /* exec/icp_test.cpp:92 convergenceReached          */
  int32_t n_projected;/* correspondences that passed projectPoint         */
  int32_t reserved;
} picp_stats;

/* Solver parameters. picp_params_default() gives the reference's values. */
typedef struct picp_params {
  float threshold;      /* kernel threshold; PICPSolver ctor default 1000 (src/picp_solver.cpp:14),
                           icp_test uses 3000 (exec/icp_test.cpp:86)                          */
  float damping;        /* 1 (src/picp_solver.cpp:11)                                          */
  int32_t min_inliers;  /* 0 (src/picp_solver.cpp:12)                                          */
  int32_t keep_outliers;/* 0 in icp_test (exec/icp_test.cpp:95)                                */
  int32_t max_rounds;   /* 50 (exec/icp_test.cpp:88)                                           */
  float conv_eps;       /* 1e-5 relative chi_in change (exec/icp_test.cpp:91); < 0 disables   */
} picp_params;

void picp_params_default(picp_params* p);
int picp_abi_version(void);
const char* picp_last_error(void);
int picp_device_count(int* n);

/* ---------------- single-problem handle: the pr::PICPSolver drop-in ---------------- */

/* Replaces PICPSolver() + the Camera passed to init (src/picp_solver.cpp:8-15,17-20). */
int picp_create(picp_t** out, int device, int rows, int cols, const float K[9]);
int picp_destroy(picp_t* h);
int picp_set_camera(picp_t* h, int rows, int cols, const float K[9]);
/* Replaces PICPSolver's implicit copy constructor (src/picp_solver.h:21-82: every member is
 * copied, the world/image pointers included, so the copy keeps solving the same problem).  The
 * new handle is on the same device with its own copies of the points, the correspondences, the
 * camera and the pose. */
int picp_clone(const picp_t* src, picp_t** out);

/* Replaces PICPSolver::init's world/image arguments (src/picp_solver.cpp:17-23).  The
 * arrays are COPIED to device memory (the reference stores raw pointers; its icp_test
 * passes temporaries, exec/icp_test.cpp:81-85). */
int picp_set_points(picp_t* h, const float* world_xyz, int64_t n_world,
                    const float* image_uv, int64_t n_image);

/* Correspondences for the following rounds (the argument of PICPSolver::oneRound,
 * src/picp_solver.h:59).  Indices are range-checked (PICP_ERR_RANGE); an identical
 * repeated array is detected and not re-uploaded. */
int picp_set_correspondences(picp_t* h, const int32_t* pairs, int64_t m);

/* Camera::setWorldInCameraPose / worldInCameraPose (src/camera.h:51-52) */
int picp_set_pose(picp_t* h, const float T_wc[16]);
int picp_get_pose(picp_t* h, float T_wc[16]);

/* PICPSolver::oneRound (src/picp_solver.cpp:93-105): linearize + damping + min-inlier
 * check + LDLT solve + left update.  Returns PICP_OK, or PICP_TOO_FEW_INLIERS when the
 * reference returns false.  stats may be NULL. */
int picp_one_round(picp_t* h, float threshold, float damping, int min_inliers,
                   int keep_outliers, picp_stats* stats);

/* The whole exec/icp_test.cpp:88-107 loop fused on the device (one graph launch, no host
 * round trip per round). */
int picp_solve(picp_t* h, const picp_params* params, picp_stats* stats);

/* Linearize at the current pose without updating it (H 6x6 column-major, b 6), for
 * parity testing against PICPSolver::linearize (src/picp_solver.cpp:56-91). */
int picp_linearize(picp_t* h, float threshold, int keep_outliers, double H[36], double b[6],
                   picp_stats* stats);

/* ---------------- batched independent problems (frames) on one device ---------------- */

/* corr_offsets[n_problems+1]: problem i owns correspondences [off[i], off[i+1]) of the
 * arrays given to picp_batch_set_data.  Camera shared by all problems. */
int picp_batch_create(picp_batch_t** out, int device, int n_problems,
                      const int64_t* corr_offsets, int rows, int cols, const float K[9]);
int picp_batch_destroy(picp_batch_t* b);

/* Matched correspondences, already gathered: xyz[3*total] world points and uv[2*total]
 * image points (pairs (i,i)); copied to the device SoA planes. */
int picp_batch_set_data(picp_batch_t* b, const float* xyz, const float* uv);
/* Device-resident variant: the five SoA planes of length total, already on this device
 * (e.g. produced by a previous kernel); copied device-to-device. */
int picp_batch_set_data_device(picp_batch_t* b, const float* d_x, const float* d_y,
                               const float* d_z, const float* d_u, const float* d_v);

int picp_batch_set_poses(picp_batch_t* b, const float* T_wc /* 16*n_problems */);
int picp_batch_get_poses(picp_batch_t* b, float* T_wc /* 16*n_problems */);
int picp_batch_get_stats(picp_batch_t* b, picp_stats* stats /* n_problems */);

/* Fused icp_test loop for every problem; blocking. */
int picp_batch_solve(picp_batch_t* b, const picp_params* params);
/* Same, enqueued on the batch's stream (graph replay); pair with picp_batch_sync. */
int picp_batch_solve_async(picp_batch_t* b, const picp_params* params);
int picp_batch_sync(picp_batch_t* b);

/* Run `reps` back-to-back fused solves on the batch's stream between two HIP events and nothing
 * else.  total_ms = event time of the whole region; launch_us (nullable) = mean launch period
 * of the dominant kernel in it (total / (reps x launches per solve): max_rounds round launches in
 * graph mode, one launch otherwise).  Blocking; results readable with picp_batch_get_poses/stats
 * afterwards. */
int picp_batch_time(picp_batch_t* b, const picp_params* params, int reps, float* total_ms,
                    float* launch_us);
/* Diagnostic: one solve with an event pair around every launch (graph mode: the mean over its
 * round launches; otherwise the single launch), an upper bound that adds the event overhead. */
int picp_batch_time_single(picp_batch_t* b, const picp_params* params, float* us);
/* Introspection: total correspondences, blocks per launch, and the execution mode chosen for
 * the batch: 0 = one launch per GN round replayed from a hipGraph (any batch); 1 = the whole
 * loop in one persistent launch; 2 = one block (or a few cooperating blocks) per problem
 * (env PICP_MODE=graph|persistent|block forces one where the batch is eligible). */
int picp_batch_info(picp_batch_t* b, int64_t* total_corr, int* n_blocks, int* mode);
/* Co-residency of the layout's cross-block hand-off launch (persistent mode, or block mode with
 * two or four blocks per problem): grid = its blocks, resident = blocks the device holds at once
 * for that kernel (occupancy query x CUs; 0/0 when the layout considered none).  Such a launch is
 * used only when grid <= resident; if a hand-off wait still times out (CUs held by other work),
 * the solve is re-run without hand-offs and the batch keeps that layout: fallbacks counts it. */
int picp_batch_residency(picp_batch_t* b, int* grid, int* resident, int* fallbacks);

/* ---------------- batch split across GPUs: one process per GPU ---------------- */

/* The node's GPUs each run one process with its own picp_batch holding a contiguous shard of the
 * independent problems; the only collective is one RCCL all-gather (over xGMI) of the results.
 * The communicator wraps an RCCL communicator created from a 128-byte unique id that rank 0 makes
 * with picp_comm_unique_id and the launcher hands to every rank out of band.  librccl is loaded
 * on the first picp_comm_* call (dlopen), so single-GPU use never needs it. */
#define PICP_COMM_ID_BYTES 128
typedef struct picp_comm picp_comm_t;

/* Contiguous balanced split of n_items over world ranks: rank owns [*first, *last); sizes differ
 * by at most one (lower ranks take the remainder). */
int picp_shard_range(int64_t n_items, int world, int rank, int64_t* first, int64_t* last);
/* The layout picp_batch_allgather moves: every rank contributes its shard padded to
 * picp_shard_pad(n_items, world) = ceil(n_items / world) items, the all-gather concatenates them
 * in rank order, and picp_shard_unpack turns that padded buffer (world * pad items of item_bytes
 * each) back into the n_items items in problem order (rank r's items at picp_shard_range's
 * [first, last)).  Host memory, no device: the CPU tests drive it for ragged shards. */
int64_t picp_shard_pad(int64_t n_items, int world);
int picp_shard_unpack(int64_t n_items, int world, int64_t item_bytes, const void* padded, void* out);
int picp_comm_unique_id(uint8_t id[PICP_COMM_ID_BYTES]);
/* Collective over the world: blocks until every rank has joined. */
int picp_comm_create(picp_comm_t** out, int device, int world, int rank,
                     const uint8_t id[PICP_COMM_ID_BYTES]);
int picp_comm_destroy(picp_comm_t* c);
int picp_comm_info(picp_comm_t* c, int* device, int* world, int* rank);
/* Element-wise max over ranks of n (1..64) host doubles, in place (e.g. the timed region's wall
 * time); blocking. */
int picp_comm_allreduce_max(picp_comm_t* c, double* values, int n);
int picp_comm_barrier(picp_comm_t* c);
/* After a solve of this rank's batch (which must hold exactly picp_shard_range(n_total, world,
 * rank)'s problems): completes it, then all-gathers every rank's per-problem results so that
 * T_all[16 * n_total] (column-major camera poses, problem order) and st_all[n_total] (nullable)
 * hold all of them on every rank.  Collective: every rank calls it.  Every rank's local checks
 * (shard size, the solve's completion, the staging buffer) are agreed on by one max-allreduce
 * BEFORE the all-gather, so a rank that fails makes every rank return an error instead of
 * leaving the others blocked in the collective. */
int picp_batch_allgather(picp_batch_t* b, picp_comm_t* c, int64_t n_total, float* T_all,
                         picp_stats* st_all);
/* The same gather with the byte exchange supplied by the caller instead of RCCL, for launchers
 * whose ranks cannot form an RCCL communicator (several ranks on one GPU -- RCCL refuses a
 * duplicate device -- or a CPU process group) and for testing the split at any world size.
 * exchange(user, send, recv, bytes) must all-gather `bytes` from every rank's host buffer `send`
 * into `recv` (world * bytes, rank order) and return 0.  One exchange per call: each rank sends
 * a 16-byte header (its local status) and its shard's 128-byte states padded to
 * picp_shard_pad(n_total, world) -- the layout picp_batch_allgather moves -- so a rank whose local
 * checks failed makes every rank return an error after the one exchange.  A non-zero return of
 * exchange is returned as PICP_ERR_STATE. */
typedef int (*picp_exchange_fn)(void* user, const void* send, void* recv, size_t bytes);
int picp_batch_allgather_host(picp_batch_t* b, int world, int rank, picp_exchange_fn exchange, void* user,
                              int64_t n_total, float* T_all, picp_stats* st_all);

/* ---------------- linear triangulation (cv::triangulatePoints replacement) ---------------- */

/* src/cam.cpp:94-140: per point DLT with two 3x4 row-major projection matrices, then
 * dehomogenisation.  uv1/uv2: float[2*q]; xyz_out: float[3*q].  Host pointers. */
int picp_triangulate(int device, const float P1[12], const float P2[12], const float* uv1,
                     const float* uv2, int64_t q, float* xyz_out);
/* Helper: P = K * inverse(T_cw)(0:3,0:4) from a camera-in-world pose (src/cam.cpp:109-112). */
int picp_projection_matrix(const float K[9], const float T_cw[16], float P[12]);

/* ---------------- descriptor matching (match_points replacement) ---------------- */

/* src/my_utilities.h:70-120: for each of the n1 descriptors of set 1 (float[dim], packed) the
 * nearest set-2 descriptor by squared L2 (best_idx, -1 if set 2 is empty), its distance and the
 * second-nearest distance; accepted[i] = best < dist_thr && best/second < ratio_thr (the
 * reference uses 0.2 and 0.8, src/my_utilities.h:44-46).  The accepted (i, best_idx[i]) pairs
 * are the reference's IntPairVector.  dim in [1, 32].  Host pointers. */
int picp_match(int device, const float* desc1, int64_t n1, const float* desc2, int64_t n2, int dim,
               float dist_thr, float ratio_thr, int32_t* best_idx, float* best_dist,
               float* second_dist, int32_t* accepted);
/* Many independent (set 1, set 2) pairs in one launch: problem i matches desc1 rows
 * [off1[i], off1[i+1]) against desc2 rows [off2[i], off2[i+1]); best_idx is relative to
 * off2[i].  n_problems <= 65535. */
int picp_match_batch(int device, int n_problems, const int64_t* off1, const int64_t* off2,
                     const float* desc1, const float* desc2, int dim, float dist_thr,
                     float ratio_thr, int32_t* best_idx, float* best_dist, float* second_dist,
                     int32_t* accepted);
/* picp_match_batch in an explicit kernel form:
 *   PICP_MATCH_FORM_FULL        the default (MFMA pre-filter + exact rescan; every output);
 *   PICP_MATCH_FORM_ACCEPT_ONLY the radius form the VO sequence runs: only accepted[] and
 *                               best_idx of accepted queries are defined (the others are not);
 *   PICP_MATCH_FORM_EXACT       the exact full scan (the same bits as FULL; a check path). */
#define PICP_MATCH_FORM_FULL 0
#define PICP_MATCH_FORM_ACCEPT_ONLY 1
#define PICP_MATCH_FORM_EXACT 2
int picp_match_batch_form(int device, int n_problems, const int64_t* off1, const int64_t* off2,
                          const float* desc1, const float* desc2, int dim, float dist_thr,
                          float ratio_thr, int32_t* best_idx, float* best_dist, float* second_dist,
                          int32_t* accepted, int form);

/* ---------------- essential-matrix bootstrap (src/cam.cpp:37-91) ---------------- */

/* Cam::computeEssentialAndRecoverPose: cv::findEssentialMat(p1, p2, K, cv::RANSAC) then
 * cv::recoverPose(E, p1, p2, K, R, t, mask), for many independent two-view problems.  The RANSAC
 * subsets are OpenCV's (its RNG((uint64)-1) stream), the minimal solver is Nister's five-point
 * algorithm, and the selection rule and adaptive iteration bound are OpenCV's. */
typedef struct picp_essential_params {
  double prob;       /* findEssentialMat prob      (default 0.999) */
  double threshold;  /* findEssentialMat threshold (default 1.0 px) */
  int max_iters;     /* findEssentialMat maxIters  (default 1000) */
  int reserved;
  double dist;       /* recoverPose distanceThresh (default 50) */
} picp_essential_params;

void picp_essential_params_default(picp_essential_params* p);

/* Problem i: the pixel pairs (p1[k], p2[k]) for k in [offs[i], offs[i+1]) (float x, y each).
 * K: column-major 3x3.  prm may be NULL (defaults).  Out, per problem: T_out[16 i ..] = the
 * camera-in-world pose of the second view with the first at the origin, [R | t]^-1 column-major
 * (Cam::getPose, src/cam.cpp:81,227; unit baseline), inliers = findEssentialMat's inlier count
 * (0: no model, T = I), good = recoverPose's count.  mask (may be NULL): offs[n] bytes, 1 for
 * the points recoverPose keeps. */
int picp_essential_batch(int device, int n_problems, const int64_t* offs, const float* p1,
                         const float* p2, const float K[9], const picp_essential_params* prm,
                         float* T_out, int32_t* inliers, int32_t* good, uint8_t* mask);

/* ---------------- device-resident VO sequence (exec/icp_test.cpp:36-136) ---------------- */

/* The reference's per-frame loop (match next<->map, PICP from the previous pose, match
 * curr<->next, add_new_world_points, triangulate, append) run entirely on the GPU over
 * independent SEGMENTS of a sequence that advance in lockstep.  Segment s
 * covers frames first[s] .. first[s]+steps[s]: it bootstraps its map by triangulating the
 * matches of its first two frames with the given camera-in-world poses (a stand-in for
 * computeEssentialAndRecoverPose, exec/icp_test.cpp:44-58), then estimates frames
 * first[s]+1 .. first[s]+steps[s].  Matching uses DISTANCE_THRESHOLD 0.2 / RATIO 0.8. */
typedef struct picp_vo picp_vo_t;

/* One pose slot's record; slot 0 of a segment is its bootstrap (only n_new set). */
typedef struct {
  int32_t n_corr;   /* map correspondences of the frame (size of the PICP problem) */
  int32_t n_in;     /* numInliers() after the last round */
  int32_t rounds;   /* oneRound calls */
  int32_t n_new;    /* points triangulated into the map after this frame */
  float chi_in;
  float chi_out;
  int32_t converged;
  int32_t n_projected;
} picp_vo_step;

/* Upload (copy) a packed sequence: frame f = observations [frame_off[f], frame_off[f+1]) of
 * uv (float2, meas-*.dat "point" u v) and desc (float[dim]); frame_off[0] == 0. */
int picp_vo_create(picp_vo_t** out, int device, int rows, int cols, const float K[9],
                   int64_t n_frames, const int64_t* frame_off, const float* uv,
                   const float* desc, int dim);
int picp_vo_destroy(picp_vo_t* h);
/* boot_poses: per segment two column-major 4x4 camera-in-world poses (frames first, first+1).
 * params: threshold (icp_test: 3000), damping, min_inliers, keep_outliers, max_rounds,
 * conv_eps of the per-frame PICP loop. */
int picp_vo_set_segments(picp_vo_t* h, int n_seg, const int64_t* first, const int32_t* steps,
                         const float* boot_poses, const picp_params* params);
int picp_vo_run(picp_vo_t* h);        /* enqueue the whole sequence and wait */
int picp_vo_run_async(picp_vo_t* h);
int picp_vo_sync(picp_vo_t* h);
/* poses: sum(steps+1) camera-in-world 4x4 (segment-major; slot 0 = the bootstrap pose) */
int picp_vo_get_poses(picp_vo_t* h, float* poses);
int picp_vo_get_steps(picp_vo_t* h, picp_vo_step* steps);
/* segment map: *n = its size; the first min(n, cap) points are copied to xyz / desc (nullable) */
int picp_vo_get_map(picp_vo_t* h, int seg, int64_t cap, float* xyz, float* desc, int64_t* n);
/* mean device time of `reps` back-to-back runs (HIP events on the handle's stream) */
int picp_vo_time(picp_vo_t* h, int reps, float* ms_per_run);
int picp_vo_info(picp_vo_t* h, int64_t* n_obs, int64_t* n_slots, int64_t* map_slots, int* npt);
/* Diagnostic: the last run's match outputs per observation (n_obs int32): which = 0 frame->next
 * best index, 1 its accept flag, 2 frame->map best index, 3 its accept flag.  Best indices are
 * defined only where the flag is 1 (the sequence runs the matcher's accept-only form). */
int picp_vo_debug_matches(picp_vo_t* h, int which, int32_t* dst);
/* Diagnostic: with PICP_VO_GUARD=1 at create, every device buffer of the handle is bracketed by
 * 1 MiB pads of a fixed pattern; *bad_bytes = pad bytes that changed, *bad_buffer = 2 * (buffer
 * index in allocation order) + (0 before / 1 after) of the first changed pad, or -1. */
int picp_vo_debug_guard(picp_vo_t* h, int64_t* bad_bytes, int* bad_buffer);

/* ---------------- self-test ---------------- */
/* The projection's reciprocal 1/z must be the correctly rounded one (src/camera.h:30; the
 * chi2 gate is bit-exact): the kernels use a 3-instruction form, valid for every float in
 * [2^-100, 2^100] iff it matches the IEEE division on every float of a binade range.  Counts
 * the mismatching floats of both signs with exponents in [e_lo, e_hi); expected 0. */
int picp_selftest_rcp(int device, int e_lo, int e_hi, uint64_t* mismatches);

#ifdef __cplusplus
}
#endif
#endif /* PICP_C_H */
