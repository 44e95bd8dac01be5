// picp_host.h -- host-side internals shared by the runtime translation units (not installed).
#pragma once
#include <hip/hip_runtime.h>

#include "picp_c.h"

// the descriptor matcher's launchers (picp_match.hip)
extern "C" hipError_t picp_launch_match_prep(hipStream_t stream, const float* desc, int64_t n, int dim,
                                             _Float16* h, float* n1, float* n2);
extern "C" hipError_t picp_launch_match_mfma(hipStream_t stream, int n_problems, int64_t max_nq,
                                             const float* q_desc, const float* r_desc,
                                             const _Float16* q_h, const float* q_n1,
                                             const _Float16* r_h, const float* r_n1, const float* r_n2,
                                             const struct MatchProblem* probs, int dim, float dist_thr,
                                             float ratio_thr, int32_t* best_idx, float* best_dist,
                                             float* second_dist, int32_t* accepted, int form, int ksplit,
                                             float4* part, int64_t part_cap);
extern "C" hipError_t picp_launch_match_mfma_parts(hipStream_t stream, int n_problems, int64_t max_nq,
                                                   const float* q_desc, const float* r_desc, const _Float16* q_h,
                                                   const float* q_n1, const _Float16* r_h, const float* r_n1,
                                                   const float* r_n2, const struct MatchProblem* probs, int dim,
                                                   float dist_thr, float ratio_thr, int form, int ksplit, int slot0,
                                                   float4* part, int64_t part_cap);
extern "C" hipError_t picp_launch_match_merge(hipStream_t stream, const struct MatchProblem* probs, int n_problems,
                                              int64_t max_nq, int ksplit, int extra, const float4* part,
                                              int64_t part_cap, float dist_thr, float ratio_thr,
                                              int32_t* best_idx, float* best_dist, float* second_dist,
                                              int32_t* accepted);
// picp_match_ksplit reads PICP_MATCH_KSPLIT each call; picp_match_ksplit_forced takes the forced
// count (0: none) from the caller, so a handle can read the variable once and size its scratch and
// its launches from the same value
extern "C" int picp_match_ksplit(int n_problems, int64_t max_nq, int64_t max_nr, int form);
extern "C" int picp_match_ksplit_forced(int n_problems, int64_t max_nq, int64_t max_nr, int form, int force);
extern "C" int picp_match_ksplit_env(void);
// float4 of scratch a split launch needs (the ranges' partials)
extern "C" int64_t picp_match_split_scratch(int ksplit, int n_problems, int64_t max_nq);
extern "C" int picp_match_prep_kch(int dim);

// records the thread's last error message (picp_last_error) and returns `code`
__attribute__((visibility("hidden"), format(printf, 2, 3))) int picp_set_err(int code, const char* fmt, ...);

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return picp_set_err(e_ == hipErrorOutOfMemory ? PICP_ERR_NOMEM : PICP_ERR_DEVICE,     \
                          "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,  \
                          __LINE__);                                                        \
  } while (0)

#define CHECK_ARG(cond, msg)                                                                \
  do {                                                                                      \
    if (!(cond)) return picp_set_err(PICP_ERR_ARG, "%s", msg);                              \
  } while (0)
