// picp_host.h -- host-side internals shared by the runtime translation units (not installed).
#pragma once
#include <hip/hip_runtime.h>

#include "picp_c.h"

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
