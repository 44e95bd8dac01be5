#!/bin/bash
# hipcc with packed-FP32 VALU code (v_pk_fma/mul/add_f32) disabled for the whole device compile
# (csrc/picp_internal.h explains why).  The feature goes to every function of the translation unit,
# HIP's own header functions included, so they keep inlining into the kernels (a per-kernel
# target attribute blocks that: the callees' features are no subset of the kernel's).  clang also
# hands the feature to the x86 host compile, which ignores it with a note per TU: dropped here.
"${HIPCC:-/opt/rocm/bin/hipcc}" -Xclang -target-feature -Xclang -packed-fp32-ops "$@" \
  2> >(grep -v "packed-fp32-ops' is not a recognized feature for this target" >&2)
