#!/bin/bash
# Round 5, call 16: the two-level fan-in (PICP_PXCD: XCD partials summed in the L2, then the eight
# of them) against the one-level multi-solver sweep (-DPICP_PXCD=0, lib/libpicp_amd_px0.so) and
# the one-level sweep with the followers' polls 2 x 64 clocks apart (lib/libpicp_amd_st2.so); the
# parity suite on the candidate first; C2 and C3 interleaved, 3 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t16}
mkdir -p $OUT
OUT=$OUT/ab TESTS="tests/test_gpu_parity.py" WLS="c2 c3" LIBS="libpicp_amd_px0 libpicp_amd_st2 libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
