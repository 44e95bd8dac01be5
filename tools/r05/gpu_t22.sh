#!/bin/bash
# Round 5, call 22: the persistent kernel's round loop instantiated per role (solver / follower)
# against one loop branching on the role (HEAD, lib/libpicp_amd_head.so): the persistent parity
# tests on the candidate, then C2 and C3 interleaved, 3 reps; phase stamps of the candidate.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t22}
mkdir -p $OUT
OUT=$OUT/ab TESTS="tests/test_gpu_parity.py" WLS="c2 c3" LIBS="libpicp_amd_head libpicp_amd" REPS=3 bash tools/gpu_ab.sh || exit 1
timeout -k 10 200 python tools/pstamps.py --n 100000 > $OUT/pstamps_c2.log 2>&1 || { tail $OUT/pstamps_c2.log; exit 1; }
cat $OUT/pstamps_c2.log
timeout -k 10 200 python tools/pstamps.py --n 1000000 --outlier 0.3 > $OUT/pstamps_c3.log 2>&1 || { tail $OUT/pstamps_c3.log; exit 1; }
cat $OUT/pstamps_c3.log
