#!/bin/bash
# Round-2 session c: matcher (single-asm candidate mask) A/B + phase stamps of the wave solve.
export TMPDIR=/tmp
OUT=gpurun_out/r02c
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo.py tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
OUT=$OUT/ab WLS="c5" LIBS="libpicp_amd_solve libpicp_amd" REPS=3 TESTS="" bash tools/gpu_ab.sh || exit 1
OUT=gpurun_out/r02c/pst PICP_STAMPS_LIB=$PWD/02-visualodometry_amd/lib/libpicp_amd_stamps_new.so bash tools/gpu_pstamps.sh > /dev/null 2>&1 || { echo "pstamps new failed"; exit 1; }
mv gpurun_out/r02c/pst/pstamps_c2.log gpurun_out/r02c/pst/pstamps_c2_new.log; mv gpurun_out/r02c/pst/pstamps_c3.log gpurun_out/r02c/pst/pstamps_c3_new.log
OUT=gpurun_out/r02c/pst PICP_STAMPS_LIB=$PWD/02-visualodometry_amd/lib/libpicp_amd_stamps_base.so bash tools/gpu_pstamps.sh > /dev/null 2>&1 || { echo "pstamps base failed"; exit 1; }
tail -12 gpurun_out/r02c/pst/*.log
OUT=gpurun_out/r02c/bst VARS="base new" bash tools/gpu_bstamps_ab.sh
