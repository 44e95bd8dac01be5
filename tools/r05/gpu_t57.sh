#!/bin/bash
# Round 5, call 57: the triangulation's rotation angle from the raw rcp / rsqrt estimates (only
# c = 1/sqrt(1+t^2) Newton-refined; lib/libpicp_amd_traw.so) against both refined (lib/libpicp_amd.so):
# triangulation and VO tests, then C5 / per-rank / 8e, 2 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t57}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
PICP_LIB=$L/libpicp_amd_traw.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vo.py tests/test_gpu_scale.py tests/test_gpu_vo_long.py -x -q -k "triangulation or vo or scale or long" --timeout 300 --timeout-method thread > $OUT/pytest_traw.log 2>&1
rc=$?; echo "pytest traw rc=$rc"; tail -2 $OUT/pytest_traw.log; [ $rc -eq 0 ] || exit 1
: > $OUT/ab.log
for args in "" "--frames 1281" "--seg-len 1250 --steps 2 --warmup 1 --samples 1"; do for rep in 1 2; do for v in libpicp_amd libpicp_amd_traw; do
  PICP_LIB=$L/$v.so timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras $args > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 $args', '$v', d['value'], d.get('ms_per_step'), d.get('ate_m'))" | tee -a $OUT/ab.log
done; done; done
