#!/bin/bash
# Round 5, call 43: the VO step kernel's linearize at issue priority 1 / 2 (lib/libpicp_amd_vp1,
# _vp2.so; the matcher's waves stay at 0) against 0: VO tests on vp1, then C5 and the N = 8
# per-rank shape, 2 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t43}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
PICP_LIB=$L/libpicp_amd_vp1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_vo.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_vp1.log 2>&1
rc=$?; echo "pytest vp1 rc=$rc"; tail -2 $OUT/pytest_vp1.log; [ $rc -eq 0 ] || exit 1
: > $OUT/ab.log
for args in "" "--frames 1281"; do for rep in 1 2; do for v in libpicp_amd libpicp_amd_vp1 libpicp_amd_vp2; do
  PICP_LIB=$L/$v.so timeout -k 10 200 python bench.py --workload c5 --no-cpu --skip-extras --steps 20 $args > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 $args', '$v', d['value'], d.get('ms_per_step'))" | tee -a $OUT/ab.log
done; done; done
