#!/bin/bash
# Round 5, call 46: the VO sequence's side-stream chunks enqueued a few steps ahead of the steps
# that wait for them (VO_CHUNK_AHEAD 4: lib/libpicp_amd.so; 1, 2, 64: _ca1/_ca2/_ca64.so) instead
# of all before the bootstrap append (HEAD, lib/libpicp_amd_head.so): VO tests (every schedule
# bit-identical), then C5 and the N = 8 per-rank shape, 2 reps.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t46}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_vo.py tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
: > $OUT/ab.log
for args in "" "--frames 1281"; do for rep in 1 2; do for v in libpicp_amd_head libpicp_amd_ca1 libpicp_amd_ca2 libpicp_amd libpicp_amd_ca64; do
  PICP_LIB=$L/$v.so timeout -k 10 200 python bench.py --workload c5 --no-cpu --skip-extras --steps 20 $args > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 $args', '$v', d['value'], d.get('ms_per_step'), d.get('pose_err_vs_gt_se3_max'))" | tee -a $OUT/ab.log
done; done; done
