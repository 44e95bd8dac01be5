#!/bin/bash
# Round 5, call 35: the VO step's PICP block at 1,024 threads (PICP_VO_BS=1024: four waves per
# SIMD, one register item per lane, the rest in the LDS stage) against 512: VO tests with it (but
# the fused-vs-separate gather identity: the separate path keeps 512 threads, other lanes),
# then C5 (250 x 40) and the N = 8 per-rank shape (32 x 40, --frames 1281), HEAD / 512 / 1024.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t35}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
PICP_VO_BS=1024 timeout -k 10 600 python -u -m pytest tests/test_gpu_vo.py -k "not fused_gather" -x -q --timeout 120 --timeout-method thread > $OUT/pytest_bs1024.log 2>&1
rc=$?; echo "pytest bs1024 rc=$rc"; tail -2 $OUT/pytest_bs1024.log; [ $rc -eq 0 ] || exit 1
: > $OUT/ab.log
for args in "" "--frames 1281"; do for rep in 1 2; do for v in head bs512 bs1024; do
  lib=$L/libpicp_amd.so; env=""
  [ $v = head ] && lib=$L/libpicp_amd_head.so
  [ $v = bs1024 ] && env="PICP_VO_BS=1024"
  env $env PICP_LIB=$lib timeout -k 10 200 python bench.py --workload c5 --no-cpu --skip-extras --steps 20 $args > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 $args', '$v', d['value'], d.get('ms_per_step'), d.get('pose_err_vs_gt_se3', d.get('pose_err_vs_gt_se3_max')))" | tee -a $OUT/ab.log
done; done; done
