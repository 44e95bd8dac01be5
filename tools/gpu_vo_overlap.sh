#!/bin/bash
# C5 A/B of VO runtime variants: the VO GPU tests on the candidate, then REPS interleaved C5
# bench runs per variant ("lib[:ENV=V[,ENV=V]]"), plus one kernel trace of the candidate.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/vo_ov}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_vo.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
: > $OUT/ab.log
for rep in $(seq ${REPS:-2}); do for v in ${VARS}; do
  lib=${v%%:*}; envs=""; [ "$v" != "$lib" ] && envs=$(echo ${v#*:} | tr ',' ' ')
  env PICP_LIB=$L/$lib.so $envs timeout -k 10 200 python bench.py --workload c5 --no-cpu --skip-extras --steps 10 > $OUT/run.log 2>&1 || { echo "c5 $v failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5', '$v', d['value'], d['pose_err_vs_gt_se3_max'])" | tee -a $OUT/ab.log
done; done
if [ -n "$TRACE" ]; then
  lib=${TRACE%%:*}; envs=""; [ "$TRACE" != "$lib" ] && envs=$(echo ${TRACE#*:} | tr ',' ' ')
  export PICP_LIB=$L/$lib.so; for kv in $envs; do export $kv; done
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/tr -o run --output-format csv -- python3 bench.py --workload c5 --no-cpu --skip-extras --steps 3 > $OUT/tr.log 2>&1 || { echo "trace failed"; tail $OUT/tr.log; exit 1; }
  cut -d, -f1-4 $OUT/tr/run_kernel_stats.csv
fi
