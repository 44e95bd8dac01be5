#!/bin/bash
# The fused VO step kernel in 256-thread blocks (PICP_VO_BS=256 in an A/B build of picp_vo_runtime.cpp:
# NPT doubled, two segments per CU)
# vs 512: the VO oracle-parity tests under 256, then C5 interleaved, three repetitions.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/vobs}
mkdir -p $O
PICP_VO_BS=256 timeout -k 10 600 python -u -m pytest tests/test_gpu_vo.py -x -q --timeout 240 --timeout-method thread -k "reference_data or synthetic_segments or replay" > $O/pytest_vo256.log 2>&1
rc=$?; tail -2 $O/pytest_vo256.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest_vo256.log | head; exit 1; }
: > $O/ab_c5.log
for rep in 1 2 3; do
  for b in 512 256; do
    PICP_VO_BS=$b timeout -k 10 240 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu --skip-extras > $O/c5.json 2> $O/c5.err || { echo "c5 bs=$b failed"; tail -5 $O/c5.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]); print('bs=$b', round(d['value']), d['unit'], d['ms_per_step'], d['pose_err_vs_gt_se3_max'])" | tee -a $O/ab_c5.log
  done
done
