#!/bin/bash
# Round 3: persistent parity at 2 and 4 items per lane, the reference's two-view bootstrap on every
# C5 segment vs ground truth (tools/c5_boot_check.py), and C5 with --c5-boot essential.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r03/boot}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "persistent_and_graph" -v --timeout 240 --timeout-method thread > $O/pers_parity.log 2>&1 || { echo "parity failed"; tail -30 $O/pers_parity.log; exit 1; }
tail -1 $O/pers_parity.log
timeout -k 10 200 python tools/c5_boot_check.py > $O/c5_boot_check.log 2>&1 || { echo "boot check failed"; tail $O/c5_boot_check.log; exit 1; }
cat $O/c5_boot_check.log
for B in gt essential; do
  timeout -k 10 240 python bench.py --workload c5 --steps 10 --warmup 3 --samples 3 --no-cpu --skip-extras --c5-boot $B > $O/c5_$B.json 2> $O/c5_$B.err || { echo "c5 $B failed"; tail $O/c5_$B.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c5_$B.json').read().strip().splitlines()[-1]); print('$B', d['value'], d['pose_err_vs_gt_se3_max'], d['bootstrap'])"
done
