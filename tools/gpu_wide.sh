#!/bin/bash
# C3 with the wide persistent variant (1024-thread blocks, 4 items per lane, scalar Acc) vs the
# 512-thread packed one: parity at 1M with the wide variant forced, interleaved bench runs, stamps
export TMPDIR=/tmp
O=gpurun_out/wide
mkdir -p $O
PICP_PERSIST_WIDE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "full_size or persistent_and_graph or tag_bases" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.log
for rep in 1 2 3; do for W in 0 1; do
  PICP_PERSIST_WIDE=$W timeout -k 10 200 python bench.py --workload c3 --no-cpu --skip-extras --steps 20 > $O/run.log 2>&1 || { echo "bench W=$W failed"; tail $O/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/run.log').read().strip().splitlines()[-1]); r=d['roofline']; print('c3 wide=$W', d['value'], r['kernel_us'], r['blocks_per_launch'], d['pose_err_vs_gt_se3'])" | tee -a $O/ab.log
done; done
PICP_PERSIST_WIDE=1 PICP_STAMPS_LIB=$PWD/02-visualodometry_amd/lib/libpicp_amd_stamps_new.so timeout -k 10 200 python tools/pstamps.py --n 1000000 --outlier 0.3 > $O/pstamps_c3_wide.log 2>&1 || { echo "pstamps failed"; tail $O/pstamps_c3_wide.log; exit 1; }
tail -6 $O/pstamps_c3_wide.log
