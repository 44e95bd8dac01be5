#!/bin/bash
# Round 3: the wide persistent shape for npt 8 (1024 threads x 4 items, default) vs 512 x 8
# (make abvariant AB=pnarrow AB_FLAGS=-DPICP_PWIDE=0): the GPU suite, then A/B of C3 and C2.

export TMPDIR=/tmp
O=${OUT:-gpurun_out/r03/pwide}
mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
if [ -z "$SKIP_PYTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
fi
for rep in 1 2; do
  for lib in libpicp_amd.so ${LIBS:-libpicp_amd_pnarrow.so}; do
    for wl in ${WLS:-c3 c2}; do
      PICP_LIB=$L/$lib timeout -k 10 240 python bench.py --workload $wl --steps 10 --warmup 3 --samples 3 --no-cpu --skip-extras > $O/ab.json 2> $O/ab.err || { echo "$wl $lib failed"; tail -5 $O/ab.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('%-3s %-24s %10.0f %s  ms/step %.4f  err %.2e' % ('$wl', '$lib', d['value'], d['unit'], d['ms_per_step'], d.get('pose_err_vs_gt_se3', d.get('pose_err_vs_gt_se3_max', 0))))"
    done
  done
done
