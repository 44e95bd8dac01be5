#!/bin/bash
# Round 3: staggered pose polls in the persistent kernel's follower wait.  Default build
# (PICP_POSE_STAGGER=8) vs 0 (one poll, the round-2 loop) and 16: the GPU suite on the default,
# then interleaved A/B of C2 and C3.  Each step time-limited; stop at the first failure.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r03/stagger}
mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
if [ -z "$SKIP_PYTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit 1; }
tail -1 $O/pytest_gpu.log
fi
for rep in 1 2 3; do
  for lib in ${LIBS:-libpicp_amd_stag0.so libpicp_amd.so libpicp_amd_stag16.so}; do
    for wl in ${WLS:-c2 c3}; do
      PICP_LIB=$L/$lib timeout -k 10 240 python bench.py --workload $wl --steps 20 --warmup 3 --samples 5 --no-cpu --skip-extras > $O/ab.json 2> $O/ab.err || { echo "$wl $lib failed"; tail -5 $O/ab.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('%-3s %-26s %10.0f %s  ms/step %.4f  round %.3f us' % ('$wl', '$lib', d['value'], d['unit'], d['ms_per_step'], d['roofline']['kernel_us'] / 50))"
    done
  done
done
