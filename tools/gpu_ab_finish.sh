#!/bin/bash
# Round 3: the finishing wave's DPP-row solve (default, PICP_FINISH_WAVE=1) vs the one-lane form
# (make abvariant AB=lanesolve AB_FLAGS=-DPICP_FINISH_WAVE=0): the GPU suite, a bit-identity check
# of the poses of both builds (tools/pose_dump.py), then interleaved A/B of C2 / C4 / C5.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r03/finish}
mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
if [ -z "$SKIP_PYTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; exit 1; }
tail -1 $O/pytest_gpu.log
fi
for lib in libpicp_amd.so libpicp_amd_lanesolve.so; do
  PICP_LIB=$L/$lib timeout -k 10 300 python tools/pose_dump.py dump $O/poses_$lib.npz > $O/dump_$lib.log 2>&1 || { echo "dump $lib failed"; tail -5 $O/dump_$lib.log; exit 1; }
done
python tools/pose_dump.py cmp $O/poses_libpicp_amd.so.npz $O/poses_libpicp_amd_lanesolve.so.npz | tee $O/bitcmp.log
for rep in 1 2; do
  for lib in libpicp_amd.so libpicp_amd_lanesolve.so; do
    for wl in c2 c4 c5; do
      PICP_LIB=$L/$lib timeout -k 10 240 python bench.py --workload $wl --steps 10 --warmup 3 --samples 3 --no-cpu --skip-extras > $O/ab.json 2> $O/ab.err || { echo "$wl $lib failed"; tail -5 $O/ab.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('%-3s %-26s %10.0f %s  ms/step %.4f' % ('$wl', '$lib', d['value'], d['unit'], d['ms_per_step']))"
    done
  done
done
