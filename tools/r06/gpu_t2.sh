#!/bin/bash
# Round 6, call 2 (Jacobi triangulation restored as the default): the matcher's range merge fused
# into the matcher (no merge launch) and the append's reordered loads + LDS pairs -- whole GPU suite,
# a dump of the 8e segment 0 at this library, then A/B at the C5 shapes: the separate merge kernel
# (lib/libpicp_amd_mergek.so), the round-5 append (lib/libpicp_amd_app0.so), and the VO step
# chains (PICP_VO_CHAINS = 2, 4, 8) at the latency-bound shapes.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t2}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u tools/r05/vo_dump.py $OUT/seg0_8e.npz || exit 1
run() {  # tag env...   (bench args in $ARGS)
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $ARGS > $OUT/run.log 2>&1 || { echo "bench $tag failed"; tail $OUT/run.log; return 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('$tag', '$ARGS', d['value'], d.get('chain_step_us'), d.get('ate_m'), d.get('rounds_sync'))" | tee -a $OUT/ab.log
}
: > $OUT/ab.log
for ARGS in "" "--seg-len 1250 --steps 2 --warmup 1 --samples 1" "--frames 1281"; do for rep in 1 2; do
  run mergek PICP_LIB=$L/libpicp_amd_mergek.so || exit 1
  run app0 PICP_LIB=$L/libpicp_amd_app0.so || exit 1
  run new PICP_LIB=$L/libpicp_amd.so || exit 1
done; done
for ARGS in "--seg-len 1250 --steps 2 --warmup 1 --samples 1" "--frames 1281"; do for ch in 1 2 4 8; do
  run chains$ch PICP_VO_CHAINS=$ch || exit 1
done; done
