#!/bin/bash
# Round 4: one block per problem with two blocks per CU (PICP_BLOCK_DUAL=1: the 128-VGPR kernel,
# half the LDS stage, the rest streamed) vs the default one block per CU, C4 at 256-1024 frames.
export TMPDIR=/tmp
O=gpurun_out/dual; mkdir -p $O
PICP_BLOCK_DUAL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -k "not pair_mode" -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1
rc=$?; tail -2 $O/pt.log; [ $rc -eq 0 ] || exit 1
run() {  # tag problems env...
  tag=$1; P=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --workload c4 --problems $P --no-cpu --skip-extras --steps 20 --warmup 5 --samples 3 > $O/b.log 2>&1 || { echo "bench $tag $P failed"; tail $O/b.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('%-5s %5d %12.1f %s' % ('$tag', $P, d['value'], r.get('kernel_us')))" | tee -a $O/ab.log
}
: > $O/ab.log
for rep in 1 2 3; do
  for P in 256 512 1024; do
    run base $P PICP_BLOCK_DUAL=0
    run dual $P PICP_BLOCK_DUAL=1
  done
done
