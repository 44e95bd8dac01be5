#!/bin/bash
# Round 4: 1024-thread blocks for split 1/2 (PICP_BLOCK_BS=1024: four waves per SIMD, one partner
# exchange) vs the 512-thread block and the split-4 default: block parity under the variant, then
# C4 at 128, 256 and 1024 frames (the pair-mode bit-identity test compares with the 512-thread
# layout, so it is deselected here).
export TMPDIR=/tmp
O=gpurun_out/bs1024; mkdir -p $O
PICP_BLOCK_BS=1024 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "not pair_mode" -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1
rc=$?; tail -3 $O/pt.log; [ $rc -eq 0 ] || exit 1
run() {  # tag problems env...
  tag=$1; P=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --workload c4 --problems $P --no-cpu --skip-extras --steps 30 --warmup 3 --samples 3 > $O/b.log 2>&1 || { echo "bench $tag failed"; tail $O/b.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', $P, d['value'], r['kernel_us'])" | tee -a $O/ab.log
}
: > $O/ab.log
for rep in 1 2; do
  run s4_default 128
  run s2_512 128 PICP_BLOCK_SPLIT=2
  run s2_1024 128 PICP_BLOCK_SPLIT=2 PICP_BLOCK_BS=1024
  run s1_512 256
  run s1_1024 256 PICP_BLOCK_BS=1024
  run s1_512 1024
  run s1_1024 1024 PICP_BLOCK_BS=1024
done
