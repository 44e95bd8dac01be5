#!/bin/bash
# Round 4: C4 at the N = 8 per-rank shape (128 frames x 10k) -- split 2 vs split 4 (256- and
# 512-thread parts), with and without tail priority; parity of the block splits first.
export TMPDIR=/tmp
mkdir -p gpurun_out/c4_128
O=gpurun_out/c4_128
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "block_split or tag_bases or uniform_multi" --timeout 200 --timeout-method thread > $O/pt.log 2>&1
rc=$?; tail -2 $O/pt.log; [ $rc -eq 0 ] || exit 1
PICP_LIB=$L/libpicp_amd_prio.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "block_split" --timeout 200 --timeout-method thread > $O/pt_prio.log 2>&1
rc=$?; tail -2 $O/pt_prio.log; [ $rc -eq 0 ] || exit 1
run() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --workload c4 --problems 128 --no-cpu --skip-extras --steps 50 --warmup 5 --samples 3 > $O/b.log 2>&1 || { echo "bench $tag failed"; tail $O/b.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], r['kernel_us'], r.get('blocks_per_launch'))" | tee -a $O/ab.log
}
: > $O/ab.log
for rep in 1 2; do
  run s2 PICP_BLOCK_SPLIT=2
  run s4_256 PICP_BLOCK_SPLIT=4 PICP_BLOCK_S4BS=256
  run s4_512 PICP_BLOCK_SPLIT=4
  run s2_prio PICP_BLOCK_SPLIT=2 PICP_LIB=$L/libpicp_amd_prio.so
  run s4_256_prio PICP_BLOCK_SPLIT=4 PICP_BLOCK_S4BS=256 PICP_LIB=$L/libpicp_amd_prio.so
  run s4_512_prio PICP_BLOCK_SPLIT=4 PICP_LIB=$L/libpicp_amd_prio.so
done
timeout -k 10 200 python bench.py --workload c4 --no-cpu --skip-extras --steps 20 --warmup 3 --samples 3 > $O/b1024.log 2>&1 && tail -c 600 $O/b1024.log
