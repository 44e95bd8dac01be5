#!/bin/bash
# Round 4: pair mode (two frames per block, tails interleaved) -- parity vs the block kernel,
# then C4 per-rank shapes (128, 256, 512 frames) and the 1024-frame batch, pair off / on;
# the VO append fused into the PICP kernel (PICP_VO_FUSE=2) and the split world match
# (PICP_VO_SPLIT): VO and matcher GPU tests, then C5 A/B.
export TMPDIR=/tmp
O=gpurun_out/pair; mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "pair_mode or block_split or tag_bases" --timeout 300 --timeout-method thread > $O/pt.log 2>&1
rc=$?; tail -12 $O/pt.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_vo.py tests/test_gpu_match.py -x -v --timeout 300 --timeout-method thread > $O/pt_vo.log 2>&1
rc=$?; tail -8 $O/pt_vo.log; [ $rc -eq 0 ] || exit 1
run() {  # tag problems env...
  tag=$1; P=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --workload c4 --problems $P --no-cpu --skip-extras --steps 30 --warmup 3 --samples 3 > $O/b.log 2>&1 || { echo "bench $tag failed"; tail $O/b.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', $P, d['value'], r['kernel_us'])" | tee -a $O/ab.log
}
runvo() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload c5 --no-cpu --skip-extras --steps 10 --warmup 2 --samples 3 > $O/c5.log 2>&1 || { echo "c5 $tag failed"; tail $O/c5.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/c5.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['chain_step_us'], d['trajectory']['ate_rmse_m'])" | tee -a $O/ab.log
}
: > $O/ab.log
for rep in 1 2; do
  run s4_prio 128 PICP_BLOCK_SPLIT=4 PICP_LIB=$L/libpicp_amd_prio.so
  run pair 128 PICP_BLOCK_PAIR=1
  run pair_s2 128 PICP_BLOCK_PAIR=1 PICP_BLOCK_SPLIT=2
  run base 256
  run pair 256 PICP_BLOCK_PAIR=1
  run base 512
  run pair 512 PICP_BLOCK_PAIR=1
  run base 1024
  run pair 1024 PICP_BLOCK_PAIR=1
  runvo c5_split0 PICP_VO_SPLIT=0
  runvo c5_split1 PICP_VO_SPLIT=1
  runvo c5_split1_fuse2 PICP_VO_SPLIT=1 PICP_VO_FUSE=2
done
