#!/bin/bash
# Round 4, second pass: pair mode with one finishing wave per frame (parity vs the block kernel,
# C4 at 128-1024 frames) and the C5 step-chain A/B (world match split, early-stream priority,
# step-kernel issue priority, append fused).
export TMPDIR=/tmp
O=gpurun_out/pair2; mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "pair_mode or block_split" --timeout 300 --timeout-method thread > $O/pt.log 2>&1
rc=$?; tail -3 $O/pt.log; [ $rc -eq 0 ] || exit 1
PICP_LIB=$L/libpicp_amd_voprio.so timeout -k 10 400 python -u -m pytest tests/test_gpu_vo.py -x -q -k "fused_gather or schedules or beside" --timeout 300 --timeout-method thread > $O/pt_vo.log 2>&1
rc=$?; tail -2 $O/pt_vo.log; [ $rc -eq 0 ] || exit 1
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
  run pair2 128 PICP_BLOCK_PAIR=1
  run pair2_prio 128 PICP_BLOCK_PAIR=1 PICP_LIB=$L/libpicp_amd_prio.so
  run base 256
  run pair2 256 PICP_BLOCK_PAIR=1
  run pair2 512 PICP_BLOCK_PAIR=1
  run pair2 1024 PICP_BLOCK_PAIR=1
  runvo split0 PICP_VO_SPLIT=0
  runvo split0_fuse2 PICP_VO_SPLIT=0 PICP_VO_FUSE=2
  runvo split1_elo PICP_VO_SPLIT=1 PICP_VO_EPRIO=0
  runvo split0_voprio PICP_VO_SPLIT=0 PICP_LIB=$L/libpicp_amd_voprio.so
  runvo split1_voprio PICP_VO_SPLIT=1 PICP_LIB=$L/libpicp_amd_voprio.so
  runvo split1_elo_voprio PICP_VO_SPLIT=1 PICP_VO_EPRIO=0 PICP_LIB=$L/libpicp_amd_voprio.so
  runvo split1_elo_voprio_fuse2 PICP_VO_SPLIT=1 PICP_VO_EPRIO=0 PICP_VO_FUSE=2 PICP_LIB=$L/libpicp_amd_voprio.so
done
