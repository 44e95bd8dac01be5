#!/bin/bash
# Round 4: the one-slot accumulation with the per-item math in pairs (PICP_P1, picp_device.h
# accumulate_pinhole_p1; the same bits as item by item): parity, then C4 at 128 frames (split 4
# with tail priority, pair mode) and C5, P1 vs the item-by-item build (P0).
export TMPDIR=/tmp
O=gpurun_out/p1; mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vo.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1
rc=$?; tail -3 $O/pt.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/pose_dump.py dump $O/dump_p1.npz > $O/dump_p1.log 2>&1 || { tail $O/dump_p1.log; exit 1; }
PICP_LIB=$L/libpicp_amd_p0.so timeout -k 10 300 python -u tools/pose_dump.py dump $O/dump_p0.npz > $O/dump_p0.log 2>&1 || { tail $O/dump_p0.log; exit 1; }
python -u tools/pose_dump.py cmp $O/dump_p0.npz $O/dump_p1.npz > $O/dump_cmp.log 2>&1; cat $O/dump_cmp.log
run() {  # tag problems env...
  tag=$1; P=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --workload c4 --problems $P --no-cpu --skip-extras --steps 30 --warmup 3 --samples 3 > $O/b.log 2>&1 || { echo "bench $tag failed"; tail $O/b.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', $P, d['value'], r['kernel_us'])" | tee -a $O/ab.log
}
runvo() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload c5 --no-cpu --skip-extras --steps 10 --warmup 2 --samples 3 > $O/c5.log 2>&1 || { echo "c5 $tag failed"; tail $O/c5.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/c5.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['chain_step_us'])" | tee -a $O/ab.log
}
: > $O/ab.log
for rep in 1 2; do
  run s4prio_p1 128 PICP_BLOCK_SPLIT=4 PICP_LIB=$L/libpicp_amd_prio.so
  run s4prio_p0 128 PICP_BLOCK_SPLIT=4 PICP_LIB=$L/libpicp_amd_p0prio.so
  run pair_p1 128 PICP_BLOCK_PAIR=1
  run pair_p0 128 PICP_BLOCK_PAIR=1 PICP_LIB=$L/libpicp_amd_p0.so
  run s2 128 PICP_BLOCK_SPLIT=2
  run pair_p1 256 PICP_BLOCK_PAIR=1
  runvo c5_p1
  runvo c5_p0 PICP_LIB=$L/libpicp_amd_p0.so
done
