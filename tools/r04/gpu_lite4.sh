#!/bin/bash
# Round 4: LITE zeroing with the per-wave item check (after the block-wide __syncthreads_and form never
# took LITE).  Parity, pose bits vs the previous build, SQ passes, A/B base / new / nolite / liteforce.
export TMPDIR=/tmp
O=gpurun_out/lite4; mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vo.py -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1
rc=$?; tail -3 $O/pt.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/pose_dump.py dump $O/dump_new.npz > $O/dump_new.log 2>&1 || { tail $O/dump_new.log; exit 1; }
PICP_LIB=$L/libpicp_amd_base.so timeout -k 10 300 python -u tools/pose_dump.py dump $O/dump_base.npz > $O/dump_base.log 2>&1 || { tail $O/dump_base.log; exit 1; }
python -u tools/pose_dump.py cmp $O/dump_base.npz $O/dump_new.npz > $O/dump_cmp.log 2>&1; cat $O/dump_cmp.log
for v in base new liteforce; do
  lib=libpicp_amd_$v.so; [ $v = new ] && lib=libpicp_amd.so
  export PICP_LIB=$L/$lib
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/sq_$v -o run --output-format csv -- python3 bench.py --workload c4 --no-cpu --skip-extras --steps 5 --warmup 1 --samples 1 > $O/sq_$v.log 2>&1 || { echo "pmc $v failed"; tail $O/sq_$v.log; exit 1; }
  python3 tools/parse_pmc.py $O/sq_$v/run_counter_collection.csv picp_block > $O/c4_sq_$v.json
  python3 -c "import json; d=json.load(open('$O/c4_sq_$v.json')); print('$v', {k: v['mean'] for k, v in d.items()})"
  unset PICP_LIB
done
run() {  # tag lib workload extra...
  tag=$1; lib=$2; wl=$3; shift 3
  PICP_LIB=$L/$lib timeout -k 10 150 python bench.py --workload $wl "$@" --no-cpu --skip-extras --steps 20 --warmup 3 --samples 3 > $O/b.log 2>&1 || { echo "bench $tag $wl failed"; tail $O/b.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('%-7s %-5s %-14s %12.1f %s' % ('$tag', '$wl', '$*', d['value'], r.get('kernel_us')))" | tee -a $O/ab.log
}
: > $O/ab.log
for rep in 1 2; do
  for v in base:libpicp_amd_base.so new:libpicp_amd.so nolite:libpicp_amd_nolite.so force:libpicp_amd_liteforce.so; do
    t=${v%%:*}; lib=${v#*:}
    run $t $lib c4
    run $t $lib c4 --problems 128
    run $t $lib c3
    run $t $lib c2
    run $t $lib c5
  done
done
