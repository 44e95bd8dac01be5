#!/bin/bash
# Round 4: the LITE zeroing of the pair accumulation (picp_device.h accumulate_pinhole2: iz and e
# only, under lite_bounds) and per-lane counts (cnt_add).  Parity suite on the new default, pose
# bits vs the previous build (libpicp_amd_base.so), then interleaved A/B: base / new / nolite
# (-DPICP_LITE=0) / ballot (-DPICP_LANE_COUNTS=0).
export TMPDIR=/tmp
O=gpurun_out/lite; mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vo.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1
rc=$?; tail -3 $O/pt.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/pose_dump.py dump $O/dump_new.npz > $O/dump_new.log 2>&1 || { tail $O/dump_new.log; exit 1; }
PICP_LIB=$L/libpicp_amd_base.so timeout -k 10 300 python -u tools/pose_dump.py dump $O/dump_base.npz > $O/dump_base.log 2>&1 || { tail $O/dump_base.log; exit 1; }
python -u tools/pose_dump.py cmp $O/dump_base.npz $O/dump_new.npz > $O/dump_cmp.log 2>&1; cat $O/dump_cmp.log
run() {  # tag lib workload extra...
  tag=$1; lib=$2; wl=$3; shift 3
  PICP_LIB=$L/$lib timeout -k 10 150 python bench.py --workload $wl "$@" --no-cpu --skip-extras --steps 20 --warmup 3 --samples 3 > $O/b.log 2>&1 || { echo "bench $tag $wl failed"; tail $O/b.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('%-7s %-5s %-14s %12.1f %s' % ('$tag', '$wl', '$*', d['value'], r.get('kernel_us')))" | tee -a $O/ab.log
}
: > $O/ab.log
for rep in 1 2; do
  for v in base:libpicp_amd_base.so new:libpicp_amd.so nolite:libpicp_amd_nolite.so ballot:libpicp_amd_ballot.so; do
    t=${v%%:*}; lib=${v#*:}
    run $t $lib c4
    run $t $lib c4 --problems 128
    run $t $lib c3
    run $t $lib c2
    [ $t = ballot ] || run $t $lib c5
  done
done
