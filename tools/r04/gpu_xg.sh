#!/bin/bash
# Round 4: the split exchange's partner loads batched (PICP_XG_BATCH=1: one round trip per poll)
# vs partner by partner (xg0).  Block-mode parity, pose bits vs xg0, then interleaved A/B on C4
# at 128 (split 4), 256 and 512 frames and 1,024 (split 1: unaffected).
export TMPDIR=/tmp
O=gpurun_out/xg; mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1
rc=$?; tail -2 $O/pt.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/pose_dump.py dump $O/dump_new.npz > $O/dump_new.log 2>&1 || { tail $O/dump_new.log; exit 1; }
PICP_LIB=$L/libpicp_amd_xg0.so timeout -k 10 300 python -u tools/pose_dump.py dump $O/dump_xg0.npz > $O/dump_xg0.log 2>&1 || { tail $O/dump_xg0.log; exit 1; }
python -u tools/pose_dump.py cmp $O/dump_xg0.npz $O/dump_new.npz > $O/dump_cmp.log 2>&1; cat $O/dump_cmp.log
run() {  # tag lib problems
  tag=$1; lib=$2; P=$3
  PICP_LIB=$L/$lib timeout -k 10 150 python bench.py --workload c4 --problems $P --no-cpu --skip-extras --steps 20 --warmup 5 --samples 3 > $O/b.log 2>&1 || { echo "bench $tag $P failed"; tail $O/b.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('%-5s %5d %12.1f %s' % ('$tag', $P, d['value'], r.get('kernel_us')))" | tee -a $O/ab.log
}
: > $O/ab.log
for rep in 1 2 3; do
  for P in 128 256 512 1024; do
    run new libpicp_amd.so $P
    run xg0 libpicp_amd_xg0.so $P
  done
done
