#!/bin/bash
# Round 4: the leader's adaptive sweep wait (PICP_SWEEP_WAIT=M ticks): parity under it, the sweep
# stamps with it, then interleaved C2/C3 A/B against the default (no wait).
export TMPDIR=/tmp
O=gpurun_out/sww; mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
PICP_LIB=$L/libpicp_amd_sw40.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pt.log 2>&1
rc=$?; tail -2 $O/pt.log; [ $rc -eq 0 ] || exit 1
PICP_STAMPS_LIB=$L/libpicp_amd_stamps_sw40.so timeout -k 10 200 python tools/pstamps.py --n 100000 > $O/pstamps_c2_sw40.log 2>&1 || { tail $O/pstamps_c2_sw40.log; exit 1; }
cat $O/pstamps_c2_sw40.log
run() {  # tag lib workload
  PICP_LIB=$L/$2 timeout -k 10 150 python bench.py --workload $3 --no-cpu --skip-extras --steps 20 --warmup 5 --samples 3 > $O/b.log 2>&1 || { echo "bench $1 $3 failed"; tail $O/b.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('%-5s %-3s %12.1f %s' % ('$1', '$3', d['value'], r.get('kernel_us')))" | tee -a $O/ab.log
}
: > $O/ab.log
for rep in 1 2 3; do
  for v in base:libpicp_amd.so sw20:libpicp_amd_sw20.so sw40:libpicp_amd_sw40.so sw70:libpicp_amd_sw70.so; do
    run ${v%%:*} ${v#*:} c2
    run ${v%%:*} ${v#*:} c3
  done
done
