#!/bin/bash
# Round 4: the followers' pose polls in the persistent kernel: two in flight 8 x 64 clocks apart
# (default) vs three in flight (PICP_POSE_NPOLL=3), 4 x 64 clocks apart, and both; C2 and C3.
export TMPDIR=/tmp
O=gpurun_out/poll; mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
run() {
  PICP_LIB=$L/$2 timeout -k 10 150 python bench.py --workload $3 --no-cpu --skip-extras --steps 20 --warmup 5 --samples 3 > $O/b.log 2>&1 || { echo "bench $1 $3 failed"; tail $O/b.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('%-6s %-3s %12.1f %s' % ('$1', '$3', d['value'], r.get('kernel_us')))" | tee -a $O/ab.log
}
: > $O/ab.log
for rep in 1 2 3; do
  for v in base:libpicp_amd.so np3:libpicp_amd_np3.so stag4:libpicp_amd_stag4.so np3s4:libpicp_amd_np3s4.so; do
    run ${v%%:*} ${v#*:} c2
    run ${v%%:*} ${v#*:} c3
  done
done
