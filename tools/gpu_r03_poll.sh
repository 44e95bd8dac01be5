#!/bin/bash
# Round 3: the followers' pose polls -- phase stamps with and without the stagger (C2, C3), then
# an interleaved C2 A/B of one poll (stag0), two polls 4 or 8 x 64 clocks apart (np2k4, default)
# and three polls 5 x 64 apart (np3k5).  Each step time-limited; stop at the first failure.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r03/poll}
mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
for lib in libpicp_amd_stamps.so libpicp_amd_stamps_stag0.so; do
  PICP_STAMPS_LIB=$L/$lib timeout -k 10 200 python tools/pstamps.py --n 100000 > $O/pstamps_c2_$lib.log 2>&1 || { tail $O/pstamps_c2_$lib.log; exit 1; }
  echo "== $lib"; grep -E "round period|others pose_received|leader" $O/pstamps_c2_$lib.log
done
for rep in 1 2 3; do
  for lib in libpicp_amd_stag0.so libpicp_amd.so libpicp_amd_np2k4.so libpicp_amd_np3k5.so; do
    PICP_LIB=$L/$lib timeout -k 10 240 python bench.py --workload c2 --steps 20 --warmup 3 --samples 5 --no-cpu --skip-extras > $O/ab.json 2> $O/ab.err || { echo "c2 $lib failed"; tail -5 $O/ab.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('c2 %-26s %10.0f %s  round %.3f us' % ('$lib', d['value'], d['unit'], d['roofline']['kernel_us'] / 50))"
  done
done
