#!/bin/bash
# A/B of the packed-FP32 block kernel (shipped) vs the no-packed variant (make variant VAR=nopk
# VAR_FLAGS=-DPICP_NO_PK), interleaved on one box: C4 and C5 (block kernel), C3 (persistent).
export TMPDIR=/tmp
OUT=gpurun_out/r03/${TAG:-abpk}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
for rep in 1 2; do
  for lib in libpicp_amd.so ${LIBS:-libpicp_amd_nopk.so}; do
    for wl in ${WLS:-c4 c5}; do
      PICP_LIB=$L/$lib timeout -k 10 240 python bench.py --workload $wl --steps ${STEPS:-10} --warmup 3 --no-cpu --skip-extras > $OUT/${wl}_${lib}_$rep.json 2> $OUT/${wl}_${lib}_$rep.err || { echo "$wl $lib failed"; tail -5 $OUT/${wl}_${lib}_$rep.err; exit 1; }
      python - $OUT/${wl}_${lib}_$rep.json $wl $lib <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%-4s %-28s value %.4g %s  ms/step %.4f" % (sys.argv[2], sys.argv[3], d["value"], d["unit"], d["ms_per_step"]))
PY
    done
  done
done
