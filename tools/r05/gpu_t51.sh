#!/bin/bash
# Round 5, call 51: how much of the VO append is the FP64 triangulation -- a diagnostic timing
# build without it (lib/libpicp_amd_notri.so, VO_DIAG_NOTRI: wrong positions) against the shipped
# one: rocprofv3 kernel stats of C5 and the 8e partition (append time per launch).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t51}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
for v in libpicp_amd libpicp_amd_notri; do for W in c5 c5_8e; do
  case $W in
    c5) A="--workload c5 --steps 3 --warmup 2" ;;
    c5_8e) A="--workload c5 --seg-len 1250 --steps 1 --warmup 1" ;;
  esac
  PICP_LIB=$L/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${v}_$W -o run --output-format csv -- python3 bench.py $A --no-cpu --skip-extras --samples 1 --detail - > $OUT/${v}_$W.log 2>&1 || { echo "trace $v $W failed"; tail $OUT/${v}_$W.log; exit 1; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("$OUT/${v}_$W/run_kernel_stats.csv")):
    if "append" in r["Name"] or "block_kernel" in r["Name"]: print("$v $W", r["Name"][:30], r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
  rm -f $OUT/${v}_$W/run_kernel_trace.csv
done; done
