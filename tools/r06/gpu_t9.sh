#!/bin/bash
# Round 6, call 9: the 8e world match in isolation under the kernel tracer (tools/r06/match_8e.py),
# then the two-deep tile prefetch (-DMM_PF=2, lib/libpicp_amd_pf2.so) against the shipped library
# at the 8e partition, the N = 8 per-rank shape and the default C5 shape, interleaved.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t9}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u tools/r06/match_8e.py > $OUT/trace.log 2>&1 || { echo "trace run failed"; tail $OUT/trace.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY' | tee $OUT/match_durations.txt
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "picp_match_mfma" in r["Kernel_Name"] or "merge" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-24:]:
    print(r["Kernel_Name"][:50], r["Grid_Size"], r["Workgroup_Size"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us")
PY
PICP_LIB=02-visualodometry_amd/lib/libpicp_amd_pf2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_pf2.log 2>&1 || { echo "pf2 tests failed"; tail -30 $OUT/pytest_pf2.log; exit 1; }
tail -2 $OUT/pytest_pf2.log
: > $OUT/ab.log
for rep in 1 2; do for A in "--seg-len 1250 --steps 2 --warmup 1 --samples 3" "--frames 1281" ""; do for v in base pf2; do
  L=02-visualodometry_amd/lib/libpicp_amd.so; [ $v = pf2 ] && L=02-visualodometry_amd/lib/libpicp_amd_pf2.so
  PICP_LIB=$L timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 [$A]', '$v', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done; done
