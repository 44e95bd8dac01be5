#!/bin/bash
# Round 6, call 17: kernel trace of the 8e partition with the split world match (early part after
# the step's merge): per-stream timeline and the raw launch order of a 1.5 ms window.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t17}
mkdir -p $OUT
for v in 1; do
  PICP_VO_SPLIT=$v timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/tr$v -o run --output-format csv -- python3 bench.py --workload c5 --no-cpu --skip-extras --seg-len 1250 --steps 1 --warmup 1 --samples 1 > $OUT/tr$v.log 2>&1 || { echo "trace failed"; tail $OUT/tr$v.log; exit 1; }
  f=$(find $OUT/tr$v -name '*kernel_trace.csv' | head -1)
  python3 tools/vo_timeline.py $f 20 > $OUT/timeline_split$v.txt
  python3 - "$f" > $OUT/window_split$v.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
t_end = max(int(r["End_Timestamp"]) for r in rows)
w0 = t_end - 30_000_000
sel = [r for r in rows if w0 <= int(r["Start_Timestamp"]) < w0 + 1_500_000]
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%9.1f %7.1f  stream %s  %s" % ((s - w0) / 1e3, (e - s) / 1e3, r.get("Stream_Id"), r["Kernel_Name"][:48]))
PY
done
cat $OUT/timeline_split1.txt; head -40 $OUT/window_split1.txt
