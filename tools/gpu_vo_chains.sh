#!/bin/bash
# VO scheduling: determinism across settings (tools/vo_chains_check.py), then a kernel trace of
# one C5 run under TRACE's settings.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/vo_ch}
mkdir -p $OUT
timeout -k 10 300 python -u tools/vo_chains_check.py ${FRAMES:-10000} ${SETTINGS:-"PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0" "PICP_VO_CHAINS=3"} > $OUT/check.log 2>&1 || { echo "check failed"; tail $OUT/check.log; exit 1; }
cat $OUT/check.log
if [ -n "$TRACE" ]; then
  for kv in $(echo $TRACE | tr ',' ' '); do export $kv; done
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/tr -o run --output-format csv -- python3 bench.py --workload c5 --no-cpu --skip-extras --steps 3 > $OUT/tr.log 2>&1 || { echo "trace failed"; tail $OUT/tr.log; exit 1; }
  tail -1 $OUT/tr.log | cut -c1-200
fi
