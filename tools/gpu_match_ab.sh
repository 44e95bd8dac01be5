#!/bin/bash
# A/B of matcher builds on C5 (2000 frames): lib/libpicp_amd_v*.so via PICP_LIB, interleaved.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/match_ab.log
for rep in 1 2; do
  for v in ${VARIANTS:-0 1 2}; do
    PICP_LIB=$PWD/02-visualodometry_amd/lib/libpicp_amd_v$v.so timeout -k 10 200 python bench.py --workload c5 --frames ${FRAMES:-2000} --no-cpu --steps 10 --warmup 2 > gpurun_out/ab_$v.log 2>&1 || { echo "v$v failed"; tail gpurun_out/ab_$v.log; exit 1; }
    echo "v$v $(tail -1 gpurun_out/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/match_ab.log
  done
done
