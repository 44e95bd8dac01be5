#!/bin/bash
# C5 with 2..4 step chains (PICP_VO_CHAINS; the library caps it at 2: lift the cap in
# picp_vo_runtime.cpp for this A/B), interleaved, two repetitions, and the schedule
# bit-identity check of 3 and 4 chains against the serial order.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/chains}
mkdir -p $O
timeout -k 10 400 python -u tools/vo_chains_check.py 2001 "PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0" "PICP_VO_CHAINS=3,PICP_VO_OVERLAP=1" "PICP_VO_CHAINS=4,PICP_VO_OVERLAP=1" > $O/vo_chains.log 2>&1 || { echo "chains check failed"; tail -20 $O/vo_chains.log; exit 1; }
grep -v amdgpu.ids $O/vo_chains.log
: > $O/ab_c5.log
for rep in 1 2; do
  for c in ${CHAINS:-2 3 4}; do
    PICP_VO_CHAINS=$c timeout -k 10 240 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu --skip-extras > $O/c5.json 2> $O/c5.err || { echo "c5 chains=$c failed"; tail -5 $O/c5.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]); print('chains=$c', round(d['value']), d['unit'], d['ms_per_step'])" | tee -a $O/ab_c5.log
  done
done
