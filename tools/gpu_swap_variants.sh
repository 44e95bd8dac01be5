#!/bin/bash
# Which wave-reduction build is bit-stable under the concurrent VO schedule, and what does it cost?
# For each library in LIBS: the 1,201-frame determinism check (serial vs concurrent), then C2/C4/C5.
export TMPDIR=/tmp
L=$PWD/02-visualodometry_amd/lib
mkdir -p gpurun_out/sv
: > gpurun_out/sv/summary.log
for v in ${LIBS}; do
  PICP_LIB=$L/$v.so OUT=gpurun_out/sv/$v FRAMES=1201:1200:5 SETTINGS="dummy=1 PICP_VO_OVERLAP=1,PICP_VO_CHAINS=2 PICP_VO_CHAINS=2" bash tools/gpu_vo_chains.sh > gpurun_out/sv/$v.chk 2>&1 || { echo "$v check failed"; tail gpurun_out/sv/$v.chk; exit 1; }
  grep "^setting" gpurun_out/sv/$v.chk | sed "s/^/$v /" | tee -a gpurun_out/sv/summary.log
  for W in c2 c4 c5; do
    PICP_LIB=$L/$v.so timeout -k 10 200 python bench.py --workload $W --no-cpu --skip-extras --steps 10 > gpurun_out/sv/run.log 2>&1 || { echo "bench $v $W failed"; tail gpurun_out/sv/run.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/sv/run.log').read().strip().splitlines()[-1]); print('$v', '$W', d['value'], d.get('pose_err_vs_gt_se3', d.get('pose_err_vs_gt_se3_max')))" | tee -a gpurun_out/sv/summary.log
  done
done
