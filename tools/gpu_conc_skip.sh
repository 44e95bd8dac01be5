#!/bin/bash
# Which VO kernel kind perturbs a block-mode batch beside it (tools/conc_skip.py per PICP_VO_DIAG_SKIP value).
export TMPDIR=/tmp
mkdir -p gpurun_out/cs
for sk in 0 4 2 6 1 5 8; do
  PICP_VO_DIAG_SKIP=$sk timeout -k 10 120 python -u tools/conc_skip.py >> gpurun_out/cs/log 2>&1 || { echo "skip $sk failed"; tail -5 gpurun_out/cs/log; exit 1; }
done
grep skip= gpurun_out/cs/log
