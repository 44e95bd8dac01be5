#!/bin/bash
# Does the append's FP64 triangulation perturb a block-mode batch beside the VO?  tools/conc_skip.py
# with the shipped library and with a diagnostic build whose append skips the triangulation.
export TMPDIR=/tmp
mkdir -p gpurun_out/cn
L=$PWD/02-visualodometry_amd/lib
for v in libpicp_amd libpicp_amd_notri libpicp_amd libpicp_amd_notri; do
  PICP_LIB=$L/$v.so timeout -k 10 120 python -u tools/conc_skip.py > gpurun_out/cn/run.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/cn/run.log; exit 1; }
  echo "$v $(grep skip= gpurun_out/cn/run.log)" | tee -a gpurun_out/cn/log
done
