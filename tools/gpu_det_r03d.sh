#!/bin/bash
# Round-3 fix check, one box: the VO schedules with the shipped (no packed FP32) library and with
# the packed A/B build, the batch-beside-VO concurrency check, then the packed vs scalar A/B bench.
export TMPDIR=/tmp
OUT=gpurun_out/r03/${TAG:-fix}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
for lib in libpicp_amd.so libpicp_amd_pk.so; do
  PICP_LIB=$L/$lib timeout -k 10 300 python -u tools/bdiag_vo.py 2001 "PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0" "PICP_VO_OVERLAP=1" "PICP_VO_CHAINS=2" "PICP_VO_OVERLAP=1,PICP_VO_CHAINS=2" > $OUT/vo_$lib.log 2>&1 || { echo "vo $lib failed"; tail $OUT/vo_$lib.log; exit 1; }
  echo "== $lib"; grep "rep" $OUT/vo_$lib.log | sed 's/; lane disagreement records 0; reduction mismatch records 0//'
done
timeout -k 10 300 python -u tools/concurrency_check.py > $OUT/conc.log 2>&1 || { echo "conc failed"; tail $OUT/conc.log; exit 1; }
grep -v "beside:\|residency\|amdgpu.ids" $OUT/conc.log
