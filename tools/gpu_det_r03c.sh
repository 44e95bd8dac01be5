#!/bin/bash
# Round-3 determinism probe, one box: per-step PICP snapshots of the VO schedules (diagnostic VO
# runtime, shipped block kernel), then the block-kernel variants of tools/gpu_det_r03b.sh.
export TMPDIR=/tmp
OUT=gpurun_out/r03/${TAG:-detc}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
PICP_LIB=$L/libpicp_amd_vodiag.so timeout -k 10 300 python -u tools/vo_snap.py 2001 > $OUT/vo_snap.log 2>&1 || { echo "vo_snap failed"; tail $OUT/vo_snap.log; exit 1; }
cat $OUT/vo_snap.log
for lib in ${LIBS:-libpicp_amd.so}; do
  PICP_LIB=$L/$lib timeout -k 10 300 python -u tools/bdiag_vo.py 2001 > $OUT/vo_$lib.log 2>&1 || { echo "$lib failed"; tail $OUT/vo_$lib.log; exit 1; }
  echo "== $lib"; grep -v "^  records identical" $OUT/vo_$lib.log | grep -v "CHAINS=1,PICP_VO_OVERLAP=0 rep" | sed 's/; lane disagreement records 0; reduction mismatch records 0//' | head -40
done
