#!/bin/bash
# Round-3 determinism probe, one box: the VO schedule comparison with the shipped library (poses
# only: the control), then with the diagnostic block-kernel builds (per-round records).
export TMPDIR=/tmp
OUT=gpurun_out/r03/${TAG:-detb}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
for lib in libpicp_amd.so ${LIBS:-libpicp_amd_bdiag_nochk.so}; do
  PICP_LIB=$L/$lib timeout -k 10 300 python -u tools/bdiag_vo.py 2001 > $OUT/vo_$lib.log 2>&1 || { echo "$lib failed"; tail $OUT/vo_$lib.log; exit 1; }
  echo "== $lib"; grep -v "^  records identical" $OUT/vo_$lib.log | head -40
done
