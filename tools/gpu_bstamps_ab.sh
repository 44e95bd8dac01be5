#!/bin/bash
# block-kernel phase stamps for two stamp builds (lib/libpicp_amd_stamps_{A,B}.so), C5-like and C4
OUT=${OUT:-gpurun_out/bst}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
for cfg in "250 2000" "1024 10000"; do set -- $cfg; for v in ${VARS:-c1 new}; do
  PICP_STAMPS_LIB=$L/libpicp_amd_stamps_$v.so timeout -k 10 200 python tools/bstamps.py --problems $1 --n $2 > $OUT/bst_${v}_$1.log 2>&1 || { tail $OUT/bst_${v}_$1.log; exit 1; }
  echo "== $v $1x$2"; tail -3 $OUT/bst_${v}_$1.log
done; done
