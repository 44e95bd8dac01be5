#!/bin/bash
# Round 3: persistent-kernel phase stamps, C2 and C3: staggered pose polls (default) vs one poll
# (make stamps STAMP_LIB=lib/libpicp_amd_stamps_stag0.so with -DPICP_POSE_STAGGER=0).
OUT=${OUT:-gpurun_out/r03/pst_stag}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
for lib in libpicp_amd_stamps.so libpicp_amd_stamps_stag0.so; do
  PICP_STAMPS_LIB=$L/$lib timeout -k 10 200 python tools/pstamps.py --n 100000 > $OUT/pstamps_c2_$lib.log 2>&1 || { tail $OUT/pstamps_c2_$lib.log; exit 1; }
  PICP_STAMPS_LIB=$L/$lib timeout -k 10 200 python tools/pstamps.py --n 1000000 --outlier 0.3 > $OUT/pstamps_c3_$lib.log 2>&1 || { tail $OUT/pstamps_c3_$lib.log; exit 1; }
  echo "== $lib"; cat $OUT/pstamps_c2_$lib.log $OUT/pstamps_c3_$lib.log
done
