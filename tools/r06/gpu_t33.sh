#!/bin/bash
# Round 6, call 33: the matcher's tile-loop phases at HEAD (one barrier per tile), -DMM_TSTAMP build.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t33}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/r06/match_8e.py --save $OUT/maps.npz > $OUT/save.log 2>&1 || { echo "save failed"; tail $OUT/save.log; exit 1; }
PICP_LIB=02-visualodometry_amd/lib/libpicp_amd_tstamp.so timeout -k 10 300 python3 -u tools/r06/match_tstamp.py $OUT/maps.npz > $OUT/tstamp.txt 2>&1 || { echo "tstamp failed"; tail $OUT/tstamp.txt; exit 1; }
cat $OUT/tstamp.txt
rm -f $OUT/maps.npz
