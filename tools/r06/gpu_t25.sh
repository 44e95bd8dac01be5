#!/bin/bash
# Round 6, call 25: the VO append's phases (tools/r06/append_tstamp.py, -DVOA_TSTAMP build).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t25}
mkdir -p $OUT
PICP_LIB=02-visualodometry_amd/lib/libpicp_amd_voats.so timeout -k 10 400 python3 -u tools/r06/append_tstamp.py > $OUT/append_tstamp.txt 2>&1 || { echo "failed"; tail $OUT/append_tstamp.txt; exit 1; }
cat $OUT/append_tstamp.txt
