#!/bin/bash
# Round 5, call 25: the SQ counters this box offers (names only), for the matcher's stall breakdown.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t25}
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || timeout -k 10 120 rocprofv3 --list-avail > $OUT/counters.txt 2>&1
grep -o "SQ_[A-Z0-9_]*" $OUT/counters.txt | sort -u | tr '\n' ' ' | head -c 6000
