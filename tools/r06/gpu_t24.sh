#!/bin/bash
# Round 6, call 24: the block kernel's round phases (tools/bstamps.py, stamp build) at VO-like
# shapes: 4, 16 and 125 problems of 1,500 correspondences (one block per problem, as a VO chain's
# PICP launch at the 8e, per-rank and default shapes).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t24}
mkdir -p $OUT
: > $OUT/bstamps.txt
for P in 4 16 125; do
  timeout -k 10 200 python3 -u tools/bstamps.py --problems $P --n 1500 >> $OUT/bstamps.txt 2>&1 || { echo "bstamps $P failed"; tail $OUT/bstamps.txt; exit 1; }
done
cat $OUT/bstamps.txt
