#!/bin/bash
# persistent-kernel phase stamps (diagnostic stamp build): C2 (100k) and C3 (1M, 30 % outliers)
OUT=${OUT:-gpurun_out/pst}
mkdir -p $OUT
timeout -k 10 200 python tools/pstamps.py --n 100000 > $OUT/pstamps_c2.log 2>&1 || { tail $OUT/pstamps_c2.log; exit 1; }
cat $OUT/pstamps_c2.log
timeout -k 10 200 python tools/pstamps.py --n 1000000 --outlier 0.3 > $OUT/pstamps_c3.log 2>&1 || { tail $OUT/pstamps_c3.log; exit 1; }
cat $OUT/pstamps_c3.log
