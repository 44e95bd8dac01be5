#!/bin/bash
# permlane_stress matrix (tools/ubench/permlane_stress.hip): every victim beside every aggressor.
OUT=gpurun_out/r03/${TAG:-permlane}
mkdir -p $OUT
for v in ${VICTIMS:-0 1 2}; do
  for a in ${AGGRS:-0 1 2 3 4 5 6 7 8}; do
    timeout -k 5 60 ./tools/ubench/permlane_stress $v $a ${ITERS:-2000} >> $OUT/matrix.log 2>&1 || { echo "victim $v aggressor $a failed rc=$?"; tail -3 $OUT/matrix.log; exit 1; }
  done
done
cat $OUT/matrix.log
