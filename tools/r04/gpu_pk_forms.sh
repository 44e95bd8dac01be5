#!/bin/bash
# Round 4: the packed form pk_bisect.py isolated, as inline asm (permlane_stress victims 24-27),
# beside the MFMA aggressor and alone; victim 9 (the compiler's apply_update) and 23 (no packed)
# for reference.
export TMPDIR=/tmp
O=gpurun_out/pkforms; mkdir -p $O
: > $O/stress.log
for v in 9 23 24 25 26 27 12; do
  for a in 1 0; do
    timeout -k 5 60 ./tools/ubench/permlane_stress $v $a 2000 >> $O/stress.log 2>&1 || { echo "stress $v $a failed"; tail -3 $O/stress.log; exit 1; }
  done
done
cat $O/stress.log
