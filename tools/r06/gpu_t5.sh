#!/bin/bash
# Round 6, call 5: is the VO append bound by co-residency with the matcher's blocks?  Diagnostic
# builds (wrong maps): the append without its triangulation at 512 threads (74 VGPRs; two waves
# per SIMD do not fit beside four matcher waves) and at 256 threads (one wave per SIMD: fits), and
# the shipped append at 256 threads (173 VGPRs), against the shipped library, at the three C5 shapes.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t5}
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
: > $OUT/ab.log
for A in "" "--seg-len 1250 --steps 2 --warmup 1 --samples 1" "--frames 1281"; do for rep in 1 2; do for v in libpicp_amd libpicp_amd_notri512 libpicp_amd_notri256 libpicp_amd_tri256; do
  PICP_LIB=$L/$v.so timeout -k 10 300 python bench.py --workload c5 --no-cpu --skip-extras --detail - $A > $OUT/run.log 2>&1 || { echo "bench $v failed"; tail $OUT/run.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/run.log').read().strip().splitlines()[-1]); print('c5 $A', '$v', d['value'], d.get('chain_step_us'))" | tee -a $OUT/ab.log
done; done; done
