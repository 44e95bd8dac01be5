#!/bin/bash
# Round-3 check of the TU-wide no-packed-FP32 build (hipcc_nopk.sh) against the packed A/B build
# (make abvariant AB=pk PK=1), one box:
#  1. the finish-path microbenchmark (tools/ubench/parts_ubench, cycles per piece, one wave)
#  2. the packed-FP32 victims of tools/ubench/permlane_stress alone and beside MFMA
#  3. VO schedule determinism and batch-beside-VO with each library
#  4. interleaved A/B bench of C2 / C5 with each library
# Each step time-limited; stop at the first failure.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r03/nopk_tu}
mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
timeout -k 10 60 ./tools/ubench/parts_ubench > $O/parts_ubench.log 2>&1 || { echo "parts ubench failed"; cat $O/parts_ubench.log; exit 1; }
cat $O/parts_ubench.log
for v in ${VICTIMS:-9 10 16 23}; do
  for a in 0 1; do
    timeout -k 5 60 ./tools/ubench/permlane_stress $v $a ${ITERS:-2000} >> $O/stress.log 2>&1 || { echo "stress $v $a failed"; tail -3 $O/stress.log; exit 1; }
  done
done
cat $O/stress.log
for lib in libpicp_amd.so libpicp_amd_pk.so; do
  PICP_LIB=$L/$lib timeout -k 10 400 python -u tools/vo_chains_check.py 2001 "PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0" "PICP_VO_OVERLAP=1" "PICP_VO_CHAINS=2" "PICP_VO_OVERLAP=1,PICP_VO_CHAINS=2" > $O/vo_chains_$lib.log 2>&1 || { echo "vo chains $lib failed"; tail -20 $O/vo_chains_$lib.log; exit 1; }
  echo "== vo chains $lib"; grep -v "amdgpu.ids" $O/vo_chains_$lib.log
  PICP_LIB=$L/$lib timeout -k 10 400 python -u tools/concurrency_check.py > $O/conc_$lib.log 2>&1 || { echo "conc $lib failed"; tail -20 $O/conc_$lib.log; exit 1; }
  echo "== concurrency $lib"; grep -v "amdgpu.ids\|beside:\|residency" $O/conc_$lib.log
done
for rep in 1 2; do
  for lib in libpicp_amd.so libpicp_amd_pk.so; do
    for wl in c2 c5; do
      PICP_LIB=$L/$lib timeout -k 10 240 python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu --skip-extras > $O/ab.json 2> $O/ab.err || { echo "$wl $lib failed"; tail -5 $O/ab.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('$wl $lib', round(d['value']), d['unit'], d['ms_per_step'])"
    done
  done
done
