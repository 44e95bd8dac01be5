#!/bin/bash
# Round 5: calibrate the VALU issue basis.  tools/ubench/issue_ubench
# (built on the CPU side, shipped device flags) prints SIMD cycles per wave64 instruction for an
# independent v_fma_f32 stream and a dependent chain at 1/2/4/8 waves per SIMD, and the block
# kernel's linearize mix at 1/2/4/8 waves per SIMD; one rocprofv3 --pmc pass counts the mix
# kernels' VALU instructions per wave.  Every step time-limited; stop at the first failure.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/issue}
mkdir -p $OUT
timeout -k 10 120 ./tools/ubench/issue_ubench 4000 2000 > $OUT/issue_ubench.log 2>&1 || { echo "ubench failed"; cat $OUT/issue_ubench.log; exit 1; }
cat $OUT/issue_ubench.log
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU -d $OUT/pmc -o run --output-format csv -- ./tools/ubench/issue_ubench 400 200 > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail $OUT/pmc.log; exit 1; }
python3 tools/parse_pmc.py $OUT/pmc/run_counter_collection.csv mix > $OUT/pmc_mix.json || true
ls $OUT/pmc
