#!/bin/bash
# matcher time decomposition: kernel traces of one accept-only 1024 x 2000 x 2000 batch (half of
# the queries with an exact match, half the references duplicated) for the shipped build and the
# diagnostic timing builds (no candidate extraction / no rescan / no vote: wrong results, timing only).
# Build them first, in 02-visualodometry_amd/, per variant V in NOCAND NORESCAN "NOCAND -DMM_DIAG_NORESCAN"
# "NOVOTE -DMM_DIAG_NORESCAN": hipcc ... -DMM_DIAG_$V -c csrc/picp_match.hip, then link it with the other
# build/*.o objects into lib/libpicp_amd_d_<v>.so (the Makefile's $(LIB) rule with that object).
export TMPDIR=/tmp
OUT=gpurun_out/mdiag
mkdir -p $OUT
L=$PWD/02-visualodometry_amd/lib
for v in libpicp_amd libpicp_amd_d_nocand libpicp_amd_d_norescan libpicp_amd_d_nocanddmm_diag_norescan libpicp_amd_d_novotedmm_diag_norescan; do
  MATCH_DUP=0.5 PICP_LIB=$L/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/tr_$v -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/tr_$v.log 2>&1 || { echo "trace $v failed"; tail $OUT/tr_$v.log; exit 1; }
  echo "$v $(grep mfma $OUT/tr_$v/run_kernel_stats.csv | cut -d, -f2-4)"
done
