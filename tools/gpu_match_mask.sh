#!/bin/bash
# A/B of matcher builds lib/libpicp_amd_v{0,1}.so (v0: carry-chain candidate mask, v1: v_perm/v_bfi row mask):
# matcher + VO tests on the candidate build, then C5 (2000 frames) interleaved
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/02-visualodometry_amd/lib
PICP_LIB=$L/libpicp_amd_v${TESTV:-2}.so timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_match.log 2>&1
rc=$?; tail -2 gpurun_out/pt_match.log; [ $rc -eq 0 ] || exit 1
for v in ${VARIANTS:-0 2 3}; do
  for shape in ${SHAPES:-"1024 2000 2000"}; do
    tag=$(echo $shape | tr ' ' x)
    PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/pp_${v}_$tag -o run --output-format csv -- python3 tools/match_ab.py $shape "PICP_MATCH_ACCEPT_ONLY=1" > gpurun_out/pp_${v}_$tag.log 2>&1 || { echo "trace v$v failed"; tail -5 gpurun_out/pp_${v}_$tag.log; exit 1; }
    python3 -c "
import csv
t=[int(x['End_Timestamp'])-int(x['Start_Timestamp']) for x in csv.DictReader(open('gpurun_out/pp_${v}_$tag/run_kernel_trace.csv')) if 'mfma' in x['Kernel_Name']]
print('v$v $tag', t)"
  done
done
: > gpurun_out/match_ab.log
for rep in 1 2 3; do
  for v in ${VARIANTS:-0 2 3}; do
    PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 python bench.py --workload c5 --frames ${FRAMES:-10000} --no-cpu --steps 10 --warmup 2 > gpurun_out/ab_$v.log 2>&1 || { echo "v$v failed"; tail gpurun_out/ab_$v.log; exit 1; }
    echo "v$v $(tail -1 gpurun_out/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/match_ab.log
  done
done
