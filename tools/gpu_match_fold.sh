#!/bin/bash
# matcher accept-only A/B (compare vs folded radius test): kernel trace, matcher + VO tests, C5
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/prof_x -o run --output-format csv -- python3 tools/match_ab.py 64 2000 8000 "PICP_MATCH_ACCEPT_ONLY=1,PICP_MATCH_NO_FOLD=1;PICP_MATCH_ACCEPT_ONLY=1" > gpurun_out/prof_x.log 2>&1 || exit 1
python3 -c "
import csv
for x in csv.DictReader(open('gpurun_out/prof_x/run_kernel_trace.csv')):
    if 'mfma' in x['Kernel_Name']: print(x['Kernel_Name'][:45], int(x['End_Timestamp'])-int(x['Start_Timestamp']))
"
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_match.log 2>&1
rc=$?; tail -2 gpurun_out/pt_match.log; [ $rc -eq 0 ] || exit 1
for x in 1 0; do
  PICP_MATCH_NO_FOLD=$x timeout -k 10 300 python bench.py --workload c5 --no-cpu --steps 5 --warmup 2 > gpurun_out/c5_nf$x.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/c5_nf$x.log').read().strip().splitlines()[-1]); print('nofold=$x', d['value'], d['ms_per_step'])"
done
