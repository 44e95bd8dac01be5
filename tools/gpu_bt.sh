#!/bin/bash
# 512- vs 1024-thread block kernel (PICP_BLOCK_THREADS): parity tests at 1024, stamps and C4/C5 A/B
mkdir -p gpurun_out
PICP_BLOCK_THREADS=1024 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vo.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_bt.log 2>&1
rc=$?; echo "pytest(1024) rc=$rc"; tail -2 gpurun_out/pt_bt.log; [ $rc -eq 0 ] || exit 1
PICP_BLOCK_THREADS=1024 timeout -k 10 200 python tools/bstamps.py --problems 128 --n 10000 > gpurun_out/bst_c4_1024.log 2>&1 && cat gpurun_out/bst_c4_1024.log || exit 1
PICP_BLOCK_THREADS=1024 timeout -k 10 200 python tools/bstamps.py --problems 250 --n 2000 > gpurun_out/bst_c5_1024.log 2>&1 && cat gpurun_out/bst_c5_1024.log || exit 1
for rep in 1 2; do for t in 512 1024; do for w in c4 c5; do
PICP_BLOCK_THREADS=$t timeout -k 10 200 python bench.py --workload $w --no-cpu --skip-extras --stream-n 0 > gpurun_out/bt_$w.log 2>&1 || { echo bench failed; tail gpurun_out/bt_$w.log; exit 1; }
python -c "import json,sys; d=json.loads(open('gpurun_out/bt_$w.log').read().strip().splitlines()[-1]); print('$t $w', d['value'], d['ms_per_step'])"
done; done; done
