#!/bin/bash
# Round-2 end pass: the GPU suite, the default bench line, rocprofv3 kernel stats of each
# workload and the FETCH_SIZE / WRITE_SIZE PMC passes the bench line cites (tools/gpu_prof_r02.sh).
export TMPDIR=/tmp
O=gpurun_out/r02end5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_default.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_default.log').read().strip().splitlines()[-1]); print('c2', d['value'], 'c3', d['c3']['value'], 'c4', d['c4']['value'], 'c5', d['c5']['value'])"
bash tools/gpu_prof_r02.sh
