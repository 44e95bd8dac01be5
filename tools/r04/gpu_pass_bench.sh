#!/bin/bash
# Round 4 pass at HEAD: the GPU suite, smoke(), and the default bench line.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r04/pass}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=8 -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('c2', d['value'], d['ms_per_step'], 'oracle', d.get('pose_err_vs_oracle_se3'))
print('c4', d['c4']['value'], d['c4'].get('projection'))
print('c3', d['c3']['value'])
c5=d['c5']; print('c5', c5['value'], c5.get('chain_step_us'), c5.get('trajectory', {}).get('ate_rmse_m'))
print('c5 8e', c5['partition_8e']['value'], c5['partition_8e'].get('trajectory', {}).get('ate_rmse_m'))
print('c5 n8', c5.get('projection_n8'))
"
