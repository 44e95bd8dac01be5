#!/bin/bash
# Round 4 end pass at HEAD, one box: the whole GPU suite, smoke(), the batch-beside-VO concurrency
# check, the VO schedule determinism check, and the default bench line.  Each step time-limited;
# stop at the first failure.  OUT=${OUT:-gpurun_out/r04/final}
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r04/final}
mkdir -p $O
git_head=$(cat .git_head 2>/dev/null); echo "head ${git_head:-unknown}" > $O/head.txt
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=8 -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u tools/concurrency_check.py > $O/concurrency_check.log 2>&1 || { echo "concurrency check failed"; tail -20 $O/concurrency_check.log; exit 1; }
grep -v "amdgpu.ids" $O/concurrency_check.log | tail -8
timeout -k 10 400 python -u tools/vo_chains_check.py 2001 "PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0,PICP_VO_SPLIT=0" "PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0" "PICP_VO_OVERLAP=1" "PICP_VO_CHAINS=2" "PICP_VO_OVERLAP=1,PICP_VO_CHAINS=2" "PICP_VO_SPLIT=1" "PICP_VO_FUSE=2" > $O/vo_chains_check.log 2>&1 || { echo "vo chains check failed"; tail -20 $O/vo_chains_check.log; exit 1; }
grep -v "amdgpu.ids" $O/vo_chains_check.log | tail -10
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('c2', d['value'], d['ms_per_step'], 'oracle', d.get('pose_err_vs_oracle_se3'))
print('c4', d['c4']['value'], json.dumps(d['c4'].get('projection')))
print('c3', d['c3']['value'], d['c3'].get('pose_err_vs_oracle_se3'))
c5=d['c5']; print('c5', c5['value'], c5.get('chain_step_us'), json.dumps(c5.get('trajectory')))
print('c5 8e', c5['partition_8e']['value'], c5['partition_8e'].get('chain_step_us'), json.dumps(c5['partition_8e'].get('trajectory')))
print('c5 n8', json.dumps(c5.get('projection_n8')))
"
