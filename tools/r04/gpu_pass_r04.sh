#!/bin/bash
# Round-4 pass at HEAD, one box: the whole GPU suite, smoke(), the batch-beside-VO concurrency
# check, the VO schedule determinism check (serial vs every concurrent schedule), the default bench
# line, and (AB_C5=1) a C5 A/B of the serial vs the concurrent VO schedule.  Each step
# time-limited; stop at the first failure.  OUT=${OUT:-gpurun_out/r04/pass}
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r04/pass}
mkdir -p $O
if [ -z "$SKIP_PYTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=8 -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u tools/concurrency_check.py > $O/concurrency_check.log 2>&1 || { echo "concurrency check failed"; tail -20 $O/concurrency_check.log; exit 1; }
grep -v "amdgpu.ids" $O/concurrency_check.log
timeout -k 10 400 python -u tools/vo_chains_check.py 2001 "PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0,PICP_VO_SPLIT=0" "PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0" "PICP_VO_OVERLAP=1" "PICP_VO_CHAINS=2" "PICP_VO_OVERLAP=1,PICP_VO_CHAINS=2" > $O/vo_chains_check.log 2>&1 || { echo "vo chains check failed"; tail -20 $O/vo_chains_check.log; exit 1; }
grep -v "amdgpu.ids" $O/vo_chains_check.log
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-400
if [ -n "$AB_C5" ]; then for rep in 1 2; do
  for S in "PICP_VO_CHAINS=1 PICP_VO_OVERLAP=0" "PICP_VO_CHAINS=2 PICP_VO_OVERLAP=1"; do
    env $S timeout -k 10 240 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu --skip-extras > $O/c5_ab.json 2> $O/c5_ab.err || { echo "c5 $S failed"; tail -5 $O/c5_ab.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/c5_ab.json').read().strip().splitlines()[-1]); print('c5 $S', round(d['value']), d['unit'], d['ms_per_step'])"
  done
done; fi
