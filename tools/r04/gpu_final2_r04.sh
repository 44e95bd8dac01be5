#!/bin/bash
# Round 4 end pass after the exchange batching, one box: the GPU suite, smoke(), the concurrency
# and VO-schedule checks, then the default bench line and the kernel traces beside it
# (gpu_final_same_box.sh).  OUT=${OUT:-gpurun_out/r04/final2}
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r04/final2}
mkdir -p $O
git_head=$(cat .git_head 2>/dev/null); echo "head ${git_head:-unknown}" > $O/head.txt
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=8 -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u tools/concurrency_check.py > $O/concurrency_check.log 2>&1 || { echo "concurrency check failed"; tail -20 $O/concurrency_check.log; exit 1; }
grep -v "amdgpu.ids" $O/concurrency_check.log | tail -8
timeout -k 10 400 python -u tools/vo_chains_check.py 2001 "PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0,PICP_VO_SPLIT=0" "PICP_VO_OVERLAP=1,PICP_VO_CHAINS=2" "PICP_VO_SPLIT=1" "PICP_VO_FUSE=2" > $O/vo_chains_check.log 2>&1 || { echo "vo chains check failed"; tail -20 $O/vo_chains_check.log; exit 1; }
grep -v "amdgpu.ids" $O/vo_chains_check.log | tail -6
OUT=$O bash tools/r04/gpu_final_same_box.sh
