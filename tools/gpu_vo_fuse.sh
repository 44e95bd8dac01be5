#!/bin/bash
# The VO step's gather fused into the PICP block kernel (PICP_VO_FUSE, default 1): the VO GPU tests
# (fused vs separate gather bit for bit included), the 2001-frame schedule check with the separate
# gather as the reference, then C5 interleaved, three repetitions.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/fuse}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_vo.py -x -v --timeout 240 --timeout-method thread > $O/pytest_vo.log 2>&1
rc=$?; tail -3 $O/pytest_vo.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_vo.log | head -20; exit 1; }
timeout -k 10 400 python -u tools/vo_chains_check.py 2001 "PICP_VO_FUSE=0,PICP_VO_CHAINS=1,PICP_VO_OVERLAP=0" "PICP_VO_FUSE=1" "PICP_VO_OVERLAP=1,PICP_VO_CHAINS=2" > $O/vo_chains_fuse.log 2>&1 || { echo "chains check failed"; tail -20 $O/vo_chains_fuse.log; exit 1; }
grep -v amdgpu.ids $O/vo_chains_fuse.log
: > $O/ab_c5.log
for rep in 1 2 3; do
  for f in 0 1; do
    PICP_VO_FUSE=$f timeout -k 10 240 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu --skip-extras > $O/c5.json 2> $O/c5.err || { echo "c5 fuse=$f failed"; tail -5 $O/c5.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]); print('fuse=$f', round(d['value']), d['unit'], d['ms_per_step'])" | tee -a $O/ab_c5.log
  done
done
