#!/bin/bash
# A/B of two VO builds lib/libpicp_amd_v{0,1}.so: the VO GPU tests on v1, bit identity of every
# bench workload's poses (tools/pose_dump.py), then C5 interleaved, three repetitions.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/abvo}
mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
PICP_LIB=$L/libpicp_amd_v1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_vo.py -x -q --timeout 240 --timeout-method thread > $O/pytest_vo.log 2>&1
rc=$?; tail -2 $O/pytest_vo.log; [ $rc -eq 0 ] || exit 1
for v in 0 1; do PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 200 python tools/pose_dump.py dump $O/p$v.npz > $O/dump$v.log 2>&1 || { echo "dump $v failed"; tail $O/dump$v.log; exit 1; }; done
timeout -k 10 60 python tools/pose_dump.py cmp $O/p0.npz $O/p1.npz | tee $O/cmp.log
: > $O/ab_c5.log
for rep in 1 2 3; do
  for v in 0 1; do
    PICP_LIB=$L/libpicp_amd_v$v.so timeout -k 10 240 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu --skip-extras > $O/c5.json 2> $O/c5.err || { echo "c5 v$v failed"; tail -5 $O/c5.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]); print('v$v', round(d['value']), d['unit'], d['ms_per_step'])" | tee -a $O/ab_c5.log
  done
done
