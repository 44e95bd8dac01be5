export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vo.py -x -q -k "block or batch or uniform or vo" --timeout 300 --timeout-method thread > gpurun_out/pt_b.log 2>&1; rc=$?; tail -2 gpurun_out/pt_b.log; [ $rc -eq 0 ] || exit 1
for w in c4 c5; do timeout -k 10 300 python bench.py --workload $w --no-cpu > gpurun_out/b_$w.log 2>&1 || exit 1; python -c "import json; d=json.loads(open('gpurun_out/b_$w.log').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'])"; done
