#!/bin/bash
# The tightened n_in parity tests, then the stale-state probe (tools/poison_check.py).
# Each GPU step time-limited; the probe runs only if pytest ended normally (pass or assertion).
export TMPDIR=/tmp
O=gpurun_out/poison
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -v --timeout 240 --timeout-method thread -k "ragged or streaming or block_split or c4_full or solve or persistent" > $O/pytest_nin.log 2>&1
rc=$?
tail -15 $O/pytest_nin.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
[ -n "$SKIP_POISON" ] && exit $rc; timeout -k 10 300 python -u tools/poison_check.py > $O/poison_check.log 2>&1
rc2=$?
cat $O/poison_check.log | tail -20
exit $(( rc > rc2 ? rc : rc2 ))
