#!/bin/bash
# Round 6, call 36: the matcher suite with the unsafe-tile test at two row blocks per wave.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t36}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" $OUT/pytest.log | tail -30; exit 1; }
grep -E "unsafe_tiles|passed|failed" $OUT/pytest.log | tail -8
