#!/bin/bash
# Round 5, call 9: dump segment 0 of the 8e partition twice (determinism check; CPU re-runs of its
# steps read the dump).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t9}
mkdir -p $OUT
timeout -k 10 300 python -u tools/r05/vo_dump.py $OUT/seg8e_a.npz && \
timeout -k 10 300 python -u tools/r05/vo_dump.py $OUT/seg8e_b.npz && \
python - <<PY
import numpy as np
a, b = np.load("$OUT/seg8e_a.npz"), np.load("$OUT/seg8e_b.npz")
for k in a.files:
    print(k, "identical" if np.array_equal(a[k], b[k]) else "DIFFERS")
PY
rm -f $OUT/seg8e_b.npz
