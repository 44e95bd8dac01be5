#!/bin/bash
# Persistent-mode block-count sweep at C2 (100k): fan-in bytes vs per-block linearize work.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python tools/sweep.py --n 100000 --env PICP_PERSIST_BLOCKS --ipb 256,196,128,98,64,49 --reps 20 --interleave 3 > gpurun_out/sweep_pblocks.log 2>&1
timeout -k 10 200 python tools/sweep.py --n 1000000 --outlier 0.3 --env PICP_PERSIST_BLOCKS --ipb 256,196,128 --reps 20 --interleave 3 >> gpurun_out/sweep_pblocks.log 2>&1
