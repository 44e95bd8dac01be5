#!/bin/bash
# block-kernel phase stamps: C5-like (250 x 2000, one block per frame) and C4 (128 x 10k, split 2)
mkdir -p gpurun_out
timeout -k 10 200 python tools/bstamps.py --problems 250 --n 2000 > gpurun_out/bstamps_c5.log 2>&1 || { tail gpurun_out/bstamps_c5.log; exit 1; }
cat gpurun_out/bstamps_c5.log
timeout -k 10 200 python tools/bstamps.py --problems 250 --n 1000 > gpurun_out/bstamps_c5b.log 2>&1 || { tail gpurun_out/bstamps_c5b.log; exit 1; }
cat gpurun_out/bstamps_c5b.log
timeout -k 10 200 python tools/bstamps.py --problems 128 --n 10000 > gpurun_out/bstamps_c4.log 2>&1 || { tail gpurun_out/bstamps_c4.log; exit 1; }
cat gpurun_out/bstamps_c4.log
