#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamps.py --n 100000 > gpurun_out/stamps_c2.log 2>&1; echo rc=$?; cat gpurun_out/stamps_c2.log | tail -25
timeout -k 10 200 python tools/stamps.py --n 10000 --problems 256 > gpurun_out/stamps_c4.log 2>&1; echo rc=$?; cat gpurun_out/stamps_c4.log | tail -25
