#!/bin/bash
# PMC traffic of the default C2 kernel (picp_persistent_kernel, one launch per solve), separate
# FETCH_SIZE / WRITE_SIZE passes, at 50 rounds (the bench config) and 10 rounds: the two fix
# FETCH(R) = a + b*R, whose a is the one-time read of the 2 MB frame (calibrates the gfx950 x2
# rule for this kernel's 4-byte loads).  Then the default bench line.
set -o pipefail
mkdir -p gpurun_out
WL=c2 KERNEL=picp_persistent_kernel EXTRA="--stream-n 0" bash tools/gpu_pmc.sh > gpurun_out/pmc_c2p.log 2>&1 || { echo pmc failed; tail -20 gpurun_out/pmc_c2p.log; exit 1; }
mkdir -p gpurun_out/pmc50 && cp gpurun_out/pmc/c2_*.json gpurun_out/pmc/c2_trace/run_kernel_stats.csv gpurun_out/pmc50/
WL=c2 KERNEL=picp_persistent_kernel EXTRA="--stream-n 0 --rounds 10" bash tools/gpu_pmc.sh > gpurun_out/pmc_c2p_r10.log 2>&1 || { echo pmc r10 failed; tail -20 gpurun_out/pmc_c2p_r10.log; exit 1; }
mkdir -p gpurun_out/pmc10 && cp gpurun_out/pmc/c2_*.json gpurun_out/pmc/c2_trace/run_kernel_stats.csv gpurun_out/pmc10/
cat gpurun_out/pmc50/*.json gpurun_out/pmc10/*.json
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
