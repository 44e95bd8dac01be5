#!/bin/bash
# HBM traffic of the streaming round kernel (16M single frame, 320 MB per round): kernel trace,
# then FETCH_SIZE and WRITE_SIZE in SEPARATE rocprofv3 passes (MI355X_MICROARCH.md: they cannot
# share a pass; gfx950 FETCH_SIZE counts half of a wide coalesced stream -> x2).
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--no-cpu --skip-extras --steps 3 --warmup 1 --workload c2 --n ${N:-16000000} --stream-n 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc/s16m_trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/s16m_trace.log 2>&1 || { echo trace failed; tail gpurun_out/pmc/s16m_trace.log; exit 1; }
cat gpurun_out/pmc/s16m_trace/run_kernel_stats.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d gpurun_out/pmc/s16m_$C -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/s16m_$C.log 2>&1 || { echo pmc $C failed; tail gpurun_out/pmc/s16m_$C.log; exit 1; }
  python3 tools/parse_pmc.py gpurun_out/pmc/s16m_$C/run_counter_collection.csv picp_round_kernel > gpurun_out/pmc/s16m_$C.json
  cat gpurun_out/pmc/s16m_$C.json
done
