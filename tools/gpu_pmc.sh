#!/bin/bash
# HBM traffic counters for the round kernel: FETCH_SIZE and WRITE_SIZE in SEPARATE passes
# (MI355X_MICROARCH.md: they cannot share a pass), kernel-trace/stats in its own pass.
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
WL=${WL:-c2}
ARGS="--no-cpu --skip-extras --steps 5 --warmup 1 --workload $WL ${EXTRA:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc/${WL}_trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/${WL}_trace.log 2>&1 || { echo trace failed; tail gpurun_out/pmc/${WL}_trace.log; exit 1; }
tail -1 gpurun_out/pmc/${WL}_trace.log
cat gpurun_out/pmc/${WL}_trace/run_kernel_stats.csv
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d gpurun_out/pmc/${WL}_$C -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/${WL}_$C.log 2>&1 || { echo pmc $C failed; tail gpurun_out/pmc/${WL}_$C.log; exit 1; }
  python3 tools/parse_pmc.py gpurun_out/pmc/${WL}_$C/run_counter_collection.csv ${KERNEL:-picp_} > gpurun_out/pmc/${WL}_$C.json
  cat gpurun_out/pmc/${WL}_$C.json
done
