#!/bin/bash
# SQ counters of the folded accept-only matcher (1024 x 2000 x 2000, two row blocks per wave):
# one --pmc pass (8 SQ counters), kernel trace in its own pass
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_match
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_match/trace -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > gpurun_out/pmc_match/trace.log 2>&1 || { echo trace failed; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_match/sq -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > gpurun_out/pmc_match/sq.log 2>&1 || { echo pmc failed; tail -5 gpurun_out/pmc_match/sq.log; exit 1; }
python3 tools/parse_pmc.py gpurun_out/pmc_match/sq/run_counter_collection.csv picp_match_mfma > gpurun_out/pmc_match/sq.json
cat gpurun_out/pmc_match/sq.json | python3 -c "import json,sys; d=json.load(sys.stdin); print({k:round(v['mean']) for k,v in d.items()})"
grep mfma gpurun_out/pmc_match/trace/run_kernel_stats.csv | cut -c1-200
