#!/bin/bash
# Round 5, call 26: where the folded matcher's waves wait (1,024 x 2,000 x 2,000 accept-only, the C5
# kernel form): two SQ counter passes, each its own run.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05/t26}
mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
n=0
for P in "$P1" "$P2"; do n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$n -o run --output-format csv -- python3 tools/match_ab.py 1024 2000 2000 "PICP_MATCH_ACCEPT_ONLY=1" > $OUT/p$n.log 2>&1 || { echo "pass $n failed"; tail $OUT/p$n.log; exit 1; }
  python3 tools/parse_pmc.py $OUT/p$n/run_counter_collection.csv picp_match_mfma > $OUT/match_pmc_p$n.json
  python3 -c "import json; d=json.load(open('$OUT/match_pmc_p$n.json')); print({k: v['mean'] for k, v in d.items()})"
done
