#!/bin/bash
# Round 6, call 34 (HEAD): SQ counters of the isolated 8e world match (4 problems x the whole maps,
# tools/r06/match_8e.py --fracs 1.0), two --pmc passes of 8 SQ counters, each its own run.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t34}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/r06/match_8e.py --save $OUT/maps.npz > $OUT/save.log 2>&1 || { echo "save failed"; tail $OUT/save.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/sqa -o run --output-format csv -- python3 -u tools/r06/match_8e.py --load $OUT/maps.npz --fracs 1.0 > $OUT/sqa.log 2>&1 || { echo "pmc a failed"; tail $OUT/sqa.log; exit 1; }
python3 tools/parse_pmc.py $(find $OUT/sqa -name '*counter_collection.csv' | head -1) picp_match_mfma > $OUT/sqa.json
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d $OUT/sqb -o run --output-format csv -- python3 -u tools/r06/match_8e.py --load $OUT/maps.npz --fracs 1.0 > $OUT/sqb.log 2>&1 || { echo "pmc b failed"; tail $OUT/sqb.log; exit 1; }
python3 tools/parse_pmc.py $(find $OUT/sqb -name '*counter_collection.csv' | head -1) picp_match_mfma > $OUT/sqb.json
rm -f $OUT/maps.npz
python3 -c "
import json
for f in ('$OUT/sqa.json', '$OUT/sqb.json'):
    d = json.load(open(f)); print({k: round(v['mean']) for k, v in d.items()})
"
