#!/bin/bash
# Round 6, call 30: L2 behaviour of the default-like world match (tools/r06/match_default_like.py):
# TCC hits/misses and TCP->TCC read requests, each pass its own rocprofv3 --pmc run.
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/t30}
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/tcc -o run --output-format csv -- python3 tools/r06/match_default_like.py > $OUT/tcc.log 2>&1 || { echo "pmc tcc failed"; tail -5 $OUT/tcc.log; exit 1; }
python3 tools/parse_pmc.py $(find $OUT/tcc -name '*counter_collection.csv' | head -1) picp_match_mfma > $OUT/tcc.json
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $OUT/tcp -o run --output-format csv -- python3 tools/r06/match_default_like.py > $OUT/tcp.log 2>&1 || { echo "pmc tcp failed"; tail -5 $OUT/tcp.log; exit 1; }
python3 tools/parse_pmc.py $(find $OUT/tcp -name '*counter_collection.csv' | head -1) picp_match_mfma > $OUT/tcp.json
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/r06/match_default_like.py > $OUT/fetch.log 2>&1 || { echo "pmc fetch failed"; tail -5 $OUT/fetch.log; exit 1; }
python3 tools/parse_pmc.py $(find $OUT/fetch -name '*counter_collection.csv' | head -1) picp_match_mfma > $OUT/fetch.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/tr -o run --output-format csv -- python3 tools/r06/match_default_like.py > $OUT/tr.log 2>&1 || { echo "trace failed"; exit 1; }
grep mfma $(find $OUT/tr -name '*kernel_stats.csv' | head -1) | cut -d, -f1-4 | tee $OUT/kstats.txt
python3 -c "
import json
for f in ('tcc', 'tcp', 'fetch'):
    d = json.load(open('$OUT/%s.json' % f)); print(f, {k: round(v['mean']) for k, v in d.items()})
"
