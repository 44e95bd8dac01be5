#!/bin/bash
# Round 6: the C2 persistent kernel's FETCH_SIZE, three separate passes (the end pass read 11,060 KiB
# per launch against round 5's 2,420 KiB on an unchanged kernel; C3's pass matched round 5's), and
# one WRITE_SIZE pass.  Each pass its own rocprofv3 --pmc run (MI355X_MICROARCH.md).
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r06/pmc_c2}
mkdir -p $OUT
A="--no-cpu --skip-extras --steps 5 --warmup 1 --samples 1 --workload c2"
for i in 1 2 3; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$i -o run --output-format csv -- python3 bench.py $A > $OUT/fetch_$i.log 2>&1 || { echo "pmc $i failed"; tail $OUT/fetch_$i.log; exit 1; }
  python3 tools/parse_pmc.py $OUT/fetch_$i/run_counter_collection.csv picp_persistent > $OUT/c2_fetch_$i.json
  python3 -c "import json; d=json.load(open('$OUT/c2_fetch_$i.json')); print('c2 FETCH_SIZE pass $i', d['FETCH_SIZE'])"
done
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $A > $OUT/write.log 2>&1 || exit 1
python3 tools/parse_pmc.py $OUT/write/run_counter_collection.csv picp_persistent > $OUT/c2_write.json
python3 -c "import json; d=json.load(open('$OUT/c2_write.json')); print('c2 WRITE_SIZE', d['WRITE_SIZE'])"
