#!/bin/bash
# the default bench line alone (OUT=gpurun_out/r04/bench)
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r04/bench}
mkdir -p $O
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('c2', d['value'], d['ms_per_step'], 'oracle', d.get('pose_err_vs_oracle_se3'))
print('c4', d['c4']['value'], json.dumps(d['c4'].get('projection')))
print('c3', d['c3']['value'], d['c3'].get('pose_err_vs_oracle_se3'))
c5=d['c5']; print('c5', c5['value'], c5.get('chain_step_us'), json.dumps(c5.get('trajectory')))
print('c5 8e', c5['partition_8e']['value'], c5['partition_8e'].get('chain_step_us'), json.dumps(c5['partition_8e'].get('trajectory')))
print('c5 n8', json.dumps(c5.get('projection_n8')))
"
