#!/bin/bash
# Round 3: (1) which packed-FP32 instruction form gives lanes 48-63 other bits beside MFMA work
# (tools/ubench/permlane_stress victims 11-22, each beside the MFMA aggressor and alone);
# (2) C5 interleaved A/B of the serial vs the concurrent VO schedule with the no-packed build;
# (3) the default bench line.  Each step time-limited; stop at the first failure.
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r03/f}
mkdir -p $O
for v in ${VICTIMS:-11 12 13 14 15 17 18 19 20 21 22}; do
  for a in 1 0; do
    timeout -k 5 60 ./tools/ubench/permlane_stress $v $a ${ITERS:-2000} >> $O/stress.log 2>&1 || { echo "stress $v $a failed"; tail -3 $O/stress.log; exit 1; }
  done
done
cat $O/stress.log
for rep in 1 2 3; do
  for S in "PICP_VO_CHAINS=1 PICP_VO_OVERLAP=0" "PICP_VO_CHAINS=2 PICP_VO_OVERLAP=1"; do
    env $S timeout -k 10 240 python bench.py --workload c5 --steps 10 --warmup 3 --samples 3 --no-cpu --skip-extras > $O/c5_ab.json 2> $O/c5_ab.err || { echo "c5 $S failed"; tail -5 $O/c5_ab.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c5_ab.json').read().strip().splitlines()[-1]); print('c5 $S', round(d['value']), d['unit'], d['ms_per_step'], d['timing']['values'])"
  done
done
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-300
