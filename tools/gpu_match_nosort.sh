#!/bin/bash
# matcher without the candidate sort (lib v1) vs before (v0): matcher + VO tests on v1 with the
# row blocks forced 1, 2 and adaptive, then kernel traces and C5 interleaved
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/02-visualodometry_amd/lib
for rb in 1 2 auto; do
  if [ $rb = auto ]; then unset PICP_MATCH_RB; else export PICP_MATCH_RB=$rb; fi
  PICP_LIB=$L/libpicp_amd_v1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_vo.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_ns_$rb.log 2>&1
  rc=$?; echo "rb=$rb $(tail -1 gpurun_out/pt_ns_$rb.log)"; [ $rc -eq 0 ] || exit 1
done
unset PICP_MATCH_RB
bash tools/gpu_match_rb.sh 2>&1 | tail -8
