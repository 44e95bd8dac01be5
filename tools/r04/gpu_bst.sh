#!/bin/bash
# Round 4: block-kernel phase stamps + placement at the C4 per-rank shape (128 x 10k)
export TMPDIR=/tmp
O=gpurun_out/bst; mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
for v in stamps stamps_prio; do for sp in 2 4; do
  PICP_STAMPS_LIB=$L/libpicp_amd_$v.so PICP_BLOCK_SPLIT=$sp timeout -k 10 120 python tools/bstamps.py --problems 128 --n 10000 > $O/${v}_s$sp.log 2>&1 || { tail $O/${v}_s$sp.log; exit 1; }
  echo "== $v split $sp"; cat $O/${v}_s$sp.log
done; done
