#!/bin/bash
# Round 4: phase stamps at the C4 per-rank shape (128 x 10k): the block kernel at split 2 and at
# split 4 (512-thread parts, tail priority), and the pair-mode kernel.
export TMPDIR=/tmp
O=gpurun_out/stamps2; mkdir -p $O
L=$PWD/02-visualodometry_amd/lib
PICP_STAMPS_LIB=$L/libpicp_amd_stamps.so PICP_BLOCK_SPLIT=2 timeout -k 10 120 python tools/bstamps.py --problems 128 --n 10000 > $O/bst_s2.log 2>&1 || { tail $O/bst_s2.log; exit 1; }
echo "== block split 2"; cat $O/bst_s2.log
PICP_STAMPS_LIB=$L/libpicp_amd_stamps_prio.so PICP_BLOCK_SPLIT=4 timeout -k 10 120 python tools/bstamps.py --problems 128 --n 10000 > $O/bst_s4prio.log 2>&1 || { tail $O/bst_s4prio.log; exit 1; }
echo "== block split 4 prio"; cat $O/bst_s4prio.log
PICP_STAMPS_LIB=$L/libpicp_amd_stamps.so PICP_BLOCK_SPLIT=1 timeout -k 10 120 python tools/bstamps.py --problems 256 --n 10000 > $O/bst_s1_256.log 2>&1 || { tail $O/bst_s1_256.log; exit 1; }
echo "== block split 1, 256 frames"; cat $O/bst_s1_256.log
PICP_STAMPS_LIB=$L/libpicp_amd_pairstamps.so timeout -k 10 120 python tools/pair_stamps.py --problems 128 --n 10000 > $O/pair.log 2>&1 || { tail $O/pair.log; exit 1; }
echo "== pair"; cat $O/pair.log
