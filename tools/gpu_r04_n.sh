#!/bin/bash
# Round-4 final build (conf load ordering): bit-identity against tools/ab/lib_prev.so, then
# the measurement set (tools/gpu_r04_final.sh) into gpurun_out/r04n.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
PREV=$PWD/tools/ab/lib_prev.so
ONEPOSE_LIB=$PREV timeout -k 10 300 python tools/bitcmp.py dump $O/prev.npz > $O/dump_prev.log 2>&1 || { tail -20 $O/dump_prev.log; exit 1; }
timeout -k 10 300 python tools/bitcmp.py dump $O/new.npz > $O/dump_new.log 2>&1 || { tail -20 $O/dump_new.log; exit 1; }
python tools/bitcmp.py cmp $O/prev.npz $O/new.npz > $O/cmp.log 2>&1
rc=$?; tail -2 $O/cmp.log; rm -f $O/*.npz
[ $rc -ne 0 ] && exit 1
OUT=r04n bash tools/gpu_r04_final.sh
