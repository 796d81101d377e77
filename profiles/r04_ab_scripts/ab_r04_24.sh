#!/bin/bash
# round-4 batch 24: the world-8 DistCircuit proof repeated with the parent holding a GPU context (as pytest's
# session context does), current library then the round's morning library (fin4): is the intermittent
# wrong digest new?
mkdir -p gpurun_out/r4aa
(while true; do date > gpurun_out/r4aa/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
DIAG_PARENT_GPU=1 timeout -k 10 500 python -u tools/diag_dprove.py 8 12 1 > gpurun_out/r4aa/diag_cur.log 2>&1 || exit 1
STARK_LIB=$PWD/variants/fin4.so DIAG_PARENT_GPU=1 timeout -k 10 500 python -u tools/diag_dprove.py 8 12 1 > gpurun_out/r4aa/diag_fin4.log 2>&1 || exit 2
