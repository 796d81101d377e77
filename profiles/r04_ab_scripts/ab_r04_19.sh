#!/bin/bash
# round-4 batch 19: the world-8 prepared (DistCircuit) proof repeated, reporting which StarkProof field
# differs on a mismatch (one of five full GPU runs gave a wrong digest for test_prove_distributed_synth_2_20
# [8-True]).
mkdir -p gpurun_out/r4v
(while true; do date > gpurun_out/r4v/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 700 python -u tools/diag_dprove.py 8 8 1 > gpurun_out/r4v/diag.log 2>&1 || exit 1
