#!/bin/bash
# round-4 batch 12: the prover's GPU tests with the late-bad-wire cases.
mkdir -p gpurun_out/r4n
timeout -k 10 600 python -u -m pytest tests/test_gpu_r1cs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4n/tests.log 2>&1 || exit 1
