#!/bin/bash
# round-4 batch 27: the sequence that gave the second wrong world-8 digest (test_gpu_r1cs, test_gpu_verify,
# test_gpu_dprove), twice, with the test now naming the differing StarkProof fields on a mismatch.
mkdir -p gpurun_out/r4ae
(while true; do date > gpurun_out/r4ae/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
for k in 1 2; do
  timeout -k 10 500 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_verify.py tests/test_gpu_dprove.py -v --timeout 300 --timeout-method thread > gpurun_out/r4ae/tests_$k.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
