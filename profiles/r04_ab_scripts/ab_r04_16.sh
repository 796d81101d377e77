#!/bin/bash
# round-4 batch 16: the distributed prover with the shared F0 extension and 1/Zb3 (in-tree = variants/dz.so):
# the prover / distributed GPU tests, then prove_distributed at world 2 (gloo, both ranks on the one GPU).
mkdir -p gpurun_out/r4r
(while true; do date > gpurun_out/r4r/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_dprove.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4r/tests.log 2>&1 || exit 1
STARK_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 tools/time_dprove.py 20 3 > gpurun_out/r4r/dprove_w2.log 2>&1 || exit 2
