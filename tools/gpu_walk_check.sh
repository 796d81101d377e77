#!/bin/bash
# The split record walk on the GPU box's host share: the harness's timing, then the r1cs/verify GPU tests,
# the cold 2^20-step proof's host phases and the verifier's.
set -e
mkdir -p gpurun_out/w
make -s -C tests/host_walk walk_check
timeout -k 10 120 tests/host_walk/walk_check bench > gpurun_out/w/walk_bench.txt 2>&1
timeout -k 10 120 tests/host_walk/walk_check check 2 >> gpurun_out/w/walk_bench.txt 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_verify.py tests/test_gpu_r1cs.py tests/test_gpu_group.py tests/test_gpu_dprove.py tests/test_gpu_streams.py tests/test_abi_client.py > gpurun_out/w/tests.log 2>&1
STARK_PROFILE=1 timeout -k 10 180 python tools/time_r1cs.py --fixtures "" --synth 20 --reps 6 > gpurun_out/w/phases.log 2>&1
STARK_PROFILE=1 timeout -k 10 200 python -u tools/verify_phases.py synth20 4 > gpurun_out/w/vphase.log 2>&1
