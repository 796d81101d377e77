#!/bin/bash
# round-4 GPU batch: NTT A/Bs (prefetch, 2^20 plans), the distributed/cache tests, the world-8 gloo rehearsal
mkdir -p gpurun_out/r4b
(while true; do date > gpurun_out/r4b/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
bash tools/ab_r04_1.sh || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_distributed.py tests/test_gpu_dprove.py tests/test_gpu_large.py::test_twiddle_cache_stays_under_cap tests/test_gpu_field.py tests/test_abi_client.py tests/test_gpu_r1cs.py -m gpu > gpurun_out/r4b/tests.log 2>&1 || exit 2
STARK_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 8 --steps 3 --warmup 1 > gpurun_out/r4b/bench_gloo8.json 2> gpurun_out/r4b/bench_gloo8.err || exit 3
