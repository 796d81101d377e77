# distributed prover: A chain beside the coset LDE; dprove/distributed/streams GPU tests, then the N = 8 gloo rehearsal
set -e
mkdir -p gpurun_out/r05q
timeout -k 10 600 python -u -m pytest tests/test_gpu_dprove.py tests/test_gpu_distributed.py tests/test_gpu_streams.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05q/tests.log 2>&1
STARK_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 8 --steps 3 --warmup 1 > gpurun_out/r05q/bench_gloo8.json 2> gpurun_out/r05q/bench_gloo8.err
echo ok
