# full GPU suite + default bench on the in-tree library
set -e
mkdir -p gpurun_out/r05l
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05l/gpu_tests.log 2>&1
timeout -k 10 500 python bench.py > gpurun_out/r05l/bench.json 2> gpurun_out/r05l/bench.err
echo ok
