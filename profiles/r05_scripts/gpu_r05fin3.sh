# full GPU suite + default bench + smoke on the in-tree library
set -e
mkdir -p gpurun_out/r05fin3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05fin3/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05fin3/smoke.log 2>&1
timeout -k 10 500 python bench.py > gpurun_out/r05fin3/bench.json 2> gpurun_out/r05fin3/bench.err
echo ok
