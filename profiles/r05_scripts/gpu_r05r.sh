# new tests: the verifier's arena edges, FRI exclusion divisors 2 and 3 (device indices)
set -e
mkdir -p gpurun_out/r05r
timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_merkle_fri.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05r/tests.log 2>&1
echo ok
