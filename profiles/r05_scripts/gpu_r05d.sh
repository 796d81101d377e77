set -e
mkdir -p gpurun_out/r05d
timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_ntt.py tests/test_gpu_distributed.py tests/test_gpu_merkle_fri.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05d/tests.log 2>&1
STARK_PROFILE=1 timeout -k 10 120 python tools/verify_phases.py pedersen_test 8 > gpurun_out/r05d/verify_phases.log 2>&1
timeout -k 10 300 python tools/time_verify_libs.py variants/head.so variants/new1.so variants/head.so variants/new1.so --reps 30 > gpurun_out/r05d/ab_verify.txt 2>&1
timeout -k 10 300 python tools/ab_libs.py --cases ntt20,ntt26 --reps 30 --rounds 5 variants/head.so variants/new1.so > gpurun_out/r05d/ab_ntt.txt 2>&1
echo ok
