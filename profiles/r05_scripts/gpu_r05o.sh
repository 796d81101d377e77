# prover: A chain beside the main LDE + parallel r tables (aside2) vs ver2; tests then 3 alternations
set -e
mkdir -p gpurun_out/r05o
timeout -k 10 400 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_dprove.py tests/test_gpu_verify.py tests/test_gpu_streams.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05o/tests.log 2>&1
timeout -k 10 400 python tools/time_r1cs_libs.py variants/ver2.so variants/aside2.so variants/ver2.so variants/aside2.so variants/ver2.so variants/aside2.so --steps 20 --reps 10 > gpurun_out/r05o/ab_proof20.txt 2>&1
timeout -k 10 300 python tools/time_r1cs_libs.py variants/ver2.so variants/aside2.so variants/ver2.so variants/aside2.so variants/ver2.so variants/aside2.so --fixture pedersen_test --reps 30 > gpurun_out/r05o/ab_pedersen.txt 2>&1
echo ok
