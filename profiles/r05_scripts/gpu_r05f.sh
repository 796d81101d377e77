set -e
mkdir -p gpurun_out/r05f
(cd variants/vp && ./vp_instr pedersen_proof.json > ../../gpurun_out/r05f/vp_instr.txt 2>&1)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05f/gpu_tests.log 2>&1
timeout -k 10 300 python tools/time_r1cs_libs.py variants/head.so variants/new2.so variants/head.so variants/new2.so --steps 20 --reps 6 > gpurun_out/r05f/ab_proof20.txt 2>&1
timeout -k 10 300 python tools/time_r1cs_libs.py variants/head.so variants/new2.so variants/head.so variants/new2.so --fixture pedersen_test --reps 20 > gpurun_out/r05f/ab_pedersen.txt 2>&1
timeout -k 10 300 python tools/time_verify_libs.py variants/head.so variants/new2.so variants/head.so variants/new2.so --reps 30 > gpurun_out/r05f/ab_verify.txt 2>&1
echo ok
