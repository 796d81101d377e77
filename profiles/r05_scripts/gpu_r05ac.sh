# long factors' running sums by a wave scan (running_sum_long_kernel): r1cs, verify, dprove suites; prover A/B
set -e
mkdir -p gpurun_out/r05ac
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_r1cs.py tests/test_gpu_verify.py tests/test_gpu_dprove.py > gpurun_out/r05ac/tests.log 2>&1
A=variants/head_804c68d.so; B=stark-pure-rust_amd/libstark_hip.so
for i in 1 2 3; do
  timeout -k 10 120 python tools/time_r1cs_libs.py $A $B --fixture pedersen_test --reps 30 >> gpurun_out/r05ac/abped.log 2>&1
done
timeout -k 10 120 python tools/time_r1cs_libs.py $A $B $A $B --fixture bits --reps 30 >> gpurun_out/r05ac/abbits.log 2>&1
timeout -k 10 120 python tools/time_r1cs_libs.py $A $B $A $B --steps 20 --reps 10 >> gpurun_out/r05ac/ab20.log 2>&1
echo ok
