# L tree leaf digests written by the lincomb kernel (no separate leaf pass over L): r1cs/verify/merkle suites; prover A/B
set -e
mkdir -p gpurun_out/r05af
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_r1cs.py tests/test_gpu_verify.py tests/test_gpu_merkle_fri.py tests/test_gpu_dprove.py > gpurun_out/r05af/tests.log 2>&1
A=variants/head_c0df5fd.so; B=stark-pure-rust_amd/libstark_hip.so
for i in 1 2 3; do
  timeout -k 10 120 python tools/time_r1cs_libs.py $A $B --steps 20 --reps 10 >> gpurun_out/r05af/ab20.log 2>&1
  timeout -k 10 120 python tools/time_r1cs_libs.py $A $B --fixture pedersen_test --reps 30 >> gpurun_out/r05af/abped.log 2>&1
done
echo ok
