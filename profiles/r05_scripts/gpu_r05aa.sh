# proof JSON sized first and written in place (no per-piece strings, no assembly copy): r1cs suites
# (golden digests), verify suite under STARK_POISON, prover A/B vs the previous commit
set -e
mkdir -p gpurun_out/r05aa
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_r1cs.py tests/test_gpu_merkle_fri.py > gpurun_out/r05aa/tests.log 2>&1
STARK_POISON=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_verify.py > gpurun_out/r05aa/poison.log 2>&1
A=variants/head_3217aa9.so; B=stark-pure-rust_amd/libstark_hip.so
for i in 1 2 3; do
  timeout -k 10 120 python tools/time_r1cs_libs.py $A $B --fixture pedersen_test --reps 30 >> gpurun_out/r05aa/abped.log 2>&1
  timeout -k 10 120 python tools/time_r1cs_libs.py $A $B --steps 20 --reps 10 >> gpurun_out/r05aa/ab20.log 2>&1
done
echo ok
