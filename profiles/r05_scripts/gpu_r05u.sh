# Merkle tail in one launch (last workgroup hashes the grid's nodes to the root): GPU suites, prover A/B
set -e
mkdir -p gpurun_out/r05u
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_merkle_fri.py tests/test_gpu_verify.py tests/test_gpu_r1cs.py tests/test_gpu_dprove.py tests/test_gpu_distributed.py > gpurun_out/r05u/tests.log 2>&1
A=variants/base_r05t.so; B=stark-pure-rust_amd/libstark_hip.so
for i in 1 2 3; do
  timeout -k 10 120 python tools/time_r1cs_libs.py $A $B --steps 20 --reps 10 >> gpurun_out/r05u/ab20.log 2>&1
  timeout -k 10 120 python tools/time_r1cs_libs.py $A $B --fixture pedersen_test --reps 30 >> gpurun_out/r05u/abped.log 2>&1
done
timeout -k 10 300 python tools/time_verify_libs.py $A $B > gpurun_out/r05u/abver.log 2>&1
echo ok
