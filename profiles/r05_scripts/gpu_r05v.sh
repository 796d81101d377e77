# cold verifier from the circuit columns' first forward passes (no extensions): GPU suites, verify A/B, phases
set -e
mkdir -p gpurun_out/r05v
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_verify.py tests/test_gpu_r1cs.py > gpurun_out/r05v/tests.log 2>&1
A=variants/head_9eadd9d.so; B=stark-pure-rust_amd/libstark_hip.so
timeout -k 10 300 python tools/time_verify_libs.py $A $B $A $B --synth > gpurun_out/r05v/ab.log 2>&1
STARK_PROFILE=1 timeout -k 10 180 python tools/verify_phases.py synth20 4 > gpurun_out/r05v/verify_phases.log 2>&1
echo ok
