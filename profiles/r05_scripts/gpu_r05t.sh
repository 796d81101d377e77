# verifier cold build without the slot copies / Montgomery images: GPU verify/r1cs/dprove suites, A/B, phases
set -e
mkdir -p gpurun_out/r05t
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_verify.py tests/test_gpu_r1cs.py tests/test_gpu_dprove.py > gpurun_out/r05t/tests.log 2>&1
timeout -k 10 300 python tools/time_verify_libs.py variants/base_r05t.so stark-pure-rust_amd/libstark_hip.so variants/base_r05t.so stark-pure-rust_amd/libstark_hip.so --synth > gpurun_out/r05t/ab.log 2>&1
STARK_PROFILE=1 timeout -k 10 180 python tools/verify_phases.py synth20 4 > gpurun_out/r05t/verify_phases.log 2>&1
echo ok
