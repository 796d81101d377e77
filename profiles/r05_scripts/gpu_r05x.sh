# spot verifier with F0's / IDX's first passes cached + SIMD host path checks: verify suite, A/B vs a498a5e
set -e
mkdir -p gpurun_out/r05x
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_verify.py tests/test_verify_host.py > gpurun_out/r05x/tests.log 2>&1
A=variants/head_a498a5e.so; B=stark-pure-rust_amd/libstark_hip.so
timeout -k 10 300 python tools/time_verify_libs.py $A $B $A $B --synth > gpurun_out/r05x/ab.log 2>&1
STARK_PROFILE=1 timeout -k 10 120 python tools/time_verify.py > gpurun_out/r05x/verify_phases_ped.log 2>&1
STARK_PROFILE=1 timeout -k 10 180 python tools/verify_phases.py synth20 4 > gpurun_out/r05x/verify_phases20.log 2>&1
echo ok
