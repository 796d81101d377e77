# verifier pre-parse: branch keys found by memchr('{') + compare instead of memmem; parity then A/B
set -e
mkdir -p gpurun_out/r05aq
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_verify.py > gpurun_out/r05aq/tests.log 2>&1
A=variants/head_c32ff37.so; B=stark-pure-rust_amd/libstark_hip.so
timeout -k 10 600 python tools/time_verify_libs.py $A $B $A $B $A $B --synth > gpurun_out/r05aq/ab.log 2>&1
STARK_PROFILE=1 timeout -k 10 120 python tools/time_verify.py > gpurun_out/r05aq/phases.log 2>&1
echo ok
