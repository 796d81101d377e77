# proof reader: numbers read from their first four bytes without branching on the length; leading zeros refused
set -e
mkdir -p gpurun_out/r05ad
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_verify.py > gpurun_out/r05ad/tests.log 2>&1
A=variants/head_c0df5fd.so; B=stark-pure-rust_amd/libstark_hip.so
timeout -k 10 300 python tools/time_verify_libs.py $A $B $A $B $A $B > gpurun_out/r05ad/ab.log 2>&1
echo ok
