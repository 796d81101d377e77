# prover: A's chain on the aux stream beside the main LDE (aside) vs ver2; tests, proof A/B, kernel trace of aside
set -e
mkdir -p gpurun_out/r05n
timeout -k 10 400 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_dprove.py tests/test_gpu_verify.py tests/test_gpu_streams.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05n/tests.log 2>&1
timeout -k 10 300 python tools/time_r1cs_libs.py variants/ver2.so variants/aside.so variants/ver2.so variants/aside.so --steps 20 --reps 6 > gpurun_out/r05n/ab_proof20.txt 2>&1
timeout -k 10 300 python tools/time_r1cs_libs.py variants/ver2.so variants/aside.so variants/ver2.so variants/aside.so --fixture pedersen_test --reps 20 > gpurun_out/r05n/ab_pedersen.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05n/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/time_r1cs_libs.py $GRAFT_REPO_ROOT/variants/aside.so --steps 20 --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r05n/trace.log 2>&1
echo ok
