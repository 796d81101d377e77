set -e
mkdir -p gpurun_out/v
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_verify.py tests/test_gpu_r1cs.py tests/test_gpu_group.py tests/test_gpu_dprove.py tests/test_gpu_streams.py tests/test_abi_client.py > gpurun_out/v/tests.log 2>&1
STARK_PROFILE=1 timeout -k 10 200 python -u tools/verify_phases.py synth20 4 > gpurun_out/v/vphase.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/v/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/verify_phases.py synth20 6 > $GRAFT_REPO_ROOT/gpurun_out/v/trace.log 2>&1
