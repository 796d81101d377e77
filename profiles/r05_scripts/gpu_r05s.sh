# phase clocks of the cold verifier on the synthetic 2^20-step proof, and its kernel trace
set -e
mkdir -p gpurun_out/r05s
STARK_PROFILE=1 timeout -k 10 180 python tools/verify_phases.py synth20 4 > gpurun_out/r05s/verify_phases.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05s/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/verify_phases.py synth20 3 > $GRAFT_REPO_ROOT/gpurun_out/r05s/trace.log 2>&1
echo ok
