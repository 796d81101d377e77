# constraint-kernel digit-basis constants: GPU tests on the in-tree build, then per-variant kernel stats
set -e
mkdir -p gpurun_out/r05g
timeout -k 10 400 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_dprove.py tests/test_gpu_verify.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05g/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
for v in base cdb2 cdb3 cdb4; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05g/$v -o run -- python3 $GRAFT_REPO_ROOT/tools/time_r1cs_libs.py $GRAFT_REPO_ROOT/variants/$v.so --steps 20 --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r05g/$v.log 2>&1
done
echo ok
