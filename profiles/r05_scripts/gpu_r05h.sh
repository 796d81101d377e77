# constraint kernel: inv(Z) products by LDS digit-basis tables (cdb5 = in-tree) vs cdb3; tests first
set -e
mkdir -p gpurun_out/r05h
timeout -k 10 400 python -u -m pytest tests/test_gpu_r1cs.py tests/test_gpu_dprove.py tests/test_gpu_verify.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05h/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
for v in cdb3 cdb5 base; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05h/$v -o run -- python3 $GRAFT_REPO_ROOT/tools/time_r1cs_libs.py $GRAFT_REPO_ROOT/variants/$v.so --steps 20 --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r05h/$v.log 2>&1
done
echo ok
