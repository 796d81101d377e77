# B2 = S / Zb2 - I2 / Zb2 with both by partial fractions (no Horner of I2 in the constraint kernel):
# parity suites, then wall A/B and kernel stats against the previous library
set -e
mkdir -p gpurun_out/r05ah
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_r1cs.py tests/test_gpu_dprove.py tests/test_gpu_verify.py > gpurun_out/r05ah/tests.log 2>&1
A=variants/head_c0df5fd.so; B=stark-pure-rust_amd/libstark_hip.so
for i in 1 2 3; do
  timeout -k 10 120 python tools/time_r1cs_libs.py $A $B --fixture pedersen_test --reps 30 >> gpurun_out/r05ah/abped.log 2>&1
  timeout -k 10 120 python tools/time_r1cs_libs.py $A $B --steps 20 --reps 10 >> gpurun_out/r05ah/ab20.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05ah/new -o run -- python3 $R/tools/time_r1cs.py --fixtures "" --synth 20 --reps 6 > $R/gpurun_out/r05ah/new.log 2>&1
cp $R/$A $R/$B
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05ah/old -o run -- python3 $R/tools/time_r1cs.py --fixtures "" --synth 20 --reps 6 > $R/gpurun_out/r05ah/old.log 2>&1
echo ok
