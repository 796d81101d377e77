set -e
mkdir -p gpurun_out/r05b
timeout -k 10 300 python tools/ab_libs.py --cases ntt20,ntt22,ntt24,ntt26,intt24 --reps 30 --rounds 5 variants/head.so variants/csub.so > gpurun_out/r05b/ab_csub.txt 2>&1
STARK_PROFILE=1 timeout -k 10 180 python tools/time_r1cs.py --fixtures "" --synth 20 --reps 4 > gpurun_out/r05b/phases.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05b/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/time_r1cs.py --fixtures "" --synth 20 --reps 4 > $GRAFT_REPO_ROOT/gpurun_out/r05b/trace.log 2>&1
echo ok
