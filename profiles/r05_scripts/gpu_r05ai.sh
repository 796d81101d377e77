# host/API timeline of the cold 2^20-step proof: what the ~1.2 ms between one proof's last kernel and the
# next proof's first kernel is made of (kernel + HIP runtime + copy traces, no counters)
set -e
mkdir -p gpurun_out/r05ai
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/r05ai/t -o run -- python3 $R/tools/time_r1cs.py --fixtures "" --synth 20 --reps 4 > $R/gpurun_out/r05ai/t.log 2>&1
echo ok
