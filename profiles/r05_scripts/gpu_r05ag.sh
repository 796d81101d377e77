# kernel stats of the cold 2^20-step proof with each library (lincomb + L-tree leaf pass, before/after);
# the second run swaps the previous commit's library in (the box's copy of the tree only)
set -e
mkdir -p gpurun_out/r05ag
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05ag/new -o run -- python3 $R/tools/time_r1cs.py --fixtures "" --synth 20 --reps 6 > $R/gpurun_out/r05ag/new.log 2>&1
cp $R/variants/head_c0df5fd.so $R/stark-pure-rust_amd/libstark_hip.so
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05ag/old -o run -- python3 $R/tools/time_r1cs.py --fixtures "" --synth 20 --reps 6 > $R/gpurun_out/r05ag/old.log 2>&1
echo ok
