set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p29 -o run -- python3 $R/tools/time_ntt.py $R/ab/N29.so > $R/gpurun_out/p29.log 2>&1
STARK_NTT29=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p32 -o run -- python3 $R/tools/time_ntt.py $R/ab/N29.so > $R/gpurun_out/p32.log 2>&1
