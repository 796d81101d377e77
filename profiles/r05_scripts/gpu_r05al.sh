# staged upload of the cold proof's 21.5 MB: stager threads (STARK_STAGERS) and one vs two copy streams
# (STARK_UP_STREAMS; temporary switches), same library in alternating processes
set -e
mkdir -p gpurun_out/r05al
L=stark-pure-rust_amd/libstark_hip.so
for i in 1 2 3; do
  for cfg in "6 1" "12 1" "6 2" "12 2"; do
    set -- $cfg
    echo "stagers=$1 streams=$2" >> gpurun_out/r05al/ab.log
    STARK_STAGERS=$1 STARK_UP_STREAMS=$2 timeout -k 10 120 python tools/time_r1cs_libs.py $L --steps 20 --reps 10 >> gpurun_out/r05al/ab.log 2>&1
  done
done
echo ok
