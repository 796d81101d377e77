# occupancy experiment: extra dynamic LDS per radix>=2^7 pass tile (STARK_NTT_LDS_PAD bytes) takes the
# pass from 3 to 2 workgroups per CU; 2^k tiles then fill whole rounds (no 1/3 tail) at 2 waves/SIMD
set -e
mkdir -p gpurun_out/r05ak
L=stark-pure-rust_amd/libstark_hip.so
for k in 20 22 24 26; do
  for i in 1 2 3; do
    for pad in 0 16384; do
      echo "log_n=$k pad=$pad" >> gpurun_out/r05ak/ab.log
      LOG_N=$k REPS=40 STARK_NTT_LDS_PAD=$pad timeout -k 10 120 python tools/time_ntt.py $L >> gpurun_out/r05ak/ab.log 2>&1
    done
  done
done
echo ok
