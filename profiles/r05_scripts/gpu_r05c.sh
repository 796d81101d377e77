set -e
mkdir -p gpurun_out/r05c
timeout -k 10 300 python tools/ab_libs.py --cases ntt20,ntt24,ntt26,intt24 --reps 30 --rounds 5 variants/head.so variants/csub_h.so > gpurun_out/r05c/ab_csub_h.txt 2>&1
timeout -k 10 300 python tools/time_r1cs_libs.py variants/head.so variants/upl.so variants/head.so variants/upl.so --steps 20 --reps 6 > gpurun_out/r05c/ab_upload.txt 2>&1
STARK_PROFILE=1 timeout -k 10 120 python tools/verify_phases.py pedersen_test 6 > gpurun_out/r05c/verify_phases.log 2>&1
echo ok
