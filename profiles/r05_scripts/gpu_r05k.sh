# NTT: second pass's column twiddle applied in the first pass's store (twmove) vs HEAD (ver2)
set -e
mkdir -p gpurun_out/r05k
timeout -k 10 400 python tools/ab_libs.py --cases ntt20,ntt22,ntt24,ntt26,intt24,ntt24 --reps 30 --rounds 6 variants/ver2.so variants/twmove.so > gpurun_out/r05k/ab_twmove.txt 2>&1
echo ok
