mkdir -p gpurun_out/ab1
export REPS=200 WARM=20
timeout -k 10 120 python tools/time_ntt.py variants/base.so variants/pf.so variants/base.so variants/pf.so > gpurun_out/ab1/pf24.log 2>&1 || exit 1
LOG_N=23 timeout -k 10 120 python tools/time_ntt.py variants/base.so variants/pf.so variants/base.so variants/pf.so > gpurun_out/ab1/pf23.log 2>&1 || exit 1
LOG_N=20 REPS=1000 timeout -k 10 180 python tools/time_ntt.py variants/base.so variants/p20_8_6_6.so variants/p20_6_6_8.so variants/p20_4_8_8.so variants/p20_7_7_6.so variants/p20_8_8_4.so variants/base.so > gpurun_out/ab1/p20.log 2>&1 || exit 1
LOG_N=20 REPS=1000 timeout -k 10 180 python tools/time_ntt.py variants/p20_8_8_4.so variants/p20_4_8_8.so variants/p20_8_6_6.so variants/base.so > gpurun_out/ab1/p20b.log 2>&1 || exit 1
