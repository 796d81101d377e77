# proof JSON: AVX-512 byte-array digits (STARK_JSON_SIMD=1, default) vs the scalar table path (=0), and
# to_json filling its str in place from the library's parallel copy; parity suites first
set -e
mkdir -p gpurun_out/r05an
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_r1cs.py tests/test_gpu_verify.py tests/test_gpu_dprove.py tests/test_json_writer.py > gpurun_out/r05an/tests.log 2>&1
for simd in 1 0; do
  FIXTURE=pedersen_test REPS=8 STARK_PROFILE=1 STARK_JSON_SIMD=$simd timeout -k 10 120 python3 profiles/r05_scripts/r05aj_phases.py > gpurun_out/r05an/phases_simd$simd.log 2>&1
done
L=stark-pure-rust_amd/libstark_hip.so
for i in 1 2 3; do
  for simd in 1 0; do
    echo "simd=$simd" >> gpurun_out/r05an/abped.log
    STARK_JSON_SIMD=$simd timeout -k 10 120 python tools/time_r1cs_libs.py $L --fixture pedersen_test --reps 30 >> gpurun_out/r05an/abped.log 2>&1
    echo "simd=$simd" >> gpurun_out/r05an/ab20.log
    STARK_JSON_SIMD=$simd timeout -k 10 120 python tools/time_r1cs_libs.py $L --steps 20 --reps 10 >> gpurun_out/r05an/ab20.log 2>&1
  done
done
echo ok
