# proof reader: AVX-512 u8 arrays (STARK_JSON_SIMD=1, default) vs the scalar loop (=0); parity suites first
set -e
mkdir -p gpurun_out/r05ap
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_verify.py tests/test_verify_host.py tests/test_json_reader_simd.py tests/test_json_writer.py > gpurun_out/r05ap/tests.log 2>&1
STARK_JSON_SIMD=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_verify.py > gpurun_out/r05ap/tests_scalar.log 2>&1
L=stark-pure-rust_amd/libstark_hip.so
for i in 1 2 3; do
  for simd in 1 0; do
    echo "simd=$simd" >> gpurun_out/r05ap/ab.log
    STARK_JSON_SIMD=$simd timeout -k 10 300 python tools/time_verify_libs.py $L --synth >> gpurun_out/r05ap/ab.log 2>&1
  done
done
for simd in 1 0; do
  STARK_JSON_SIMD=$simd STARK_PROFILE=1 timeout -k 10 120 python tools/time_verify.py > gpurun_out/r05ap/phases_simd$simd.log 2>&1
done
echo ok
