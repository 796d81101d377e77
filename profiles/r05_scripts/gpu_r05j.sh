# verifier: openings in one arena (no per-opening vectors); tests, phases, A/B against cdb5 (previous library)
set -e
mkdir -p gpurun_out/r05j
timeout -k 10 300 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_merkle_fri.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05j/tests.log 2>&1
(cd variants/vp && ./vp_arena pedersen_proof.json > ../../gpurun_out/r05j/vp_arena.txt 2>&1 && ./vp_old pedersen_proof.json > ../../gpurun_out/r05j/vp_old.txt 2>&1)
STARK_PROFILE=1 timeout -k 10 120 python tools/verify_phases.py pedersen_test 8 > gpurun_out/r05j/verify_phases.log 2>&1
timeout -k 10 300 python tools/time_verify_libs.py variants/cdb5.so variants/ver2.so variants/cdb5.so variants/ver2.so --reps 30 > gpurun_out/r05j/ab_verify.txt 2>&1
echo ok
