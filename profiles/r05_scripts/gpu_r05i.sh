# host phase clocks of the cold verifier (pedersen) and the cold 2^20-step proof
set -e
mkdir -p gpurun_out/r05i
STARK_PROFILE=1 timeout -k 10 120 python tools/verify_phases.py pedersen_test 8 > gpurun_out/r05i/verify_phases.log 2>&1
STARK_PROFILE=1 timeout -k 10 180 python tools/time_r1cs.py --fixtures "" --synth 20 --reps 4 > gpurun_out/r05i/proof_phases.log 2>&1
echo ok
