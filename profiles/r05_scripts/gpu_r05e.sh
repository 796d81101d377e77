set -e
mkdir -p gpurun_out/r05e
cd variants/vp
for i in 1 2; do ./vp_old pedersen_proof.json > ../../gpurun_out/r05e/old_$i.txt 2>&1; ./vp_fast pedersen_proof.json > ../../gpurun_out/r05e/fast_$i.txt 2>&1; done
STARK_PROFILE=1 ./vp_old pedersen_proof.json > ../../gpurun_out/r05e/old_prof.txt 2>&1
echo ok
