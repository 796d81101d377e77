# the round's rocprof evidence on the final NTT kernels: kernel stats + HBM bytes (profile_round.sh) and counters (pmc_round.sh)
set -e
bash tools/profile_round.sh r05
bash tools/pmc_round.sh r05 all
echo ok
