#!/bin/bash
# round-4 closing GPU pass (the in-tree library at the round end): every GPU test,
# smoke(), the default bench line, and the cold 2^20-step proof's phase / kernel profile.
mkdir -p gpurun_out/r4ad
(while true; do date > gpurun_out/r4ad/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4ad/tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ad/smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py > gpurun_out/r4ad/bench.json 2> gpurun_out/r4ad/bench.err || exit 3
bash tools/prof_2_20_proof.sh || exit 4
