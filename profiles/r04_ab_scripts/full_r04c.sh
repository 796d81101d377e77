#!/bin/bash
# round-4 GPU pass on the final library (shared size-only columns, partial-fraction 1/Zb2): every GPU test,
# smoke(), the default bench line, and the cold 2^20-step proof's phase / kernel profile.
mkdir -p gpurun_out/r4u
(while true; do date > gpurun_out/r4u/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4u/tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4u/smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py > gpurun_out/r4u/bench.json 2> gpurun_out/r4u/bench.err || exit 3
bash tools/prof_2_20_proof.sh || exit 4
