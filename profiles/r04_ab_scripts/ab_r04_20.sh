#!/bin/bash
# round-4 batch 20: every GPU test with STARK_POISON=1 (each new device allocation and pinned buffer
# filled with 0xA5): a kernel that reads memory nobody wrote then fails reproducibly.
mkdir -p gpurun_out/r4w
(while true; do date > gpurun_out/r4w/heartbeat; sleep 20; done) & HB=$!
trap "kill $HB" EXIT
STARK_POISON=1 timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r4w/tests.log 2>&1 || exit 1
