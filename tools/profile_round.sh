#!/bin/bash
# Collects the round's rocprofv3 evidence on the GPU box (run from the repo root):
#   1. --kernel-trace --stats of `bench.py --no-extras` (the timed NTT line alone, so
#      the per-launch average of ntt_pass_kernel is the bench's own kernel),
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit one pass on gfx950),
#   3. --kernel-trace --stats of the full default bench (every kernel of the extras),
# and summarises 1+2 into gpurun_out/prof_<tag>/summary.json (tools/profile_summary.py).
# usage: tools/profile_round.sh r01
set -e
TAG=$1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
rm -rf "$OUT"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
B="$ROOT/bench.py --no-extras --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 $B --steps 200 --warmup 10 > "$OUT/bench_stats.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $B --steps 5 --warmup 1 > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $B --steps 5 --warmup 1 > "$OUT/bench_write.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/full" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/bench_full.log" 2>&1
python3 "$ROOT/tools/profile_summary.py" "$OUT/stats" "$OUT/fetch" "$OUT/write" "$OUT/summary.json" "$OUT/bench_stats.log" > /dev/null
echo "profile $TAG done"
