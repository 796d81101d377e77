#!/bin/bash
# Counter passes over tools/prof_kernels.py (NTT 2^24 + Merkle 2^24 x 32 B / 2^21 x 256 B), one
# rocprofv3 --pmc pass per group (gfx950 slot limits: 8 SQ, 4 TCC, 2 GRBM), each under its own
# time limit; then tools/pmc_summary.py.  Run from the repo root on the GPU box:
#   tools/pmc_round.sh <tag> [WHAT]
set -e
TAG=$1
export WHAT=${2:-all}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_$TAG
rm -rf "$OUT"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
W="python3 $ROOT/tools/prof_kernels.py"
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- $W > "$OUT/$name.log" 2>&1
}
PASSES=${PASSES:-p1 p2 p3 p4}
want() { [[ " $PASSES " == *" $1 "* ]]; }
want p1 && pass p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT
want p2 && pass p2 SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_WAVES
want p3 && pass p3 FETCH_SIZE
want p4 && pass p4 WRITE_SIZE
DIRS=""
for p in $PASSES; do DIRS="$DIRS $OUT/$p"; done
python3 "$ROOT/tools/pmc_summary.py" "$OUT/summary.json" $DIRS > /dev/null
echo "pmc $TAG done"
