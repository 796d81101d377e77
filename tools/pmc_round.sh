#!/bin/bash
# Counter passes over tools/prof_kernels.py, one rocprofv3 --pmc pass per counter group (gfx950 slot
# limits per pass: 8 SQ, 4 TCC with FETCH_SIZE = 3 and WRITE_SIZE = 2, 2 GRBM), each under its own time
# limit; then tools/pmc_summary.py.  Every SQ pass carries GRBM_GUI_ACTIVE, so each dispatch's VALU
# issue fraction is priced at that dispatch's own clock (no cross-run clock).  Run from the repo root
# on the GPU box:
#   tools/pmc_round.sh <tag> [WHAT]        WHAT = all (NTT 2^24 + Merkle) | prover | ntt | merkle
set -e
TAG=$1
export WHAT=${2:-all}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_$TAG
rm -rf "$OUT"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 "$ROOT/tools/prof_kernels.py" > "$OUT/$name.log" 2>&1
  echo "pass $name ok"
}
PASSES=${PASSES:-p1 p2 p3 p4 p5}
want() { [[ " $PASSES " == *" $1 "* ]]; }
# p1: VALU issue and its cost classes (SQ_ACTIVE_INST_VALU2 = quad-cycles with two VALU instructions issued)
want p1 && pass p1 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
# p2: where waves wait
want p2 && pass p2 SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
# p3: the rest of the instruction mix
want p3 && pass p3 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE
want p4 && pass p4 FETCH_SIZE
want p5 && pass p5 WRITE_SIZE
DIRS=""
for p in $PASSES; do DIRS="$DIRS $OUT/$p"; done
python3 "$ROOT/tools/pmc_summary.py" "$OUT/summary.json" $DIRS > /dev/null
echo "pmc $TAG $WHAT done"
