#!/bin/bash
# SQ counter passes (tools/pmc_round.sh p1 + p2) over the 2^24 NTT for several builds of the library, for
# an A/B of pass kernels: tools/pmc_ab.sh <tag> <lib.so> [<lib.so> ...]
#   -> gpurun_out/pmcab_<tag>/<lib basename>/summary.json
set -e
TAG=$1; shift
ROOT=$(pwd)
for LIB in "$@"; do
  NAME=$(basename "$LIB" .so)
  OUT=$ROOT/gpurun_out/pmcab_$TAG/$NAME
  rm -rf "$OUT"; mkdir -p "$OUT"
  (cd /tmp && export TMPDIR=/tmp WHAT=ntt STARK_LIB=$ROOT/$LIB &&
   timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/tools/prof_kernels.py" > "$OUT/p1.log" 2>&1 &&
   timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/tools/prof_kernels.py" > "$OUT/p2.log" 2>&1 &&
   timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/p3" -o run -- python3 "$ROOT/tools/prof_kernels.py" > "$OUT/p3.log" 2>&1)
  python3 "$ROOT/tools/pmc_summary.py" "$OUT/summary.json" "$OUT/p1" "$OUT/p2" "$OUT/p3" > /dev/null
  echo "pmc ab $NAME done"
done
