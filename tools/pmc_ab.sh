#!/bin/bash
# SQ counter pass (issue / wait breakdown) of the NTT pass kernels for the radix-2^29 (default) and
# radix-2^32 (STARK_NTT29=0) paths: tools/pmc_ab.sh <tag>  -> gpurun_out/pmcab_<tag>/{n29,n32}.json
set -e
TAG=$1
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmcab_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp WHAT=ntt
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
C2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_WAVES"
for v in 29 32; do
  if [ $v = 32 ]; then export STARK_NTT29=0; else unset STARK_NTT29; fi
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/a$v" -o run -- python3 "$ROOT/tools/prof_kernels.py" > "$OUT/a$v.log" 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $C2 --output-format csv -d "$OUT/b$v" -o run -- python3 "$ROOT/tools/prof_kernels.py" > "$OUT/b$v.log" 2>&1
  python3 "$ROOT/tools/pmc_summary.py" "$OUT/n$v.json" "$OUT/a$v" "$OUT/b$v" > /dev/null
done
echo done
