#!/bin/bash
# SQ counter passes of the NTT kernels for several builds of the library:
#   tools/pmc_lib_ab.sh <tag> a.so b.so ...  -> gpurun_out/pmclib_<tag>/<name>.json
set -e
TAG=$1; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmclib_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp WHAT=${WHAT:-ntt}
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
C2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_WAVES"
for lib in "$@"; do
  v=$(basename "$lib" .so)
  export STARK_LIB=$ROOT/$lib
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/a_$v" -o run -- python3 "$ROOT/tools/prof_kernels.py" > "$OUT/a_$v.log" 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $C2 --output-format csv -d "$OUT/b_$v" -o run -- python3 "$ROOT/tools/prof_kernels.py" > "$OUT/b_$v.log" 2>&1
  python3 "$ROOT/tools/pmc_summary.py" "$OUT/$v.json" "$OUT/a_$v" "$OUT/b_$v" > /dev/null
done
echo done
