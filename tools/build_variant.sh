#!/bin/bash
# Builds an experimental variant of libstark_hip.so: copies csrc/ to a temp
# dir, applies a python transform to ntt.hip (or $VARIANT_FILE), compiles.
# Timing-only builds; never shipped.
# usage: [VARIANT_FILE=merkle.hip] build_variant.sh <out.so> <python-expr on s | @file.py with apply(s)> [extra hipcc flags]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1; EXPR=$2; shift 2
TMP=$(mktemp -d)
cp "$ROOT"/stark-pure-rust_amd/csrc/* "$TMP"/
python3 - "$TMP/${VARIANT_FILE:-ntt.hip}" "$EXPR" <<'PY'
import sys
p, expr = sys.argv[1], sys.argv[2]
s = open(p).read()
if expr.startswith("@"):  # a python file defining apply(s) -> s
    ns = {}
    exec(open(expr[1:]).read(), ns)
    s = ns["apply"](s)
else:
    s = eval(expr)
open(p, 'w').write(s)
PY
for f in $(cd "$TMP" && ls *.hip | sed "s/\.hip$//"); do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value -I"$ROOT/include" "$@" -c "$TMP/$f.hip" -o "$TMP/$f.o" &
done
wait
# host-only objects (worker pool, SIMD path checks, JSON digits) from the main build: make -C stark-pure-rust_amd first
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o "$OUT" "$TMP"/*.o "$ROOT"/stark-pure-rust_amd/build/host_*.o
rm -rf "$TMP"
