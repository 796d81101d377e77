#!/bin/bash
# Like build_variant.sh, but replaces whole files of csrc/ with given ones (timing-only A/B builds,
# never shipped).  usage: build_variant_files.sh <out.so> <name>=<path> [<name>=<path> ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1; shift
TMP=$(mktemp -d)
cp "$ROOT"/stark-pure-rust_amd/csrc/* "$TMP"/
for kv in "$@"; do cp "${kv#*=}" "$TMP/${kv%%=*}"; done
for f in $(cd "$TMP" && ls *.hip | sed "s/\.hip$//"); do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value -I"$ROOT/include" -c "$TMP/$f.hip" -o "$TMP/$f.o" &
done
wait
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o "$OUT" "$TMP"/*.o
rm -rf "$TMP"
