#!/usr/bin/env bash
# Builds h-numo_amd/libhnumo_engine.so for gfx950 (MI355X).  Cross-compiles without a GPU.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="${HNUMO_OUT:-$HERE/../libhnumo_engine.so}"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
"$HIPCC" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-variable -Wno-unused-function \
  -munsafe-fp-atomics -ffp-contract=off ${HNUMO_EXTRA_FLAGS:-} \
  -o "$OUT.tmp" "$HERE/engine.hip" -lrccl
mv "$OUT.tmp" "$OUT"
echo "built $OUT"
