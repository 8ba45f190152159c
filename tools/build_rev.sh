#!/bin/bash
# Build libuvhttp_ws_amd.so from git revision REV into tools/bin/libws_REV.so (for
# tools/ab_lib.py A/B runs against the working tree's build).  Run here; the .so travels.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:?usage: build_rev.sh REV}
TMP=$(mktemp -d)
mkdir -p "$TMP/include" "$TMP/csrc" "$ROOT/tools/bin"
git -C "$ROOT" show "$REV:include/uvhttp_ws_amd.h" > "$TMP/include/uvhttp_ws_amd.h"
git -C "$ROOT" show "$REV:uvhttp_amd/csrc/ws_gpu.hip" > "$TMP/csrc/ws_gpu.hip"
git -C "$ROOT" show "$REV:uvhttp_amd/csrc/ws_host.c" > "$TMP/csrc/ws_host.c"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$TMP/include" \
  -mcode-object-version=5 -c -o "$TMP/ws_gpu.o" "$TMP/csrc/ws_gpu.hip"
gcc -O2 -DNDEBUG -fPIC -std=gnu11 -I"$TMP/include" -c -o "$TMP/ws_host.o" "$TMP/csrc/ws_host.c"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/tools/bin/libws_$REV.so" \
  "$TMP/ws_gpu.o" "$TMP/ws_host.o"
rm -rf "$TMP"
echo "$ROOT/tools/bin/libws_$REV.so"
