#!/bin/bash
# Build libuvhttp_ws_amd.so from git revision REV into tools/bin/libws_REV.so (for
# tools/ab_lib.py A/B runs against the working tree's build).  Run here; the .so travels.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:?usage: build_rev.sh REV}
TMP=$(mktemp -d)
mkdir -p "$TMP/include" "$TMP/csrc" "$ROOT/tools/bin"
# every source of the library (the ctypes mirror binds all of its symbols)
for h in uvhttp_ws_amd.h uvhttp_tls_amd.h; do
  git -C "$ROOT" show "$REV:include/$h" > "$TMP/include/$h"
done
for f in ws_gpu.hip tls_gpu.hip ws_batcher.hip ws_host.c; do
  git -C "$ROOT" show "$REV:uvhttp_amd/csrc/$f" > "$TMP/csrc/$f"
done
for f in ws_gpu tls_gpu ws_batcher; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$TMP/include" \
    -mcode-object-version=5 -c -o "$TMP/$f.o" "$TMP/csrc/$f.hip"
done
gcc -O2 -DNDEBUG -fPIC -std=gnu11 -I"$TMP/include" -c -o "$TMP/ws_host.o" "$TMP/csrc/ws_host.c"
OBJS="$TMP/ws_gpu.o $TMP/tls_gpu.o $TMP/ws_batcher.o $TMP/ws_host.o"
# (the batcher group, from round 4 on)
if git -C "$ROOT" show "$REV:uvhttp_amd/csrc/ws_batcher_group.cpp" > "$TMP/csrc/ws_batcher_group.cpp" 2>/dev/null; then
  g++ -O2 -fPIC -std=c++17 -I"$TMP/include" -c -o "$TMP/ws_batcher_group.o" "$TMP/csrc/ws_batcher_group.cpp"
  OBJS="$OBJS $TMP/ws_batcher_group.o"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/tools/bin/libws_$REV.so" $OBJS
rm -rf "$TMP"
echo "$ROOT/tools/bin/libws_$REV.so"
