#!/bin/bash
# Build the working tree's library with extra compiler flags (experiment switches) into
# tools/bin/libws_NAME.so, for tools/ab_lib.py.   usage: build_variant.sh NAME [FLAGS...]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=${1:?usage: build_variant.sh NAME [FLAGS...]}
shift
TMP=$(mktemp -d)
mkdir -p "$ROOT/tools/bin"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$ROOT/include" \
  -mcode-object-version=5 "$@" -c -o "$TMP/ws_gpu.o" "$ROOT/uvhttp_amd/csrc/ws_gpu.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$ROOT/include" \
  -mcode-object-version=5 "$@" -c -o "$TMP/tls_gpu.o" "$ROOT/uvhttp_amd/csrc/tls_gpu.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$ROOT/include" \
  -mcode-object-version=5 "$@" -c -o "$TMP/ws_batcher.o" "$ROOT/uvhttp_amd/csrc/ws_batcher.hip"
gcc -O2 -DNDEBUG -fPIC -std=gnu11 -I"$ROOT/include" -c -o "$TMP/ws_host.o" "$ROOT/uvhttp_amd/csrc/ws_host.c"
g++ -O2 -fPIC -std=c++17 -I"$ROOT/include" -c -o "$TMP/ws_batcher_group.o" "$ROOT/uvhttp_amd/csrc/ws_batcher_group.cpp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/tools/bin/libws_$NAME.so" \
  "$TMP/ws_gpu.o" "$TMP/tls_gpu.o" "$TMP/ws_batcher.o" "$TMP/ws_host.o" "$TMP/ws_batcher_group.o"
rm -rf "$TMP"
echo "$ROOT/tools/bin/libws_$NAME.so"
