#!/bin/bash
# Build an A/B variant of libdgx.so with extra compile flags for ONE source file:
#   tools/build_variant.sh NAME SRC.hip [FLAGS...]  ->  abl/libdgx_NAME.so
# (the other objects from dgcnn.pytorch_amd/csrc/build; run `make` first)
set -e
NAME=$1; SRC=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/dgcnn.pytorch_amd/csrc
mkdir -p "$ROOT/abl" /tmp/abl_$NAME
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" -c "$C/$SRC" \
    -o /tmp/abl_$NAME/${SRC%.hip}.o
objs=$(ls "$C"/build/*.o | grep -v "/${SRC%.hip}.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -Wl,-soname,libdgx.so -o "$ROOT/abl/libdgx_$NAME.so" $objs \
    /tmp/abl_$NAME/${SRC%.hip}.o
echo "built abl/libdgx_$NAME.so"
