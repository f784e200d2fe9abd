#!/bin/bash
# Build an experimental engine variant (measurement only, never shipped):
#   bash tools/variant.sh <name> "<extra hipcc flags>"
# -> exp/<name>/libespgpu.so, for tools/lib_ab.sh (ESPGPU_LIB=...).
set -e
NAME=${1:?name}; EXTRA=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/exp/$NAME"
make -s -C "$ROOT/f-stack_amd" -j8 OBJDIR="$ROOT/exp/$NAME/build" LIB="$ROOT/exp/$NAME/libespgpu.so" EXTRA="$EXTRA"
echo "$ROOT/exp/$NAME/libespgpu.so"
