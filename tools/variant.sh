#!/bin/bash
# Build an experimental engine variant (measurement only, never shipped):
#   bash tools/variant.sh <name> "<extra hipcc flags>"
# -> abl/<name>/libespgpu.so (VARDIR), for tools/lib_ab.sh (ESPGPU_LIB=...).
set -e
NAME=${1:?name}; EXTRA=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
VD=${VARDIR:-abl}
mkdir -p "$ROOT/$VD/$NAME"
make -s -C "$ROOT/f-stack_amd" -j8 OBJDIR="$ROOT/$VD/$NAME/build" LIB="$ROOT/$VD/$NAME/libespgpu.so" EXTRA="$EXTRA"
echo "$ROOT/$VD/$NAME/libespgpu.so"
