#!/usr/bin/env bash
# Build an A/B variant of libnrms_hip.so with one source recompiled with extra flags:
#   bash _ab/build_variant.sh <name> <source.hip> [flags...]   -> _ab/lib_<name>.so
set -euo pipefail
NAME=$1; SRC=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/newsrecommendationsystem_amd
OBJ=$PKG/_build
TMP=$ROOT/_ab/obj_$NAME; mkdir -p "$TMP"
# (SRC_FILE=path: compile that file in place of csrc/<source.hip>)
# the product build's per-file flags (build.py FILE_FLAGS) first, then the variant's
FF=$([ -n "${NOFF:-}" ] && exit 0; cd "$ROOT" && python -c "import sys; sys.path.insert(0, '.'); from newsrecommendationsystem_amd.build import FILE_FLAGS; print(' '.join(FILE_FLAGS.get('$SRC', [])))")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$ROOT/include" -I "$PKG/csrc" $FF "$@" -c "${SRC_FILE:-$PKG/csrc/$SRC}" -o "$TMP/${SRC%.hip}.o"
objs=()
for o in "$OBJ"/*.o; do
  b=$(basename "$o"); [ "$b" = "${SRC%.hip}.o" ] && objs+=("$TMP/$b") || objs+=("$o")
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/_ab/lib_$NAME.so" "${objs[@]}"
echo "$ROOT/_ab/lib_$NAME.so"
