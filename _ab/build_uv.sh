#!/usr/bin/env bash
# user_fused.hip variants from _ab/v/uf_<name>.hip -> _ab/lib_u<name>.so (+ _ut timing build)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/newsrecommendationsystem_amd
for NAME in "$@"; do
  for T in "" "t"; do
    TMP=$ROOT/_ab/obj_u$NAME$T; mkdir -p "$TMP"
    F=(); [ -n "$T" ] && F=(-DNRMS_USER_TIMING)
    cp "$ROOT/_ab/v/uf_$NAME.hip" "$PKG/csrc/_uv_$NAME.hip"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$ROOT/include" -I "$PKG/csrc" "${F[@]}" -c "$PKG/csrc/_uv_$NAME.hip" -o "$TMP/user_fused.o"
    rm -f "$PKG/csrc/_uv_$NAME.hip"
    objs=(); for o in "$PKG/_build"/*.o; do b=$(basename "$o"); [ "$b" = user_fused.o ] && objs+=("$TMP/$b") || objs+=("$o"); done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/_ab/lib_u$NAME$T.so" "${objs[@]}"
  done
done
