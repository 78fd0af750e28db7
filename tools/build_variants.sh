#!/bin/bash
# Build tuning variants of libvr.so into tools/build/variants/<name>/ (tooling only).
# usage: tools/build_variants.sh name1:"-DFLAG=.." name2:"-D.." ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CSRC="$ROOT/volume-rendering-based-on-distribution-data_amd/csrc"
for spec in "$@"; do
  name="${spec%%:*}"; flags="${spec#*:}"
  [ "$name" = "$spec" ] && flags=""
  out="$ROOT/tools/build/variants/$name"
  make -s -C "$CSRC" BUILD="$out" EXTRA="$flags" -j2 &
done
wait
ls "$ROOT"/tools/build/variants/*/libvr.so
