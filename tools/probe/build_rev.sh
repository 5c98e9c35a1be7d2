#!/bin/bash
# Build libggs from the csrc/ + include/ of a git revision (or the working tree
# with REV=WORK) into genetic-gaussian-splats_amd/libggs_<name>.so, a product build
# for A/B timing (tools/probe/rtime.py, GGS_LIB=...).  The build runs in a scratch
# copy; the tree's own libggs.so is untouched.
#   bash tools/probe/build_rev.sh <rev|WORK> <name>
set -eu
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
TMP=$(mktemp -d /tmp/ggs_rev.XXXXXX)
mkdir -p "$TMP/pkg/csrc" "$TMP/include"
if [ "$REV" = WORK ]; then
  cp "$ROOT"/genetic-gaussian-splats_amd/csrc/{Makefile,*.hip,*.cpp,*.h} "$TMP/pkg/csrc/"
  cp "$ROOT"/include/*.h "$TMP/include/"
else
  git -C "$ROOT" archive "$REV" genetic-gaussian-splats_amd/csrc include | tar -x -C "$TMP"
  mv "$TMP/genetic-gaussian-splats_amd/csrc"/* "$TMP/pkg/csrc/"
fi
make -C "$TMP/pkg/csrc" -j8 OUT="$ROOT/genetic-gaussian-splats_amd/libggs_$NAME.so" > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
rm -rf "$TMP"
echo "built genetic-gaussian-splats_amd/libggs_$NAME.so from $REV"
