#!/bin/bash
# A/B baseline: build libctr_reach_amd.so of a git revision (default HEAD) from a copy of that
# revision's sources into gym-ctr-reach_amd/ctr_reach_amd/lib/libab_<name>.so, so the working
# tree's library can be timed against it (scripts/gpu.sh ab takes the names in $AB).
# usage: bash tools/experiments/build_rev.sh [rev] [name]
set -euo pipefail
REV=${1:-HEAD}
NAME=${2:-prev}
ROOT=$(git rev-parse --show-toplevel)
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
git -C "$ROOT" archive "$REV" gym-ctr-reach_amd/csrc gym-ctr-reach_amd/Makefile include | tar -x -C "$TMP"
make -C "$TMP/gym-ctr-reach_amd" -s LIB="$ROOT/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_$NAME.so" \
    "$ROOT/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_$NAME.so"
echo "built libab_$NAME.so from $REV"
