#!/bin/bash
# A/B baseline: build libctr_reach_amd.so of a git revision (default HEAD) from a copy of that
# revision's sources into gym-ctr-reach_amd/ctr_reach_amd/lib/libab_<name>.so, so the working
# tree's library can be timed against it (scripts/gpu.sh ab takes the names in $AB).
# usage: [PATCH=<file>] [EXTRA="<hipcc flags>"] bash tools/experiments/build_rev.sh [rev] [name]
#   PATCH  a patch (paths from the repo root, -p1) applied to the copy before the build, e.g. the
#          timing diagnostics, which are not part of the product sources:
#            PATCH=tools/experiments/diag.patch EXTRA=-DCTR_DIAG_WAVETIME  (per-wave stamps,
#              tools/wave_times.py; libab_wavet.so for scripts/gpu.sh wavet)
#            PATCH=tools/experiments/diag.patch EXTRA=-DCTR_DIAG_NOFK      (k_step without its FK)
#   EXTRA  extra hipcc flags for the copy's build
set -euo pipefail
REV=${1:-HEAD}
NAME=${2:-prev}
ROOT=$(git rev-parse --show-toplevel)
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
git -C "$ROOT" archive "$REV" gym-ctr-reach_amd/csrc gym-ctr-reach_amd/Makefile include | tar -x -C "$TMP"
if [ -n "${PATCH:-}" ]; then
    patch -d "$TMP" -p1 --quiet < "$ROOT/$PATCH"
fi
make -C "$TMP/gym-ctr-reach_amd" -s LIB="$ROOT/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_$NAME.so" \
    EXTRA="${EXTRA:-}" "$ROOT/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_$NAME.so"
echo "built libab_$NAME.so from $REV${PATCH:+ + $PATCH}${EXTRA:+ ($EXTRA)}"
