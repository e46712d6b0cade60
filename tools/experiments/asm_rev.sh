#!/bin/bash
# Device assembly of a git revision's kernels (or the working tree with rev "WT") for the
# instruction census (tools/asm_blocks.py).  usage: bash tools/experiments/asm_rev.sh REV out.s [extra flags]
set -euo pipefail
REV=$1; OUT=$2; shift 2
ROOT=$(git rev-parse --show-toplevel)
if [ "$REV" = WT ]; then SRC=$ROOT; else
  SRC=$(mktemp -d); trap 'rm -rf "$SRC"' EXIT
  git -C "$ROOT" archive "$REV" gym-ctr-reach_amd/csrc include | tar -x -C "$SRC"
fi
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -I"$SRC/include" -I"$SRC/gym-ctr-reach_amd/csrc" \
  -mllvm -amdgpu-sched-strategy=max-ilp "$@" --cuda-device-only -S "$SRC/gym-ctr-reach_amd/csrc/ctr_kernels.hip" -o "$OUT"
