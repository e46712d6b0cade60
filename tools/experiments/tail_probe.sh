#!/bin/bash
# Experiment build (never the product): k_step with E extra workgroups appended to its grid that
# each spin T ns (s_memrealtime, 100 MHz) and exit, to measure whether the SIMDs that k_step's
# waves leave idle at the end of a launch can take work without lengthening it (the
# refill in k_step's tails).  E and T come from CTR_TAIL_WG / CTR_TAIL_NS in the host library
# (hipMemcpyToSymbol once).  Library: gym-ctr-reach_amd/ctr_reach_amd/lib/libab_tail.so
# (tools/tail_probe.py times it).  usage: bash tools/experiments/tail_probe.sh
set -euo pipefail
ROOT=$(git rev-parse --show-toplevel)
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
cp -r "$ROOT/gym-ctr-reach_amd/csrc" "$ROOT/gym-ctr-reach_amd/Makefile" "$TMP/"
mkdir -p "$TMP/include" && cp "$ROOT/include/ctr_reach_amd.h" "$TMP/include/"
python3 - "$TMP/csrc/ctr_kernels.hip" <<'EOF'
import sys
p = sys.argv[1]
s = open(p).read()
def sub(old, new):
    global s
    assert old in s, old
    s = s.replace(old, new, 1)
sub("template <int MODE>\n__global__ __launch_bounds__(BLOCK) void k_step(KCfg kc, ctr_batch_t b, const float *__restrict__ actions,\n"
    "                                                   ctr_step_out_t o, int32_t autoreset)\n{\n",
    "__device__ unsigned long long g_tail_ticks;\n"
    "template <int MODE>\n__global__ __launch_bounds__(BLOCK) void k_step(KCfg kc, ctr_batch_t b, const float *__restrict__ actions,\n"
    "                                                   ctr_step_out_t o, int32_t autoreset)\n{\n"
    "    {\n        const int64_t G = ((MODE & 6) == 6) ? SEG_GROUP : 1;\n"
    "        if ((int64_t)blockIdx.x * BLOCK >= b.n * G) {\n"
    "            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), tk = g_tail_ticks;\n"
    "            while (__builtin_amdgcn_s_memrealtime() - t0 < tk) __builtin_amdgcn_s_sleep(1);\n"
    "            return;\n        }\n    }\n")
sub("        CTR_LAUNCH(k_step, kc.mode, dim3(grid_for(lanes)), lane_lds_bytes(kc), s, kc, b, actions, o, autoreset);",
    "    {\n        static int extra = -1;\n        if (extra < 0) {\n"
    "            const char *w = getenv(\"CTR_TAIL_WG\"), *t = getenv(\"CTR_TAIL_NS\");\n"
    "            extra = w ? atoi(w) : 0;\n"
    "            unsigned long long ticks = t ? (unsigned long long)(atoll(t) / 10) : 0ull;\n"
    "            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tail_ticks), &ticks, sizeof ticks);\n        }\n"
    "        CTR_LAUNCH(k_step, kc.mode, dim3(grid_for(lanes) + extra), lane_lds_bytes(kc), s, kc, b, actions, o, autoreset);\n    }")
s = s.replace("#include <algorithm>", "#include <algorithm>\n#include <stdlib.h>", 1)
open(p, "w").write(s)
EOF
rm -f "$ROOT/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_tail.so"
make -C "$TMP" -s LIB="$ROOT/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_tail.so" \
    HIPFLAGS="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -I$TMP/include -Icsrc -mllvm -amdgpu-sched-strategy=max-ilp" \
    DEPS= "$ROOT/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_tail.so"
echo "built libab_tail.so"
