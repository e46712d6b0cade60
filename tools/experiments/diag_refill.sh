#!/bin/bash
# Diagnostic build (never the product): k_refill with per-wave clock stamps (s_memrealtime, 100 MHz) at its
# phase boundaries, written with vector stores (every lane of the wave, lane-indexed) into a device
# array whose address the host tool puts into the carry header's padding (needs the carry lists).
# The working tree's sources are copied and patched in a temporary directory; the library goes to
# gym-ctr-reach_amd/ctr_reach_amd/lib/libab_diag.so (tools/diag_refill.py reads it).
# usage: bash tools/experiments/diag_refill.sh
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
# stamps: g_diag[wave][phase], wave = blockIdx * 4 + wave in block; lane 0 stores (vector store:
# the address depends on threadIdx)
sub("constexpr int BLOCK = 256;",
    "constexpr int BLOCK = 256;\n"
    "#define DIAG(ph) do { const unsigned long long _t = __builtin_amdgcn_s_memrealtime(); "
    "if (dgp && blockIdx.x < 256) "
    "dgp[((blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (ph)) * 64 + (threadIdx.x & 63)] = _t; } while (0)")
# the stamp array's address: bytes 520..527 of the carry header (its padding), set by the host tool
sub("    CarryHdr *ch = static_cast<CarryHdr *>(b.carry);\n",
    "    CarryHdr *ch = static_cast<CarryHdr *>(b.carry);\n"
    "    unsigned long long *dgp = ch ? *reinterpret_cast<unsigned long long *const *>(reinterpret_cast<const char *>(ch) + 520) : nullptr;\n"
    "    DIAG(0);\n")
sub("    __syncthreads();\n    CarryRec *recs",
    "    __syncthreads();\n    DIAG(1);\n    CarryRec *recs")
sub("            stat |= CTR_STATUS_SAMPLER_STUCK;\n        stat |= __shfl_xor(stat, 1);",
    "            stat |= CTR_STATUS_SAMPLER_STUCK;\n        DIAG(2);\n        stat |= __shfl_xor(stat, 1);")
sub("        } else if (fresh || carried) {\n            // a reset at least",
    "        }\n        DIAG(3);\n        if (had) {\n        } else if (fresh || carried) {\n            // a reset at least")
sub("            fst = st.status;\n        }\n        const bool active = fresh || carried;",
    "            fst = st.status;\n        }\n        DIAG(4);\n        const bool active = fresh || carried;")
sub("    // the last workgroup to finish clears the queue and the list it read",
    "    DIAG(5);\n    // the last workgroup to finish clears the queue and the list it read")
# k_step (the compliant one-env-per-lane path): stamps after the array's first half
sub("    StageRegs stg;\n",
    "    unsigned long long *dgp = b.carry ? *reinterpret_cast<unsigned long long *const *>("
    "reinterpret_cast<const char *>(b.carry) + 520) : nullptr;\n"
    "    if (dgp) dgp += 1024 * 8 * 64;\n    DIAG(0);\n    StageRegs stg;\n")
sub("    stage_systems<!GROUP>(kc, s_sys, s_raw, &stg);\n",
    "    stage_systems<!GROUP>(kc, s_sys, s_raw, &stg, dgp);\n    DIAG(1);\n")
sub("        set_action_substeps(sy, kc.c.constrain_alpha != 0, kc.c.n_substeps, q, a_in);\n        FkStats st",
    "        set_action_substeps(sy, kc.c.constrain_alpha != 0, kc.c.n_substeps, q, a_in);\n        DIAG(2);\n        FkStats st")
sub("        fk_dispatch<MODE>(kc, episode_sys(kc, s_sys, s_raw, s, ep_in, (uint64_t)(b.env_base + e)), q, ag, st);\n",
    "        fk_dispatch<MODE>(kc, episode_sys(kc, s_sys, s_raw, s, ep_in, (uint64_t)(b.env_base + e)), q, ag, st);\n"
    "        DIAG(3);\n")
sub("                    s_fin_ep[threadIdx.x], dg_f);\n",
    "                    s_fin_ep[threadIdx.x], dg_f);\n        DIAG(4);\n")
# k_step's end, after the refill-queue append (slot 7)
sub("            wave_append(b.refill, b.refill + 1, b.refill_cap, fl.pooled, two, 2);\n        }\n    }\n}",
    "            wave_append(b.refill, b.refill + 1, b.refill_cap, fl.pooled, two, 2);\n        }\n    }\n    DIAG(7);\n}")
# staging sub-phases in k_step (slots 5: tables copied + barrier, 6: SysK derived + barrier)
sub("                                              const StageRegs *pre = nullptr)\n{",
    "                                              const StageRegs *pre = nullptr, unsigned long long *dgp = nullptr)\n{")
# (one barrier since the SysK divisions come from the kernel config: slot 6 = slot 5)
sub("            e[7] = (double)q.present;\n        }\n    }\n    __syncthreads();\n",
    "            e[7] = (double)q.present;\n        }\n    }\n    __syncthreads();\n    DIAG(5);\n    DIAG(6);\n")
open(p, "w").write(s)
EOF
if [ "${ASM:-0}" = 1 ]; then
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -I"$TMP/include" -I"$TMP/csrc" -mllvm -amdgpu-sched-strategy=max-ilp \
    --cuda-device-only -S "$TMP/csrc/ctr_kernels.hip" -o /tmp/diag_refill.s
  echo "asm in /tmp/diag_refill.s"; exit 0
fi
rm -f "$ROOT/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_diag.so"
make -C "$TMP" -s LIB="$ROOT/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_diag.so" \
    HIPFLAGS="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -I$TMP/include -Icsrc -mllvm -amdgpu-sched-strategy=max-ilp" \
    DEPS= "$ROOT/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_diag.so"
echo "built libab_diag.so"
