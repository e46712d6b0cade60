"""Instruction census of k_step's RK45 attempt blocks from a hipcc -S listing.

usage: make -C gym-ctr-reach_amd asm  (writes /tmp/ctr_kernels.s)
       python tools/attempt_census.py /tmp/ctr_kernels.s [out.json]

Finds the attempt block of each tube level in k_step<0> (the non-careful FK variant, which every
wave of the headline workload runs): the level-3 block issues 12 table sincos (12 ds_read_b128:
two per RHS), level 2 six, level 1 none (level 3 holds 18 v_rcp_f64 of the error norm, level 2
16, level 1 13).  Opcodes are counted exactly; the FP64 arithmetic is split into algorithmic, sincos and
controller work by the source's operation counts (csrc/ctr_device.hpp rk45_attempt):
  sincos     per angle: 1 mul + 2 fma reduction + 1 mul (z) + 2 fma (polys) + 1 mul (r z) +
             2 fma (sin r, cos r) + 2 mul + 2 fma (table combine) = 13 FP64 ops, + v_rndne,
             v_cvt_i32, v_and (index & 511), v_lshl (byte offset), ds_read_b128 (table entry)
  controller per error-norm component: v_max_f64 (absmax) + fma (atol + m rtol) + v_rcp_f64;
             inv_root10 (frexp / ldexp / f32 log, exp, cvts); min_step / step-size selects
  algorithmic the rest of the FP64 FMA / MUL / ADD (stage sums, RHS, y_new, error sums, norm)
"""
import collections
import json
import re
import sys

K = "_ZN12_GLOBAL__N_16k_stepILi0EEEvNS_4KCfgE11ctr_batch_tPKf14ctr_step_out_ti"


def blocks(path, kern):
    lines = open(path).read().split("\n")
    start = [i for i, l in enumerate(lines) if l.startswith(kern + ":")][0]
    out, cur, name = {}, None, None
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            name = m.group(1)
            cur = out.setdefault(name, [])
            continue
        t = l.strip()
        if cur is None or not t or t.startswith((";", ".")):
            continue
        cur.append(t.split()[0])
    return out


def census(ops):
    c = collections.Counter(ops)
    n_rd = c["ds_read_b128"]
    angles = n_rd                           # one 16-B table entry (sin, cos) per angle
    fp64 = sum(c[o] for o in c if re.match(r"v_(fmac?|mul|add)_f64", o))
    n_rcp = c["v_rcp_f64_e32"]
    sincos_fp64 = 13 * angles
    sincos_other = sum(c[o] for o in ("v_rndne_f64_e32", "v_cvt_i32_f64_e32")) + 2 * angles + n_rd
    ctrl_fp64 = n_rcp                       # the fma(absmax, rtol, atol) of each component
    ctrl_other = (n_rcp + c["v_max_f64"] + sum(c[o] for o in c if o.startswith(("v_frexp", "v_ldexp", "v_log_f32",
                                                                                  "v_exp_f32", "v_cvt_f32_f64",
                                                                                  "v_cvt_f64_f32", "v_mul_f32"))))
    agpr = sum(c[o] for o in c if o.startswith("v_accvgpr"))
    cnd = sum(c[o] for o in c if o.startswith("v_cndmask"))
    smov = sum(c[o] for o in c if o.startswith(("s_mov_b32", "s_mov_b64")))
    nops = sum(c[o] for o in c if o.startswith(("s_nop", "s_waitcnt")))
    total = sum(c.values())
    cat = {
        "algorithmic_fp64": fp64 - sincos_fp64 - ctrl_fp64,
        "sincos_fp64": sincos_fp64,
        "sincos_index_lds": sincos_other,
        "controller_rcp_max_scale_root": ctrl_fp64 + ctrl_other,
        "selects_v_cndmask": cnd,
        "agpr_moves": agpr,
        "salu_constant_s_mov": smov,
        "s_nop_s_waitcnt": nops,
    }
    cat["other_int_cvt_cmp_branch_exec"] = total - sum(cat.values())
    return {"instructions": total, "sincos_angles": angles, "error_norm_components": n_rcp,
            "categories": cat, "categories_frac": {k: round(v / total, 4) for k, v in cat.items()},
            "opcodes": dict(sorted(c.items(), key=lambda kv: -kv[1]))}


if __name__ == "__main__":
    bl = blocks(sys.argv[1], K)
    found = {}
    for name, ops in bl.items():
        c = collections.Counter(ops)
        if len(ops) < 400 or c["v_rcp_f64_e32"] < 12 or c["v_rsq_f64_e32"]:
            continue
        # (level, error-norm components, table reads): L3 18 / 12, L2 16 / 6, L1 13 / 0
        lv = {(18, 12): 3, (16, 6): 2, (13, 0): 1}.get((c["v_rcp_f64_e32"], c["ds_read_b128"]))
        if lv:                  # the last one in the listing: the non-careful FK comes after the careful one
            found[lv] = (name, ops)
    out = {"listing": sys.argv[1], "kernel": K,
           "levels": {"L%d" % lv: dict(block=found[lv][0], **census(found[lv][1])) for lv in sorted(found)}}
    js = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(js + "\n")
    for k, v in out["levels"].items():
        print(k, v["block"], v["instructions"], v["categories"])
