"""Basic-block instruction census of one kernel in a hipcc -S listing (gfx950).

usage: python tools/asm_blocks.py listing.s <kernel-substring> [min_block_instrs]
Prints each basic block (label, #instructions, class mix) and the backward branches (loops)."""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_accvgpr"):
        return "agpr"
    if op.startswith(("v_fma_f64", "v_fmac_f64")):
        return "fma64"
    if op.startswith("v_mul_f64"):
        return "mul64"
    if op.startswith("v_add_f64"):
        return "add64"
    if op.startswith(("v_rcp_f64", "v_rsq_f64", "v_sqrt_f64", "v_frexp", "v_ldexp", "v_exp_f32", "v_log_f32", "v_rcp_f32")):
        return "trans"
    if op.startswith("v_cndmask"):
        return "cndmask"
    if op.startswith(("v_mov", "v_pk_mov")):
        return "vmov"
    if op.startswith("v_cmp"):
        return "vcmp"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait/nop"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path, kname = sys.argv[1], sys.argv[2]
    minn = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^\S*%s\S*:" % re.escape(kname), l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    blocks, cur, order = {}, "entry", ["entry"]
    blocks[cur] = []
    for l in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            continue
        blocks[cur].append(s.split()[0])
    idx = {b: i for i, b in enumerate(order)}
    tot = Counter()
    for b in order:
        ops = blocks[b]
        c = Counter(classify(o) for o in ops)
        tot.update(c)
        if len(ops) >= minn:
            print("%-14s %5d  %s" % (b, len(ops), " ".join("%s=%d" % kv for kv in c.most_common())))
    print("TOTAL", sum(tot.values()), dict(tot.most_common()))
    # loops: branches to an earlier block
    for b in order:
        pass
    text = "\n".join(lines[start:end])
    for m in re.finditer(r"^(\.LBB\S+):", text, re.M):
        pass
    cur = "entry"
    for l in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            cur = m.group(1)
            continue
        mm = re.match(r"\s*s_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if mm and mm.group(2) in idx and idx[mm.group(2)] <= idx[cur]:
            span = order[idx[mm.group(2)]:idx[cur] + 1]
            n = sum(len(blocks[x]) for x in span)
            print("loop %s -> %s: %d blocks, %d instrs" % (cur, mm.group(2), len(span), n))


if __name__ == "__main__":
    main()
