"""Instruction accounting of a kernel's steady-state loop (the last loop of its body)
from hipcc's gfx950 assembly: every instruction listed with a category, counts per
category.  Usage:
  hipcc ... --cuda-device-only -S -o k.s gym-lorenz_amd/csrc/lz_kernels.hip
  python tools/isa_account.py k.s <mangled kernel name> > report.md
Categories are by opcode and operand (the loop's role for each is in the listing)."""
import collections
import re
import sys


def loop_of(asm, name):
    i = asm.index(name + ":")
    j = asm.index(".Lfunc_end", i)
    body = asm[i:j].split("\n")
    labels = {l.split(":")[0]: n for n, l in enumerate(body) if l.startswith(".LBB")}
    loops = []
    for n, l in enumerate(body):
        t = l.strip()
        if t.startswith(("s_cbranch", "s_branch")):
            tgt = t.split()[-1]
            if tgt in labels and labels[tgt] < n:
                loops.append((labels[tgt], n))
    a, b = max(loops)
    return [l.strip() for l in body[a:b + 1]]


def category(ins):
    op = ins.split()[0]
    if op.startswith("global_load_lds") or "m0" in ins or (op == "s_nop" and False):
        return "action DMA (LDS-DMA + M0 save/set/restore)"
    if op.startswith("ds_read"):
        return "action LDS read"
    if op == "s_waitcnt":
        return "waits"
    if op == "s_nop":
        return "hazard nops"
    if op.startswith("global_store"):
        return "stores (obs half-row, reward, done)"
    if op.startswith(("v_cmp", "v_cndmask")):
        return "compares / selects (action clip, lane roles)"
    if op.startswith(("v_add_f32", "v_sub_f32", "v_mul_f32", "v_pk_", "v_fma")) or "f32" in op and op.startswith("v_"):
        return "env arithmetic (RHS, Euler update, obs, reward)"
    if op.startswith(("v_mov",)):
        return "register moves"
    if op.startswith(("v_lshl_add_u64", "v_add_u32", "v_lshl_or", "v_add_co")):
        return "address arithmetic (VALU)"
    if op.startswith(("s_and_saveexec", "s_or_saveexec", "s_xor_b64", "s_or_b64", "s_andn2", "s_cbranch_execz")):
        return "exec-mask control (lead / partner lane stores)"
    if op.startswith(("s_cbranch", "s_branch", "s_cmp", "s_cselect")):
        return "loop control"
    if op.startswith("s_"):
        return "scalar bookkeeping (slot index, counters)"
    if op.startswith("v_xor"):
        return "env arithmetic (RHS, Euler update, obs, reward)"
    return "other"


def main():
    asm = open(sys.argv[1]).read()
    name = sys.argv[2]
    lines = [l for l in loop_of(asm, name) if l and not l.startswith((";", ".")) and not l.endswith(":")]
    cats = collections.Counter()
    print("## %s: steady-state loop, %d instructions per step\n" % (name, len(lines)))
    print("| # | instruction | category |\n|---|---|---|")
    for n, l in enumerate(lines):
        c = category(l)
        cats[c] += 1
        print("| %d | `%s` | %s |" % (n, re.sub(r"\s+", " ", l.split(";")[0]).strip(), c))
    print("\n| category | count |\n|---|---|")
    for c, v in cats.most_common():
        print("| %s | %d |" % (c, v))


if __name__ == "__main__":
    main()
