"""(host) Static instruction census of one kernel in the generated assembly
(`make -C marl-nav_amd/csrc asm` -> marl-nav_amd/lib/marlnav_step.s), split at
its s_barrier instructions (the block kernel's phase boundaries), and, inside
each segment, per basic block, so that the code a phase actually runs can be
told from the rare paths (IEEE fallbacks, partial blocks, finished-env tails).

usage: python scripts/static_census.py [kernel-substring] [asm]
       default: the headline block_kernel<3,3,false,false>"""
import collections
import re
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
name = sys.argv[1] if len(sys.argv) > 1 else "block_kernelILi3ELi3ELb0ELb0E"
path = sys.argv[2] if len(sys.argv) > 2 else ROOT + "/marl-nav_amd/lib/marlnav_step.s"

TRANS = ("v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_", "v_exp_", "v_log_")


def kind(op):
    if op.startswith("v_"):
        if op.startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
            return "VALU"
        if op.startswith(TRANS):
            return "VALU.trans"
        if "_f64" in op:
            return "VALU.f64"
        if op.startswith(("v_mad_u64_u32", "v_mad_i64_i32")):
            return "VALU.mad64"
        return "VALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_load", "buffer_load", "scratch_load", "flat_load")):
        return "VMEM.rd"
    if op.startswith(("global_store", "buffer_store", "scratch_store", "flat_store", "global_atomic")):
        return "VMEM.wr"
    if op.startswith(("s_load", "s_buffer_load")):
        return "SMEM"
    if op in ("s_waitcnt", "s_barrier", "s_nop", "s_endpgm", "s_setprio") or op.startswith(
            ("s_cbranch", "s_branch", "s_sleep")):
        return "ctl"
    if op.startswith("s_"):
        return "SALU"
    return "other"


lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(name) + r"\S*:", l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
segs = [collections.OrderedDict()]  # segment -> {block label: Counter}
block = "entry"
for l in lines[start + 1:end]:
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        block = m.group(1)
        continue
    if not l.startswith("\t") or l.strip().startswith((".", ";")):
        continue
    op = l.split()[0]
    segs[-1].setdefault(block, collections.Counter())[kind(op)] += 1
    if op == "s_barrier":
        segs.append(collections.OrderedDict())
        block = block + "'"
cols = ["VALU", "VALU.trans", "VALU.f64", "VALU.mad64", "SALU", "LDS", "VMEM.rd", "VMEM.wr", "SMEM", "ctl"]
print(f"{name}: {len(segs) - 1} barriers")
print("segment/block".ljust(24) + "".join(f"{c:>11s}" for c in cols))
for k, seg in enumerate(segs):
    tot = collections.Counter()
    for b, c in seg.items():
        tot.update(c)
    print(f"seg {k} total".ljust(24) + "".join(f"{tot[c]:11d}" for c in cols))
    for b, c in seg.items():
        if sum(c.values()) >= 8:
            print(f"  {b}".ljust(24) + "".join(f"{c[x]:11d}" for x in cols))
