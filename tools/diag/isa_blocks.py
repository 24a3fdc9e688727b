"""Per-basic-block instruction mix of one kernel in a hipcc -S listing.
    python tools/diag/isa_blocks.py k.s <kernel-substring>
Prints each block: label, #VALU, #SALU, #LDS, #VMEM, #other, successors."""
import re, sys
src, pat = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % pat, l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur = [], None
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\d+_\d+|_Z\S+):", l)
    if m:
        cur = {"name": m.group(1)[:24], "v": 0, "s": 0, "ds": 0, "vm": 0, "o": 0, "succ": []}
        blocks.append(cur); continue
    t = l.strip()
    if not t or t.startswith((";", ".")) or cur is None:
        continue
    op = t.split()[0]
    if op.startswith("v_"): cur["v"] += 1
    elif op.startswith("s_cbranch") or op == "s_branch":
        cur["succ"].append(t.split()[-1]); cur["s"] += 1
    elif op.startswith("s_"): cur["s"] += 1
    elif op.startswith("ds_"): cur["ds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_", "scratch_")): cur["vm"] += 1
    else: cur["o"] += 1
tot = {k: sum(b[k] for b in blocks) for k in ("v", "s", "ds", "vm")}
print("total", tot, "blocks", len(blocks))
for b in blocks:
    print(f'{b["name"]:>24} v{b["v"]:5d} s{b["s"]:4d} ds{b["ds"]:4d} vm{b["vm"]:3d} -> {",".join(b["succ"])}')
