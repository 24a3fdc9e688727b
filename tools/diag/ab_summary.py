"""Condense tools/diag/ab_variants.sh output ("variant {json}" lines) into a
table of per-call medians: one row per variant, one column per config."""
import json, sys
rows, cols = {}, []
for line in sys.stdin:
    if "{" not in line:
        continue
    v, j = line.split(" ", 1)
    d = json.loads(j)
    c = d["config"]
    if c not in cols:
        cols.append(c)
    rows.setdefault(v, {}).setdefault(c, []).append(d["median_us"] if d["ok"] else float("nan"))
print("variant " + " ".join(f"{c:>14s}" for c in cols))
for v, r in rows.items():
    print(f"{v:8s}" + " ".join(f"{'/'.join(f'{x:.1f}' for x in r.get(c, [])):>14s}" for c in cols))
