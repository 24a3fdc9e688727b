"""Ablations of the region kernel's per-buffer work (round 6): where do `r` /
`v` lose against config 2's rate?  Writes edited copies of
nvlevelz_amd/csrc to build/abl_<name>/ and builds each as
build/libnvl_crc32c_abl_<name>.so (`make variant`); time them with
tools/diag/ab_region.py (AB_FLAGS=2: the region kernel alone).  Results are
WRONG for every variant but `base` (NVL_CRC32C_SELFTEST_REPORT_ONLY=1).

  nofoldmath  the fold keeps its loads (records, raws, quads) but no arithmetic
  nofold      no fold phase at all (no barrier, no stores)
  noevents    nofold + no event records in the unit loop
  nowin       noevents + no metadata windows / searches (pure region streaming)
  nostores    nofold + the event records computed but not stored
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "nvlevelz_amd", "csrc")
H = "crc32c_dev_region.h"


def rep(text, old, new, count=1):
    assert text.count(old) == count, (old[:60], text.count(old))
    return text.replace(old, new)


def nofoldmath(t):
    return rep(t, "        if (!(f.fast && fold_out(g, lds, lsl, lb, lane, f, q_s, q_e, (uint32_t)i, v)))\n"
                  "          v = serial_raw(ka.tables + kGSlice, f.ninit, g.grid + f.s, f.L);",
               "        v = q_s.x ^ q_e.y ^ g.raws[f.s >> 12] ^ f.vs[1] ^ f.ve[2] ^ f.xs ^ f.xe ^ f.xt;")


def nofold(t):
    return rep(t, "  NVL_TL(2);\n  uint32_t r;\n", "  NVL_TL(2);\n  if (ka.flags != 12345u) return;\n  uint32_t r;\n")


def noevents(t):
    t = nofold(t)
    return rep(t, "      region_events<U>(g, w, cursor, ca, cu, pre, Lf, cp, le, lane);",
               "      if (ka.flags == 12345u) region_events<U>(g, w, cursor, ca, cu, pre, Lf, cp, le, lane);")


def nowin(t):
    t = noevents(t)
    t = rep(t, "  uint64_t cursor = cu ? region_search(g, ca * kChunk, lane, probe) : g.n;",
            "  uint64_t cursor = g.n; (void)probe;")
    t = rep(t, "    if (cun && un < nunits) {  // the next", "    if (false) {  // the next")
    t = rep(t, "    const bool any_ev = !halo && __ballot(le.sv || le.ev) != 0u;",
            "    const bool any_ev = false; (void)le;")
    return t


def nostores(t):
    """nofold + the event records computed but not stored (the stores' own cost)"""
    t = nofold(t)
    t = rep(t, "    if (fs) g.qs[cur + (uint64_t)lane] = ", "    if (fs && g.gen == 0u) g.qs[cur + (uint64_t)lane] = ")
    t = rep(t, "    if (fe) g.qe[cur + (uint64_t)lane] = ", "    if (fe && g.gen == 0u) g.qe[cur + (uint64_t)lane] = ")
    t = rep(t, "        if (lane == 0) (t ? g.qe : g.qs)[cur + j] = r;", "        if (lane == 0 && g.gen == 0u) (t ? g.qe : g.qs)[cur + j] = r;")
    return t


VARIANTS = {"base": lambda t: t, "nofoldmath": nofoldmath, "nofold": nofold, "noevents": noevents, "nowin": nowin,
            "nostores": nostores}

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    for name in names:
        d = os.path.join(ROOT, "build", "abl_" + name)
        shutil.rmtree(d, ignore_errors=True)
        shutil.copytree(SRC, d)
        p = os.path.join(d, H)
        with open(p) as f:
            t = f.read()
        with open(p, "w") as f:
            f.write(VARIANTS[name](t))
        subprocess.run(["make", "-s", "-C", SRC, "variant", "NAME=abl_" + name, "VDIR=" + d], check=True)
        print("built", name, flush=True)
