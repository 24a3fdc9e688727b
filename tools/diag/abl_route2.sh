#!/bin/bash
# (For the tree with tools/diag/route_noplan.patch applied -- the rejected
# plan-free routing.)  Where the plan-free routed call's time goes (timed by tools/diag/ab_region.py
# with AB_FLAGS=0, region-shaped batches): `nofused` -- no body-kernel launch;
# `noproof` -- the workgroups publish "proved" without searching or walking;
# `nogate` -- the fold does not wait for the gate; `noabort` -- no early look
# at the other parts; `bare` -- all four; `base` -- unedited.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p $R/build
SRC=$R/nvlevelz_amd/csrc/crc32c_kernels.hip
python3 - "$SRC" "$R/build" <<'PY'
import sys
src, out = sys.argv[1], sys.argv[2]
s = open(src).read()
fused = "  if (lc.ev_stop)\n    hipExtLaunchKernelGGL(dev::crc32c_var_fused_kernel,"
proof = "    bool wbad = wv == 0 && !route_ends_ok(g, blockIdx.x, G, own);"
walk = "    wbad = wbad || __ballot(walk_bad(g, ka.route, own, j0, ww, lane)) != 0u;"
gate = "    if (!gate_eval(g, ka.route, G, lane, gq, kGateSpin)) return false;  // some range not region-shaped"
abort_ = "      if (wv == 0 && ++iter == 2u && gate_any_failed(ka.route, G, lane) && lane == 0)"
for a in (fused, proof, walk, gate, abort_):
    assert s.count(a) == 1, a
ed = {
    "nofused": [(fused, "  if (true) return hipSuccess;\n" + fused)],
    "noproof": [(proof, "    bool wbad = false; (void)ww;"), (walk, "    if (false)" + walk[4:])],
    "nogate": [(gate, "    (void)gq;")],
    "noabort": [(abort_, "      if (false && wv == 0 && ++iter == 2u && gate_any_failed(ka.route, G, lane) && lane == 0)")],
}
ed["bare"] = sum(ed.values(), [])
ed["base"] = []
for name, reps in ed.items():
    t = s
    for a, b in reps:
        t = t.replace(a, b)
    open(out + "/abl_%s.hip" % name, "w").write(t)
PY
for v in nofused noproof nogate noabort bare base; do
  make -C $R/nvlevelz_amd/csrc variant NAME=$v VSRC=$R/build/abl_$v.hip VFLAGS="-I$R/nvlevelz_amd/csrc" > /dev/null &
done
wait
ls $R/build/libnvl_crc32c_{nofused,noproof,nogate,noabort,bare,base}.so
