"""Ablation variants of the head kernel's drain (timing only, wrong results):
  mconst  the slot metadata (offset, length, ~init) computed from the index for
          the layout of tools/bench_configs.py config v (10^5 x 4097 B at
          stride 4101) instead of scalar loads -- run on config v only
  mnohc   mconst, and the kTInj passes' hc[i] not loaded (0)
    python tools/diag/abl_meta.py && for v in mconst mnohc; do make -C nvlevelz_amd/csrc variant NAME=$v VSRC=$PWD/build/abl_$v.hip VFLAGS=-I$PWD/nvlevelz_amd/csrc; done"""
import os
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(R, "nvlevelz_amd/csrc/crc32c_kernels.hip")).read()


def rep(s, old, new):
    assert s.count(old) == 1, old[:60]
    return s.replace(old, new)


mc = rep(src, """    o = ldc(offsets, i);
    Llo = ldc(reinterpret_cast<const uint32_t*>(lengths), 2 * i);
    s = ~(init ? ldc(init, i) : init_all);""", """    o = i * 4101ull;
    Llo = 4097u;
    s = ~init_all;""")
mn = rep(mc, """    return __builtin_nontemporal_load((const __attribute__((address_space(1))) uint32_t*)a);""",
         """    (void)a;
    return 0u;""")
os.makedirs(os.path.join(R, "build"), exist_ok=True)
for name, s in (("mconst", mc), ("mnohc", mn)):
    open(os.path.join(R, f"build/abl_{name}.hip"), "w").write(s)
    print(f"wrote build/abl_{name}.hip")
