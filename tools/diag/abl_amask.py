"""Variant: fixed-stride batches of one partial chunk per buffer (1025..4095 B)
through scheduler A with masked passes (load_general / realign_general with
hd = true, as the head kernel's drain does) instead of the head kernel.
Experiment only: the masked loads read up to 12 bytes below a buffer's first
16-byte granule, so a buffer starting in a page's first granule is unsafe --
time it on layouts where none does (tools/bench_configs.py config f).
    python tools/diag/abl_amask.py && make -C nvlevelz_amd/csrc variant NAME=amask VSRC=$PWD/build/abl_amask.hip VFLAGS=-I$PWD/nvlevelz_amd/csrc"""
import os
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
s = open(os.path.join(R, "nvlevelz_amd/csrc/crc32c_kernels.hip")).read()
def rep(old, new):
    global s
    assert old in s, old[:60]
    s = s.replace(old, new, 1)
rep("enum LoadMode : int { kAligned = 0, kGeneral = 1 };", "enum LoadMode : int { kAligned = 0, kGeneral = 1, kMasked = 2 };")
rep("""  } else {
    load_general(ce, false, (uintptr_t)bi.p, lane, ch);
  }""", """  } else {
    load_general(ce, M == kMasked, (uintptr_t)bi.p, lane, ch);
  }""")
rep("""    realign_general(chunk_end(bi, c), false, (uintptr_t)bi.p, bi.s, lane, ch, w);""",
    """    realign_general(chunk_end(bi, c), M == kMasked, (uintptr_t)bi.p, bi.s, lane, ch, w);""")
rep("""    if (g.J == 1 && !head_first(g.len)) {
      run_pairs<kGenPairU, waves_of<M>(), kGeneral>(g, ka, lds);
      return;
    }""", """    if (g.J == 1 && !head_first(g.len)) {
      run_pairs<kGenPairU, waves_of<M>(), kGeneral>(g, ka, lds);
      return;
    }
    if (g.J == 1 && g.len >= 1025) {
      run_pairs<kGenPairU, waves_of<M>(), kMasked>(g, ka, lds);
      return;
    }""")
rep("""  const bool heads = !aligned && dev::head_first(len);  // every buffer's first chunk is a head chunk""",
    """  const bool heads = !aligned && dev::head_first(len) && !(J == 1 && len >= 1025);""")
os.makedirs(os.path.join(R, "build"), exist_ok=True)
open(os.path.join(R, "build/abl_amask.hip"), "w").write(s)
print("wrote build/abl_amask.hip")
