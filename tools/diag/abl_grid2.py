"""Variant: scheduler A (aligned fixed J == 1, chunk-parallel) launched with two
workgroups per CU (two dispatch rounds: the second round's workgroups go to
whichever CUs of an XCD free up first) instead of one.
    python tools/diag/abl_grid2.py && make -C nvlevelz_amd/csrc variant NAME=grid2 VSRC=$PWD/build/abl_grid2.hip VFLAGS=-I$PWD/nvlevelz_amd/csrc"""
import os
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
s = open(os.path.join(R, "nvlevelz_amd/csrc/crc32c_kernels.hip")).read()


def rep(old, new):
    global s
    assert s.count(old) == 1, old[:60]
    s = s.replace(old, new)


rep("""    const uint32_t gc = grid_for(lc.num_cu, T);""", """    const uint32_t gc = grid_for(2 * lc.num_cu, T);""")
rep("""  if (aligned) {
    if (timed)
      hipExtLaunchKernelGGL(dev::crc32c_fixed_kernel<dev::kAligned>, dim3(grid),""",
    """  const uint32_t grid2 = J == 1 ? grid_for(2 * lc.num_cu, n) : grid;
  if (aligned) {
    if (timed)
      hipExtLaunchKernelGGL(dev::crc32c_fixed_kernel<dev::kAligned>, dim3(grid2),""")
rep("""      hipLaunchKernelGGL(dev::crc32c_fixed_kernel<dev::kAligned>, dim3(grid), dim3(dev::kThreads), 0, lc.stream, g,""",
    """      hipLaunchKernelGGL(dev::crc32c_fixed_kernel<dev::kAligned>, dim3(grid2), dim3(dev::kThreads), 0, lc.stream, g,""")
os.makedirs(os.path.join(R, "build"), exist_ok=True)
open(os.path.join(R, "build/abl_grid2.hip"), "w").write(s)
print("wrote build/abl_grid2.hip")
