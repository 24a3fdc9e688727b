"""Variant: scheduler A (aligned fixed J == 1: configs 2 and 5) with NWA waves
per workgroup instead of 16, still one workgroup per CU (the 160 KiB image).
The streaming shape ran faster at 12 waves per CU than at 16 on one box
(tools/diag/hbm_ceiling.hip OCC_SWEEP=1); this checks the engine.
    NWA=12 python tools/diag/abl_waves.py && make -C nvlevelz_amd/csrc variant NAME=w12 VSRC=$PWD/build/abl_w12.hip VFLAGS=-I$PWD/nvlevelz_amd/csrc"""
import os
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
s = open(os.path.join(R, "nvlevelz_amd/csrc/crc32c_kernels.hip")).read()
NWA = int(os.environ.get("NWA", "12"))


def rep(old, new, count=1):
    global s
    assert s.count(old) == count, (s.count(old), old[:60])
    s = s.replace(old, new)


# the region image fill for any thread count (guarded rounds)
rep("""struct RegionFill {
  uint32_t rep[8192 / kThreads];
  uint4 nib[2048 / kThreads];
};
__device__ __forceinline__ RegionFill fill_region_load(const uint32_t* __restrict__ g) {
  RegionFill f;""", """template <int NT = kThreads>
struct RegionFill {
  uint32_t rep[(8192 + NT - 1) / NT];
  uint4 nib[(2048 + NT - 1) / NT];
};
template <int NT = kThreads>
__device__ __forceinline__ RegionFill<NT> fill_region_load(const uint32_t* __restrict__ g) {
  constexpr int kThreads = NT;
  RegionFill<NT> f;""")
rep("""  for (int q = 0; q < (int)(8192 / kThreads); ++q) {
    const uint32_t off = (uint32_t)(t + q * (int)kThreads) << 4;
    const uint32_t tab""", """  for (int q = 0; q < (int)((8192 + kThreads - 1) / kThreads); ++q) {
    if (t + q * (int)kThreads >= 8192) break;
    const uint32_t off = (uint32_t)(t + q * (int)kThreads) << 4;
    const uint32_t tab""")
rep("""  for (int q = 0; q < (int)(2048 / kThreads); ++q) f.nib[q] = src[t + q * (int)kThreads];""",
    """  for (int q = 0; q < (int)((2048 + kThreads - 1) / kThreads); ++q)
    if (t + q * (int)kThreads < 2048) f.nib[q] = src[t + q * (int)kThreads];""")
rep("""__device__ __forceinline__ void fill_region_store(uint8_t* lds, const RegionFill& f, uint32_t ctr0) {
  const int t = threadIdx.x;""", """template <int NT = kThreads>
__device__ __forceinline__ void fill_region_store(uint8_t* lds, const RegionFill<NT>& f, uint32_t ctr0) {
  constexpr int kThreads = NT;
  const int t = threadIdx.x;""")
rep("""  for (int q = 0; q < (int)(8192 / kThreads); ++q) {
    const uint32_t off = (uint32_t)(t + q * (int)kThreads) << 4;
    *reinterpret_cast""", """  for (int q = 0; q < (int)((8192 + kThreads - 1) / kThreads); ++q) {
    if (t + q * (int)kThreads >= 8192) break;
    const uint32_t off = (uint32_t)(t + q * (int)kThreads) << 4;
    *reinterpret_cast""")
rep("""  for (int q = 0; q < (int)(2048 / kThreads); ++q) {
    uint4 v = f.nib[q];""", """  for (int q = 0; q < (int)((2048 + kThreads - 1) / kThreads); ++q) {
    if (t + q * (int)kThreads >= 2048) break;
    uint4 v = f.nib[q];""")
rep("""  if constexpr (NIB) fill_region_store(lds, fill_region_load(ka.tables), NW);""",
    """  if constexpr (NIB) fill_region_store<kWave * NW>(lds, fill_region_load<kWave * NW>(ka.tables), NW);""")
rep("""constexpr int waves_of() { return M == kGeneral ? kGenWaves : kWavesPerWG; }""",
    """constexpr int waves_of() { return M == kGeneral ? kGenWaves : %d; }""" % NWA)
rep("""      run_pairs<kFastU, kWavesPerWG, kAligned, FixedGeom, false, true>(g, ka, lds);""",
    """      run_pairs<kFastU, %d, kAligned, FixedGeom, false, true>(g, ka, lds);""" % NWA)
rep("""      hipExtLaunchKernelGGL(dev::crc32c_fixed_kernel<dev::kAligned>, dim3(grid), dim3(dev::kThreads), 0, lc.stream,""",
    """      hipExtLaunchKernelGGL(dev::crc32c_fixed_kernel<dev::kAligned>, dim3(grid), dim3(dev::kWave * %d), 0, lc.stream,""" % NWA)
rep("""      hipLaunchKernelGGL(dev::crc32c_fixed_kernel<dev::kAligned>, dim3(grid), dim3(dev::kThreads), 0, lc.stream, g,""",
    """      hipLaunchKernelGGL(dev::crc32c_fixed_kernel<dev::kAligned>, dim3(grid), dim3(dev::kWave * %d), 0, lc.stream, g,""" % NWA)
os.makedirs(os.path.join(R, "build"), exist_ok=True)
out = os.path.join(R, "build/abl_w%d.hip" % NWA)
open(out, "w").write(s)
print("wrote", out)
