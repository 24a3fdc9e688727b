"""Register budget of the gfx950 kernels (CPU: hipcc cross-compiles).

Every hot kernel runs 1024-thread workgroups at one workgroup per CU, so it has
128 VGPRs per lane.  A change that pushes one past that spills to scratch in
the main loop -- e.g. the fused variable-length kernel once kept its 64-bit
chunk range in VGPRs and went from 287 to 430 us on config 3 with 25 spilled
VGPRs.  The compiler's resource-usage remarks catch that without a GPU."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HIPCC = "/opt/rocm/bin/hipcc"
CSRC = os.path.join(ROOT, "nvlevelz_amd", "csrc")
# the kernel TUs (crc32c_kernels.hip until round 5)
KERNEL_TUS = ["crc32c_fixed.hip", "crc32c_batch.hip", "crc32c_region.hip", "crc32c_misc.hip"]


@pytest.fixture(scope="module")
def usage(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    kernels = {}
    for tu in KERNEL_TUS:
        out = tmp_path_factory.mktemp("ru") / (tu + ".o")
        r = subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "--offload-arch=gfx950",
                            "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-c",
                            os.path.join(CSRC, tu), "-o", str(out),
                            "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        _parse(r.stderr, kernels)
    return kernels


def _parse(stderr, kernels):
    cur = None
    for line in stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            kernels[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
        if m and cur:
            kernels[cur][m.group(1).strip()] = int(m.group(2))
    return kernels


HOT = ["crc32c_fixed_kernelILi0", "crc32c_fixed_kernelILi1", "crc32c_fixed_long_kernel", "crc32c_var_kernel", "crc32c_var_fused_kernel",
       "crc32c_region_kernel", "crc32c_chunks_kernel",
       "crc32c_plan_small", "crc32c_fixup_kernel", "crc32c_head_kernel", "crc32c_route_kernel", "crc32c_route_plan"]
# SGPR spills go to VGPR lanes (v_writelane/v_readlane), not memory: a bound
# per kernel so that a jump shows.  The fused kernel parks plan-phase scalars
# there; the variable-length kernels keep scheduler C's two chunk positions
# (current pair, next pair) in SGPRs; the head kernel keeps two items'
# metadata (current, next) live in SGPRs while the next-but-one's loads are in
# flight.
SGPR_SPILL_MAX = {"crc32c_var_fused_kernel": 48, "crc32c_var_kernel": 48, "crc32c_head_kernel": 160,
                  "crc32c_route_kernel": 48}  # (the head kernel's and the region kernel's scalars in one kernel)


@pytest.mark.parametrize("name", HOT)
def test_no_vgpr_spills(usage, name):
    hits = [k for k in usage if name in k]
    assert hits, f"kernel {name} not found in {sorted(usage)}"
    for k in hits:
        u = usage[k]
        assert u.get("VGPRs Spill", 0) == 0, (k, u)
        assert u.get("SGPRs Spill", 0) <= SGPR_SPILL_MAX.get(name, 16), (k, u)
        assert u.get("ScratchSize", 0) <= 32, (k, u)  # a small indexed private array, no spill area


def test_region_fold_claim_placement(usage):
    """The region fold deals its slices by SIMD (slice k to the waves on SIMD
    k mod 4, crc32c_dev_region.h run_region).  Correctness does not depend on
    where the 16 waves land: a SIMD that holds none of them has its slices
    adopted by the lowest populated SIMD's waves.  The balance
    does: above 102 VGPRs (512 per lane and SIMD, granule 8) a SIMD takes at
    most 4 waves, so the 16 sit 4 per SIMD and every SIMD folds a quarter."""
    # run_region runs in crc32c_region_kernel (the one-launch form) and in
    # crc32c_route_kernel (the routed region_dev / batch_dev default, ADVICE
    # r05): both must keep the 4-waves-per-SIMD placement.
    for name in ("crc32c_region_kernel", "crc32c_route_kernel"):
        hits = [k for k in usage if name in k]
        assert hits, name
        for k in hits:
            assert usage[k].get("VGPRs", 0) > 102, (k, usage[k])
