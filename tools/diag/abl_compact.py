"""Variants of the compact-image scheduler A (configs 2 and 5): waves per
workgroup (NWC), buffers per unit (UC, static ranges only), workgroups per CU
(WGC), static ranges instead of stealing (STEAL=0), the shared part of a
range (SSH: cnt >> SSH), counter spacing (SSTRIDE words), no stealing from other
workgroups (NOSCAN=1), many shrinking workgroups in dispatch order (GUIDED=avg
buffers per workgroup, with STEAL=0; EQUAL=1: equal sizes), or the 160 KiB single-workgroup kernel (FULL=1).
    NAME=c16u1 NWC=16 UC=1 python tools/diag/abl_compact.py
    NAME=full FULL=1 python tools/diag/abl_compact.py
and then make -C nvlevelz_amd/csrc variant NAME=$NAME VSRC=$PWD/build/abl_$NAME.hip VFLAGS=-I$PWD/nvlevelz_amd/csrc"""
import os, subprocess, tempfile
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the product source with tools/diag/compact_steal.patch applied (the compact
# image, crc32c_fixed_compact_kernel, run_steal; measured and not shipped)
with tempfile.TemporaryDirectory() as td:
    out = os.path.join(td, "k.hip")
    subprocess.run(["patch", "-s", "-o", out, os.path.join(R, "nvlevelz_amd/csrc/crc32c_kernels.hip"),
                    os.path.join(R, "tools/diag/compact_steal.patch")], check=True)
    s = open(out).read()


def rep(old, new):
    global s
    assert s.count(old) == 1, (s.count(old), old[:60])
    s = s.replace(old, new)


if os.environ.get("FULL"):
    rep("constexpr bool kFixedCompact = true;", "constexpr bool kFixedCompact = false;")
if os.environ.get("NWC"):
    rep("constexpr int kCompactWaves = 16;", "constexpr int kCompactWaves = %d;" % int(os.environ["NWC"]))
if os.environ.get("UC"):
    rep("constexpr int kCompactU = 1;", "constexpr int kCompactU = %d;" % int(os.environ["UC"]))
if os.environ.get("WGC"):
    rep("constexpr int kCompactWGsPerCU = 2;", "constexpr int kCompactWGsPerCU = %d;" % int(os.environ["WGC"]))
if os.environ.get("STEAL") == "0":
    rep("constexpr bool kCompactSteal = true;", "constexpr bool kCompactSteal = false;")
if os.environ.get("SSH"):
    rep("constexpr uint32_t kStealShift = 2;", "constexpr uint32_t kStealShift = %d;" % int(os.environ["SSH"]))
if os.environ.get("SSTRIDE"):
    rep("constexpr uint32_t kStealStride = 16;", "constexpr uint32_t kStealStride = %d;" % int(os.environ["SSTRIDE"]))
if os.environ.get("NOSCAN"):
    rep("      const uint32_t v = *done ? kNoUnit : scan();", "      const uint32_t v = kNoUnit; (void)scan;")
if os.environ.get("GUIDED"):  # dispatch-order ranges, GUIDED buffers per workgroup on average (STEAL=0)
    rep("constexpr bool kCompactGuided = false;", "constexpr bool kCompactGuided = true;")
    rep("constexpr uint32_t kGuidedAvg = 32;", "constexpr uint32_t kGuidedAvg = %d;" % int(os.environ["GUIDED"]))
if os.environ.get("EQUAL"):
    rep("constexpr bool kGuidedQuadratic = true;", "constexpr bool kGuidedQuadratic = false;")
os.makedirs(os.path.join(R, "build"), exist_ok=True)
open(os.path.join(R, "build", "abl_%s.hip" % os.environ["NAME"]), "w").write(s)
