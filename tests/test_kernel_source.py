"""Source-level guards on the shipped kernel sources (CPU, no GPU).

1. Wave-uniform reads.  __builtin_amdgcn_readfirstlane / readlane return
   `int`; applied to (the low half of) a 64-bit value and widened, a low half
   with bit 31 set is sign-extended into the high half.  That corrupted
   head-kernel item pointers and faulted a GPU in round 2 (DESIGN §3.4
   "Division").  Every call must go through the four helpers of
   crc32c_dev.h (uniform_u32 / uniform_u64 / lane_u32 / lane_u64),
   whose 32-bit forms static_assert on wider operands and whose 64-bit forms
   move two uint32_t halves.
2. No ablation or diagnostic variants in the product translation units:
   NVL_ABL_* / NVL_DIAG_* builds live in tools/diag (stamps.h is
   force-included into a variant build only).
3. The shipped library exports no diagnostic entry point.
"""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "nvlevelz_amd", "csrc")
LIB = os.path.join(ROOT, "nvlevelz_amd", "libnvl_crc32c.so")


def _sources(exts=(".hip", ".cpp", ".h")):
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(exts):
            yield os.path.join(CSRC, f)


def _strip_comments(text: str) -> str:
    text = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), text, flags=re.S)
    return re.sub(r"//[^\n]*", "", text)


def _function_spans(text: str, names):
    """(start, end) character spans of the bodies of the named functions."""
    spans = []
    for name in names:
        for m in re.finditer(r"\b%s\s*\([^)]*\)\s*\{" % name, text):
            depth, i = 1, m.end()
            while depth:
                depth += {"{": 1, "}": -1}.get(text[i], 0)
                i += 1
            spans.append((m.start(), i))
    return spans


def test_lane_reads_only_inside_the_helpers():
    helpers = ("uniform_u32", "lane_u32")
    seen = 0
    for path in _sources((".hip", ".h")):
        text = _strip_comments(open(path).read())
        spans = _function_spans(text, helpers)
        for m in re.finditer(r"__builtin_amdgcn_read(first)?lane\b", text):
            line = text.count("\n", 0, m.start()) + 1
            assert any(a <= m.start() < b for a, b in spans), (
                f"{os.path.basename(path)}:{line}: raw {m.group(0)} -- use uniform_u32/uniform_u64/lane_u32/lane_u64")
            seen += 1
    assert seen == 2  # one readfirstlane in uniform_u32, one readlane in lane_u32


def test_helpers_refuse_64bit_operands():
    text = open(os.path.join(CSRC, "crc32c_dev.h")).read()
    for name in ("uniform_u32", "lane_u32"):
        body = [text[a:b] for a, b in _function_spans(text, (name,))]
        assert body and "static_assert(sizeof(T) <= 4" in body[0], name


def test_no_ablation_or_diag_variants_in_product_sources():
    bad = re.compile(r"\bNVL_(ABL|DIAG)_\w+|\bNVL_LD_AUX\b|\bNVL_NO_XOR3\b|s_memrealtime")
    for path in _sources():
        text = _strip_comments(open(path).read())
        m = bad.search(text)
        assert m is None, f"{os.path.basename(path)}: {m.group(0)} belongs in tools/diag"


def test_shipped_library_exports_no_diag_entry_points():
    if not os.path.exists(LIB):
        import pytest
        pytest.skip("library not built")
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    syms = [ln.split()[-1] for ln in out.splitlines() if ln.strip()]
    assert not [s for s in syms if "diag" in s], syms
