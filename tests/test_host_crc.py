"""The single-buffer host path (nvl_crc32c_extend / _value, the drop-in's
util/crc32c.h Extend) in each of its tiers -- AVX-512 VPCLMULQDQ folding,
SSE4.2 crc32q x3, slice-by-8 (NVL_CRC32C_HOST caps the tier; each tier in
its own process, since the choice is made once) -- against the oracle over
every length 0..1100 (the folding path starts at 256 bytes: its
accumulator, lane and 16-byte tail folds), longer buffers, every start
alignment 0..63 and random inits, and the reference's own RFC 3720 vectors
(tests/golden/kat.json)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, json
sys.path.insert(0, %r)
import numpy as np
import oracle
from nvlevelz_amd import _lib, crc32c as C
p = oracle.port()
rng = np.random.default_rng(7)
buf = rng.integers(0, 256, size=400_000, dtype=np.uint8)
bad = []
lens = list(range(0, 1101)) + [2047, 2048, 4095, 4096, 4097, 8191, 65536, 65537, 131072 + 13, 399_000]
for L in lens:
    off = int(rng.integers(0, 64))
    init = int(rng.integers(0, 2**32))
    d = buf[off:off + L]
    if C.extend(init, d) != p.extend(init, d.tobytes()):
        bad.append((L, off))
for off in range(64):
    d = buf[off:off + 5000]
    if C.value(d) != p.value(d.tobytes()):
        bad.append((5000, off))
print(json.dumps({"impl": _lib.lib.nvl_crc32c_host_impl().decode(), "bad": bad[:10], "n": len(lens) + 64}))
""" % ROOT


def _run(tier):
    env = dict(os.environ)
    if tier:
        env["NVL_CRC32C_HOST"] = tier
    else:
        env.pop("NVL_CRC32C_HOST", None)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("tier", [None, "sse", "table"])
def test_host_tiers_match_oracle(tier):
    res = _run(tier)
    assert res["bad"] == [], res
    if tier == "table":
        assert res["impl"] == "slice-by-8"
    elif tier == "sse":
        assert res["impl"].startswith("sse4.2")


def test_default_tier_uses_folding_when_the_cpu_has_it():
    flags = open("/proc/cpuinfo").read()
    res = _run(None)
    if " vpclmulqdq" in flags and " avx512vl" in flags and " avx512bw" in flags:
        assert res["impl"].startswith("avx512"), res
    else:
        assert not res["impl"].startswith("avx512"), res


def test_kats_through_the_drop_in():
    from conftest import load_golden
    from nvlevelz_amd import crc32c as C
    g = load_golden("kat")
    n = 0
    for case in g.get("value", []):
        assert C.value(bytes.fromhex(case["hex"])) == case["crc"], case
        n += 1
    assert n > 0
