"""The reference's own test suites through the drop-in boundary (CPU).

oracle/reftests.mk compiles the reference's util/crc32c_test.cc
(util/crc32c_test.cc:13-65, 4 tests) and db/log_test.cc (db/log_test.cc:270-582,
38 tests) unchanged, with integration/leveldb_util_crc32c.cc in place of
util/crc32c.cc + port/port_posix_sse.cc, linked against libnvl_crc32c.so: every
Extend/Value/Mask in those suites runs through nvl_crc32c_extend.  The symbol
checks make sure nothing of the reference's CRC code got linked in beside it."""
import os
import subprocess

import pytest

from conftest import ROOT

REF = "/root/reference"
OUT = os.path.join(ROOT, "oracle", "_ref", "reftests")


@pytest.fixture(scope="module")
def suites():
    if os.path.isdir(REF):
        r = subprocess.run(["make", "-s", "-j8", "-f", os.path.join(ROOT, "oracle", "reftests.mk")], cwd=ROOT,
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
    bins = {k: os.path.join(OUT, k) for k in ("crc32c_test", "log_test")}
    if not all(os.path.exists(b) for b in bins.values()):
        pytest.skip("reference sources absent and no prebuilt suites")
    return bins


def _symbols(path):
    return subprocess.run(["nm", "-C", path], capture_output=True, text=True, check=True).stdout


@pytest.mark.parametrize("name,count", [("crc32c_test", 4), ("log_test", 38)])
def test_reference_suite_passes_through_forwarder(suites, name, count):
    path = suites[name]
    syms = _symbols(path)
    lines = syms.splitlines()
    # Extend is defined once, by the forwarder; the engine entry point is imported
    ext = [l for l in lines if "leveldb::crc32c::Extend(unsigned int, char const*, unsigned long)" in l]
    assert len(ext) == 1 and " T " in ext[0], ext
    assert any(l.split()[-1] == "nvl_crc32c_extend" and " U " in l for l in lines)
    # none of the reference's CRC implementation (util/crc32c.cc tables, the
    # SSE4.2 accelerator of port/port_posix_sse.cc)
    for bad in ("table0_", "crc32c::ExtendImpl", "AcceleratedCRC32C", "CanAccelerateCRC32C"):
        assert bad not in syms, bad
    ldd = subprocess.run(["ldd", path], capture_output=True, text=True, check=True).stdout
    assert os.path.join(ROOT, "nvlevelz_amd", "libnvl_crc32c.so") in ldd or "libnvl_crc32c.so" in ldd
    r = subprocess.run([path], capture_output=True, text=True, timeout=300, cwd=OUT)
    assert r.returncode == 0, r.stderr[-3000:]
    assert f"==== PASSED {count} tests" in r.stderr, r.stderr[-2000:]
    assert r.stderr.count("==== Test ") == count
