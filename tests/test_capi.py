"""The C ABI boundary (include/nvl_crc32c.h -> libnvl_crc32c.so), CPU side:
the library loads, exports every declared entry point, its host
(util/crc32c.h) functions match the oracle, and the batch entry points fail
loudly -- never fall back to the CPU -- when no GPU is present."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, gpu_present, load_golden


@pytest.fixture(scope="module")
def L():
    from nvlevelz_amd import _lib
    return _lib


def test_exports_every_header_symbol(L):
    syms = L.header_symbols()
    assert len(syms) >= 16
    for s in syms:
        assert hasattr(L.lib, s), s
    assert set(syms) == set(L.SIGNATURES), "ctypes table out of sync with the header"
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(syms) <= exported
    assert all(e.startswith("nvl_") for e in exported), "only the C ABI may be exported"


def test_abi_version_and_strerror(L):
    assert L.lib.nvl_crc32c_abi_version() == 1
    for code in (0, -1, -2, -3, -4, -5, 17):
        assert L.lib.nvl_crc32c_strerror(code)


def test_header_compiles_as_c_and_cpp(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "nvl_crc32c.h"\n#include "nvl_framing.h"\n'
                   'int main(void){return nvl_crc32c_abi_version()==NVL_CRC32C_ABI_VERSION?0:1;}\n')
    inc = os.path.join(ROOT, "include")
    lib = os.path.join(ROOT, "nvlevelz_amd")
    for cc, ext in (("gcc", "c"), ("g++", "cc")):
        s2 = tmp_path / f"t.{ext}"
        s2.write_text(src.read_text())
        exe = tmp_path / f"t_{ext}"
        subprocess.run([cc, "-Wall", "-Werror", "-I", inc, str(s2), "-L", lib, "-lnvl_crc32c",
                        f"-Wl,-rpath,{lib}", "-o", str(exe)], check=True)
        subprocess.run([str(exe)], check=True)


def test_host_api_matches_golden(L):
    from nvlevelz_amd import crc32c
    g = load_golden("kat")
    for v in g["value"]:
        assert crc32c.value(bytes.fromhex(v["hex"])) == v["crc"], v["name"]
    for e in g["extend"]:
        assert crc32c.extend(e["init"], bytes.fromhex(e["hex"])) == e["crc"]
    for m in g["mask"]:
        assert crc32c.mask(m["crc"]) == m["masked"]
        assert crc32c.unmask(m["crc"]) == m["unmasked"]
    assert crc32c.kMaskDelta == 0xA282EAD8


def test_host_api_matches_oracle_random(L, port):
    rng = np.random.default_rng(9)
    buf = port.fill(0x1234, 0, 1 << 18)
    for _ in range(2000):
        o = int(rng.integers(0, 4096))
        n = int(rng.integers(0, 50000))
        init = int(rng.integers(0, 2**32))
        assert L.lib.nvl_crc32c_extend(init, buf.ctypes.data + o, n) == \
            port.lib.oracle_crc32c_extend(init, buf.ctypes.data + o, n)


@pytest.mark.skipif(gpu_present(), reason="checks the no-GPU behaviour")
def test_batch_entry_points_fail_loudly_without_gpu(L):
    buf = np.zeros(8192, dtype=np.uint8)
    out = np.zeros(2, dtype=np.uint32)
    rc = L.lib.nvl_crc32c_fixed_dev(buf.ctypes.data, 4096, 4096, 2, None, 0, out.ctypes.data, 0, None, 0, None)
    assert rc in (L.ENODEV, L.EHIP)
    offs = np.array([0, 4096], dtype=np.uint64)
    lens = np.array([4096, 4096], dtype=np.uint64)
    rc = L.lib.nvl_crc32c_batch_dev(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, None, 0,
                                    out.ctypes.data, 2, 0, None, 0, None)
    assert rc in (L.ENODEV, L.EHIP)
    ptrs = (ctypes.c_void_p * 1)(buf.ctypes.data)
    rc = L.lib.nvl_crc32c_batch_host(ptrs, lens.ctypes.data, None, 0, out.ctypes.data, 1, 0)
    assert rc in (L.ENODEV, L.EHIP)
    assert L.lib.nvl_crc32c_gpu_accelerated() == 0
    assert out.tolist() == [0, 0]  # nothing was written: no CPU stand-in
    from nvlevelz_amd import crc32c
    with pytest.raises(crc32c.Crc32cError):
        crc32c.extend_batch_host([b"abc"])


def test_argument_errors(L):
    # n == 0 is a no-op even without a device; NULL outputs are rejected before any work
    assert L.lib.nvl_crc32c_fixed_dev(None, 0, 0, 0, None, 0, None, 0, None, 0, None) in (0, L.ENODEV)
    assert L.lib.nvl_crc32c_fill_splitmix(None, 1, 8, 0, 1, 0, None) == L.EINVAL
    assert L.lib.nvl_crc32c_fill_splitmix(ctypes.c_void_p(16), 1, 7, 0, 1, 0, None) == L.EINVAL
    # the read probe (bench.py's ceiling): whole 16-byte granules from a 16-byte-aligned source, a sink
    assert L.lib.nvl_crc32c_read_probe(None, 0, None, None) == 0
    assert L.lib.nvl_crc32c_read_probe(ctypes.c_void_p(16), 24, ctypes.c_void_p(16), None) == L.EINVAL
    assert L.lib.nvl_crc32c_read_probe(ctypes.c_void_p(24), 32, ctypes.c_void_p(16), None) == L.EINVAL
    assert L.lib.nvl_crc32c_read_probe(ctypes.c_void_p(16), 32, None, None) == L.EINVAL
    assert L.lib.nvl_crc32c_read_probe(ctypes.c_void_p(16), 32, ctypes.c_void_p(16), None) in (L.ENODEV, L.EHIP)


def test_product_does_not_import_oracle():
    """The shipped package must never route through the checker."""
    pkg = os.path.join(ROOT, "nvlevelz_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h", ".cc")):
                text = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in text and "oracle_crc32c" not in text, f
                assert "liboracle" not in text and "_ref/" not in text, f


def test_leveldb_mirror_header(tmp_path):
    """include/nvl_crc32c_leveldb.h: util/crc32c.h's API compiled and run in C++
    against util/crc32c_test.cc's known answers (CPU path, no GPU needed)."""
    src = tmp_path / "t.cc"
    src.write_text(r'''
#include <string.h>
#include <stdio.h>
#include "nvl_crc32c_leveldb.h"
using namespace leveldb::crc32c;
int main() {
  char buf[32];
  memset(buf, 0, 32); if (Value(buf, 32) != 0x8a9136aa) return 1;
  memset(buf, 0xff, 32); if (Value(buf, 32) != 0x62a8ab43) return 2;
  for (int i = 0; i < 32; i++) buf[i] = i;
  if (Value(buf, 32) != 0x46dd794e) return 3;
  for (int i = 0; i < 32; i++) buf[i] = 31 - i;
  if (Value(buf, 32) != 0x113fdb5c) return 4;
  if (Value("a", 1) == Value("foo", 3)) return 5;
  if (Value("hello world", 11) != Extend(Value("hello ", 6), "world", 5)) return 6;
  uint32_t crc = Value("foo", 3);
  if (crc == Mask(crc) || crc == Mask(Mask(crc))) return 7;
  if (crc != Unmask(Mask(crc)) || crc != Unmask(Unmask(Mask(Mask(crc))))) return 8;
  if (Value("TestCRCBuffer", 13) != 0xdcbc59fa) return 9;
  return 0;
}
''')
    inc = os.path.join(ROOT, "include")
    lib = os.path.join(ROOT, "nvlevelz_amd")
    exe = tmp_path / "t"
    subprocess.run(["g++", "-std=c++11", "-Wall", "-Werror", "-I", inc, str(src), "-L", lib, "-lnvl_crc32c",
                    f"-Wl,-rpath,{lib}", "-o", str(exe)], check=True)
    subprocess.run([str(exe)], check=True)


def test_routed_workspace_is_bounded(L):
    """nvl_crc32c_batch_workspace_bytes covers the routed call's region part
    (4 bytes per 4 KiB chunk of the largest region-shaped span, 32 bytes of
    event records per buffer), the chunk part capped at 2^24 chunks (a 64
    GiB span): 10^7 buffers need well under a gigabyte, not the 1.4 GB of
    raws an uncapped 36 chunks per buffer would reserve."""
    small = L.lib.nvl_crc32c_batch_workspace_bytes(100_000)
    assert 14_400_000 < small < 40_000_000
    big = L.lib.nvl_crc32c_batch_workspace_bytes(10_000_000)
    assert big < 700_000_000
    assert big - 32 * 10_000_000 >= 4 * (1 << 24)


def test_workspace_sizes_stay_bounded():
    """the checked entries reserve the routed call's region part
    (32 B of event records per buffer + 4 B per chunk of the span, at most
    2^24 chunks).  The sizes INTEGRATION.md §6 tabulates stay within these
    bounds (no GPU: the library sizes for 256 CUs)."""
    from nvlevelz_amd import _lib
    L = _lib.lib
    assert L.nvl_crc32c_batch_workspace_bytes(1) < 1 << 20
    for n in (10**3, 10**5, 10**6, 10**7):
        b = L.nvl_crc32c_batch_workspace_bytes(n)
        r = L.nvl_crc32c_region_workspace_bytes(4096 * n, n)
        assert b <= 60 * n + (64 << 20) + (1 << 20), (n, b)   # <= 60 B per buffer + the 64 MiB raw cap
        assert r <= 56 * n + (1 << 20), (n, r)                # 32 B records + 4 B raw + the batch part
    assert L.nvl_crc32c_batch_workspace_bytes(10**5) < 24 << 20
    assert L.nvl_crc32c_fixed_workspace_bytes(4096, 4096, 10**7) == 0
