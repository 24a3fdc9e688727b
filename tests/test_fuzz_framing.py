"""Host-only AddressSanitizer / UBSan fuzz of the call-site shims' parsers
(nvl_sstable_verify_table, nvl_sstable_verify_blocks, nvl_log_scan): the
driver tests/native/fuzz_framing.cc builds valid tables and logs, mutates them
(bit flips, 0xFF bytes, truncation, trailing garbage; table mutations biased
to the index/metaindex/footer end), and runs every parser in host-CRC mode on
an exact-size heap copy.  Sanitizers run on host code only (no GPU)."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

NATIVE = os.path.join(ROOT, "tests", "native")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
@pytest.mark.parametrize("seed", ["0x1", "0x5eed"])
def test_framing_parsers_under_asan(seed):
    subprocess.run(["make", "-s", "-C", NATIVE, "fuzz_framing"], check=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(NATIVE, "fuzz_framing"), "20000", seed], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    m = re.search(r"table outcomes ((?:\d+ ?){8})", r.stdout)
    counts = [int(x) for x in m.group(1).split()]
    # the mutations reach the footer, index-read and index-walk outcomes, not only clean tables
    assert counts[0] > 0 and counts[2] > 0 and counts[4] > 0 and (counts[5] + counts[6]) > 0, counts
