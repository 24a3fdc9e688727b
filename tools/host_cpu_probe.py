"""Where the host CPU of a host-resident call goes: getrusage of the calling
thread (RUSAGE_THREAD) against the whole process (RUSAGE_SELF) around
nvl_crc32c_batch_region_host calls on a registered image (DMA and zero copy)
and a staged one, plus a bare hipMemcpyAsync of the same bytes from the
registered pages with the caller asleep -- CPU-seconds per GiB each.
    python tools/host_cpu_probe.py"""
import json, os, resource, sys, time
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from nvlevelz_amd import crc32c as C


def ru(who):
    r = resource.getrusage(who)
    return r.ru_utime + r.ru_stime


C.init(0)
n, L, S = 100_000, 4097, 4101
img = np.random.default_rng(1).integers(0, 256, size=n * S, dtype=np.uint8)
offs = np.arange(n, dtype=np.uint64) * S
lens = np.full(n, L, dtype=np.uint64)
gib = n * L / 2**30
reps = 10


def probe(name, fn):
    fn()
    s0, t0, w0 = ru(resource.RUSAGE_SELF), ru(resource.RUSAGE_THREAD), time.perf_counter()
    for _ in range(reps):
        fn()
    s1, t1, w1 = ru(resource.RUSAGE_SELF), ru(resource.RUSAGE_THREAD), time.perf_counter()
    print(json.dumps({"case": name, "ms_per_call": round((w1 - w0) / reps * 1e3, 3),
                      "process_cpu_s_per_GiB": round((s1 - s0) / (reps * gib), 4),
                      "calling_thread_cpu_s_per_GiB": round((t1 - t0) / (reps * gib), 4)}), flush=True)


probe("staged", lambda: C.extend_region_host(img, offs, lens))
C.host_register(img)
probe("registered_dma", lambda: C.extend_region_host(img, offs, lens))
probe("registered_zero_copy", lambda: C.extend_region_host(img, offs, lens, zero_copy=True))
dst = torch.empty(img.nbytes, dtype=torch.uint8, device="cuda:0")
src = torch.from_numpy(img)
st = torch.cuda.current_stream()


def bare_copy(sleep):
    dst.copy_(src, non_blocking=True)  # registered pages: DMA
    if sleep:
        time.sleep(img.nbytes / 60e9)
    st.synchronize()


probe("bare_h2d_sync", lambda: bare_copy(False))
probe("bare_h2d_sleep_then_sync", lambda: bare_copy(True))
C.host_unregister(img)
