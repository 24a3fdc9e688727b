"""Latency of the call-site shims at the fork's real sizes, GPU against the
host CRC, one JSON line per (operation, size, engine):

  seal         nvl_sstable_seal_trailers over a table image (BatchingWritableFile's
               Close, table/table_builder.cc:185-187 deferred); host-resident image
  seal_tb      the reference's own TableBuilder (oracle/_ref/libref_table.so)
               writing a table through shims::BatchingWritableFile, sealed at
               Close -- the whole build, GPU seal against host seal
  verify       nvl_sstable_verify_table (Table::Open + ReadBlock of every block,
               table/format.cc:65-98), host-resident image
  verify_dev   nvl_sstable_verify_table_dev, the image already in HBM
  window64     nvl_sstable_verify_blocks over 64 data blocks (shims::TableReader's
               readahead window, db/version_set.cc:1308,1329)
  manifest10   nvl_log_seal of a 10-record MANIFEST batch (db/version_set.cc:896-909,
               db/log_writer.cc:84-109)
Sizes: tables of 256 KiB .. 128 MiB (max_file_size is 2 MiB, util/options.cc:24;
compaction outputs and L0 flushes, db/builder.cc:35-45, db/db_impl.cc:923).
Wall clock per call (synchronous entry points), median of R calls after 2 warm-ups.
    python tools/shim_latency.py [--reps 15] [--out gpurun_out/shim_latency.jsonl]
"""
import argparse, ctypes, json, os, sys, time
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np
from nvlevelz_amd import _lib
import bench

L = _lib.lib
HOST = _lib.FRAMING_HOST
GPU = getattr(_lib, "FRAMING_GPU", 0)
ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=15)
ap.add_argument("--out", default=None)
ap.add_argument("--sizes", default="0.25,2,8,32,128", help="table sizes in MiB")
a = ap.parse_args()
out = open(a.out, "w") if a.out else None


def emit(d):
    line = json.dumps(d)
    print(line, flush=True)
    if out:
        out.write(line + "\n")
        out.flush()


def med(fn, reps):
    fn(); fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), float(np.min(ts))


def table_handles(img_len, nblocks):
    stride = 4096 + 5
    return np.stack([np.arange(nblocks, dtype=np.uint64) * stride, np.full(nblocks, 4096, np.uint64)], 1)


import torch
torch.cuda.set_device(0)
rc0 = L.nvl_crc32c_init(0)
assert rc0 == 0, f"nvl_crc32c_init: {rc0}"
sptr = torch.cuda.current_stream().cuda_stream
for mib in [float(x) for x in a.sizes.split(",")]:
    nblocks = max(1, int(mib * 2**20 / 4101))
    img = bench.build_table_image(nblocks)
    nbytes = len(img)
    hd = np.ascontiguousarray(table_handles(nbytes, nblocks))
    buf = bytearray(img)
    cbuf = (ctypes.c_char * len(buf)).from_buffer(buf)
    base = {"table_bytes": nbytes, "data_blocks": nblocks}
    for eng, fl in (("gpu", GPU), ("host", HOST)):
        t, tmin = med(lambda: L.nvl_sstable_seal_trailers(cbuf, len(buf), hd.ctypes.data, nblocks, fl), a.reps)
        emit(dict(base, op="seal", engine=eng, ms=round(t * 1e3, 4), min_ms=round(tmin * 1e3, 4),
                  GiBps=round(nbytes / t / 2**30, 2)))
    cap = nblocks + 2
    arr = (_lib.TableBlock * cap)()
    n, st, nb = ctypes.c_size_t(0), ctypes.c_uint32(0), ctypes.c_uint64(0)
    for eng, fl in (("gpu", GPU), ("host", HOST)):
        def run(fl=fl):
            rc = L.nvl_sstable_verify_table(img, nbytes, arr, cap, ctypes.byref(n), ctypes.byref(st),
                                            ctypes.byref(nb), fl)
            assert rc == 0 and st.value == 0 and nb.value == 0, (rc, st.value, nb.value)
        t, tmin = med(run, a.reps)
        emit(dict(base, op="verify", engine=eng, ms=round(t * 1e3, 4), min_ms=round(tmin * 1e3, 4),
                  GiBps=round(nbytes / t / 2**30, 2)))
    dimg = torch.frombuffer(bytearray(img), dtype=torch.uint8).to("cuda")

    def run_dev():
        rc = L.nvl_sstable_verify_table_dev(dimg.data_ptr(), nbytes, arr, cap, ctypes.byref(n), ctypes.byref(st),
                                            ctypes.byref(nb), sptr)
        assert rc == 0 and st.value == 0 and nb.value == 0, (rc, st.value, nb.value)
    t, tmin = med(run_dev, a.reps)
    emit(dict(base, op="verify_dev", engine="gpu", ms=round(t * 1e3, 4), min_ms=round(tmin * 1e3, 4),
              GiBps=round(nbytes / t / 2**30, 2)))
    del dimg
    if mib == 2:
        w = np.ascontiguousarray(hd[:min(64, nblocks)])
        v = np.zeros(len(w), dtype=np.uint8)
        for eng, fl in (("gpu", GPU), ("host", HOST)):
            t, tmin = med(lambda: L.nvl_sstable_verify_blocks(img, nbytes, w.ctypes.data, len(w), v.ctypes.data,
                                                              None, fl), a.reps)
            emit({"op": "window64", "engine": eng, "blocks": len(w), "bytes": int(w[:, 1].sum()),
                  "ms": round(t * 1e3, 4), "min_ms": round(tmin * 1e3, 4)})
        try:  # the reference TableBuilder through BatchingWritableFile, sealed at Close
            import oracle
            rt = oracle.ref_table(deferred=True)
            rng = np.random.default_rng(5)
            nk = int(2**21 / 120)
            keys = [b"key%013d" % i for i in range(nk)]
            vals = [rng.integers(0, 256, 100, dtype=np.uint8).tobytes() for _ in range(nk)]
            for eng, fl in (("gpu", GPU), ("host", HOST)):
                t, tmin = med(lambda: rt.build(keys, vals, via_shim=1, seal_flags=fl), max(3, a.reps // 3))
                img2, _ = rt.build(keys, vals, via_shim=1, seal_flags=fl)
                emit({"op": "seal_tb", "engine": eng, "table_bytes": len(img2), "ms": round(t * 1e3, 3),
                      "min_ms": round(tmin * 1e3, 3), "seals": rt.seals,
                      "what": "whole reference TableBuilder build (-O0 reference objects) incl. the Close seal"})
        except Exception as e:  # noqa: BLE001 -- the builder leg needs the shipped reference build
            emit({"op": "seal_tb", "error": repr(e)})
        # 10-record MANIFEST batch: VersionEdit records of ~100-300 bytes
        rng = np.random.default_rng(9)
        recs = [rng.integers(0, 256, int(rng.integers(100, 300)), dtype=np.uint8).tobytes() for _ in range(10)]
        image, offs = bytearray(), []
        for r_ in recs:
            offs.append(len(image))
            image += bytes(7) + r_
            image[offs[-1] + 4:offs[-1] + 6] = len(r_).to_bytes(2, "little")
            image[offs[-1] + 6] = 1
        ho = np.array(offs, dtype=np.uint64)
        cimg = (ctypes.c_char * len(image)).from_buffer(image)
        for eng, fl in (("gpu", GPU), ("host", HOST)):
            t, tmin = med(lambda: L.nvl_log_seal(cimg, len(image), ho.ctypes.data, len(ho), fl), a.reps)
            emit({"op": "manifest10", "engine": eng, "bytes": len(image), "ms": round(t * 1e3, 4),
                  "min_ms": round(tmin * 1e3, 4)})
    del cbuf
