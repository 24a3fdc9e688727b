"""Phase timeline of the region kernel (run_region) from a diagnostic variant
build with tools/diag/stamps.h force-included:
    make -C nvlevelz_amd/csrc variant NAME=stamps VFLAGS_crc32c_region="-include ../../tools/diag/stamps.h"
    CFG=v|r|3 LIB=build/libnvl_crc32c_stamps.so python tools/diag/rtl.py
Stamps per wave (s_memrealtime, 100 MHz): 0 entry, 1 after the LDS fill
barrier, 2 out of units, 3 after the fold barrier, 4 a slice's records in,
5 its arithmetic done (the last slice the wave folded), 7 exit.  Per workgroup:
the spread of its waves' unit-loop exits, the barrier wait, the fold; over
the kernel: when the last workgroup left its units and when it ended."""
import ctypes, json, os, sys
import numpy as np, torch
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.getcwd())
sys.path.insert(0, ROOT)
from nvlevelz_amd import _lib
lib = ctypes.CDLL(os.path.abspath(os.environ.get("LIB", "build/libnvl_crc32c_stamps.so")), mode=os.RTLD_LOCAL)
for name, (res, args) in _lib.SIGNATURES.items():
    if hasattr(lib, name):
        f = getattr(lib, name); f.restype = res; f.argtypes = args
lib.nvl_diag_tl.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
cfg = os.environ.get("CFG", "v")
if cfg == "3":
    import oracle
    lens = oracle.port().cfg3_lengths(0x5EED0003, 1 << 30).astype(np.int64); gap = 0
else:
    lens = (np.full(100_000, 4097) if cfg == "v" else np.random.default_rng(7).integers(3364, 4110, 100_000)
            ).astype(np.int64); gap = 4
total = int((lens + gap).sum())
offs = np.concatenate([[0], np.cumsum(lens + gap)[:-1]]).astype(np.int64)
n = lens.size
buf = torch.empty(total + 64, dtype=torch.uint8, device=dev)
lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), (total + 64) // 8, 8, 0, 1, 0x5EED00B1, None)
o = torch.from_numpy(offs).to(dev); m = torch.from_numpy(lens).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
wsb = lib.nvl_crc32c_region_workspace_bytes(total, n)
ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
run = lambda: lib.nvl_crc32c_region_dev(buf.data_ptr(), total, o.data_ptr(), m.data_ptr(), None, 0, out.data_ptr(), n,
                                        0, ws.data_ptr(), wsb, st)
reps = int(os.environ.get("REPS", "5"))
res = []
lastx = []
for r in range(reps + 3):
    for _ in range(20): run()  # back to back, as in the sustained measurement; stamps of the last call
    torch.cuda.synchronize()
    if r < 3:
        continue
    G = min(256, torch.cuda.get_device_properties(0).multi_processor_count)
    W = G * 16
    h = np.zeros(8 * W, dtype=np.uint64)
    assert lib.nvl_diag_tl(h.ctypes.data, h.size) == 0
    t = h.reshape(W, 8).astype(np.int64)
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0  # 100 MHz -> us
    wg = us.reshape(G, 16, 8)
    loop_first, loop_last = wg[:, :, 2].min(1), wg[:, :, 2].max(1)
    bar = wg[:, :, 3].max(1)
    end = wg[:, :, 7].max(1)
    q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 50, 90, 100)]
    f0 = wg[:, :, 4] > 0  # waves that folded a slice: records in (4), arithmetic done (5)
    rec = (wg[:, :, 4] - wg[:, :, 3])[f0]; ari = (wg[:, :, 5] - wg[:, :, 4])[f0]; sto = (wg[:, :, 7] - wg[:, :, 5])[f0]
    lastx.append(loop_last - loop_last.mean())
    entry = wg[:, :, 0].min(1)  # workgroup dispatch (its first wave's entry)
    bi = np.arange(G)
    ent_xcd = [round(float(np.median(entry[x::8])), 2) for x in range(8)]
    print(json.dumps({"wg_entry_us": q(entry), "entry_by_xcd_us": ent_xcd,
                      "entry_slope_us_per_wg": round(float(np.polyfit(bi, entry, 1)[0]), 4),
                      "corr_entry_lastexit": round(float(np.corrcoef(entry, loop_last)[0, 1]), 3),
                      "corr_entry_unitwork": round(float(np.corrcoef(entry, loop_last - entry)[0, 1]), 3),
                      "lastexit_minus_entry_us": q(loop_last - entry)}), flush=True)
    xcd = [round(float(np.median(loop_last[x::8] - loop_last.mean())), 2) for x in range(8)]
    res.append({"wg_last_exit_by_xcd_us": xcd, "search_done_us": q(wg[:, :, 6].max(1)), "fold_records_us": q(rec), "fold_arith_us": q(ari), "fold_store_exit_us": q(sto),
                "kernel_end_us": round(float(us[:, 7].max()), 2), "last_out_of_units_us": round(float(loop_last.max()), 2),
                "fill_barrier_us": q(wg[:, :, 1].max(1)), "wg_unit_exit_spread_us": q(loop_last - loop_first),
                "wg_barrier_after_last_exit_us": q(bar - loop_last), "wg_fold_us": q(end - bar),
                "wg_end_us": q(end), "wg_last_exit_us": q(loop_last)})
for r in res:
    print(json.dumps(r), flush=True)
L = np.array(lastx)  # reps x G: is a slow workgroup slow every time?
cc = np.corrcoef(L)
print(json.dumps({"wg_last_exit_rep_corr": [round(float(cc[i, i + 1]), 3) for i in range(len(L) - 1)],
                  "wg_last_exit_std_us": round(float(L.std(1).mean()), 2),
                  "wg_last_exit_mean_over_reps_std_us": round(float(L.mean(0).std()), 2)}), flush=True)
