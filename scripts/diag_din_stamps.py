"""Per-wave s_memtime stamps of din_scores at the config-4 shape (B=2048,
T=100, k=8, (80, 40)): cycles from the workgroup's first stamp."""
import ctypes as C
import os
from pathlib import Path
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_system_amd import Attention, _lib  # noqa: E402

# the DIN stamps exist only in the diagnostic build (scripts/build_diag.sh)
_lib._LIB_PATH = Path(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))) / "recommender_system_amd" / "librs_hip_diag.so"

B, T, k, V = 2048, 100, 8, 63001
layer = Attention((80, 40), "prelu", seed=1)
layer.build(T, k)
table = torch.randn(V, k, device="cuda")
hist = torch.randint(1, V, (B, T), device="cuda")
cand = torch.randint(1, V, (B, 1), device="cuda")
lib = _lib.lib()
lib.rs_diag_din_set_dbg.argtypes = [C.c_void_p]
for _ in range(5):
    layer.forward_ids(table, V, hist, cand)
torch.cuda.synchronize()
nwg = 8192
dbg = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device="cuda")
lib.rs_diag_din_set_dbg(dbg.data_ptr())
layer.forward_ids(table, V, hist, cand)
torch.cuda.synchronize()
lib.rs_diag_din_set_dbg(None)
d = dbg.cpu().numpy().reshape(nwg, 4, 8)
d = d[d[:, :, 0].max(axis=1) > 0]
nwg = d.shape[0]
t0 = d[:, :, 0].min(axis=1, keepdims=True)
rel = d[:, :, :6] - t0[:, :, None]
for j, n in enumerate(["start", "staged", "sample0", "sample1", "sample2", "sample3"]):
    print(f"{n:10s} {int(np.median(rel[:, :, j])):8d} {int(np.median(rel[:, :, j].max(axis=1))):8d}")
rt0 = d[:, :, 6].min()
st_us = (d[:, :, 6].min(axis=1) - rt0) / 100.0
en_us = (d[:, :, 7].max(axis=1) - rt0) / 100.0
print("workgroup start (us from first): p50 %.2f p90 %.2f max %.2f" % tuple(np.percentile(st_us, [50, 90, 100])))
print("workgroup end   (us from first): p50 %.2f p90 %.2f max %.2f" % tuple(np.percentile(en_us, [50, 90, 100])))
print("workgroup life  (us): p50 %.2f max %.2f" % (np.median(en_us - st_us), (en_us - st_us).max()))
