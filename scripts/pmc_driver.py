"""Fixed-count launches for PMC collection (run under rocprofv3 --pmc):
  * rs_embed_fm_fwd_hm (the bench's entry) at the headline shape (B=4096, 26 x 1e7 x 16, int32 ids),
    50 launches over a pool of 16 batches;
  * the calibration probe (diagnostic library): random 64-B rows and line
    pairs, known byte counts (1,703,936 rows x 64 B, + 8-B row indices).
Per-dispatch counters / launch give HBM bytes per launch (profiles/)."""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from recommender_system_amd import _lib  # noqa: E402

dev = torch.device("cuda")
F, k, kfm, nd, V, B = 26, 16, 10, 13, 10_000_000, 4096
lib = _lib.lib()
table = torch.empty(F * V, k, device=dev).uniform_(-0.05, 0.05)
d = nd + F * k
w1 = torch.randn(d, 1, device=dev) * 0.05
v = torch.randn(d, kfm, device=dev) * 0.05
w0 = torch.zeros(1, device=dev)
prep = torch.empty(lib.rs_fm_prepared_size(nd, F, k, kfm), device=dev)
_lib.call("rs_fm_prepare", w1.data_ptr(), v.data_ptr(), nd, F, k, kfm, prep.data_ptr(), _lib.stream())
offs = torch.arange(F, dtype=torch.int64, device=dev) * V
voc = torch.full((F,), V, dtype=torch.int64, device=dev)
pool = [torch.randint(0, V, (B, F), dtype=torch.int32, device=dev) for _ in range(64)]
dense = torch.rand(B, nd, device=dev)
logit = torch.empty(B, device=dev)
torch.cuda.synchronize()
hoff = (C.c_int64 * F)(*[c * V for c in range(F)])
hvoc = (C.c_int64 * F)(*([V] * F))
for i in range(128):  # 64-batch rotation as in bench.py: rows not MALL-resident between uses
    ids = pool[i % 64]
    # the bench's entry (field metadata as kernel arguments: embed_fm_mfma_ka)
    _lib.call("rs_embed_fm_fwd_hm", ids.data_ptr(), 0, F, dense.data_ptr(), nd, nd, table.data_ptr(),
              offs.data_ptr(), voc.data_ptr(), C.addressof(hoff), C.addressof(hvoc), F, k, prep.data_ptr(),
              w0.data_ptr(), kfm, logit.data_ptr(), None, B, None, _lib.stream())
torch.cuda.synchronize()
diag = os.path.join(ROOT, "recommender_system_amd", "librs_hip_diag.so")
if os.path.exists(diag):
    dl = C.CDLL(diag)
    dl.rs_diag_gather_sum.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
    n = 1_703_936
    out = torch.zeros(8192, device=dev)
    for kind in ("random_rows", "line_pairs"):
        for _ in range(5):  # fresh rows per dispatch: nothing re-read from L2/MALL
            r = torch.randint(0, F * V, (n,), device=dev)
            if kind == "line_pairs":
                r = torch.stack([(r[: n // 2] // 2) * 2, (r[: n // 2] // 2) * 2 + 1], 1).reshape(-1)
            dl.rs_diag_gather_sum(table.data_ptr(), r.data_ptr(), n, 8192, out.data_ptr(), 0, _lib.stream())
    torch.cuda.synchronize()
print("pmc driver done")
