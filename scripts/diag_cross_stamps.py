"""Per-wave s_memtime stamps of the fused DCN input + CrossNet kernel at the
config-3 shape (rs_embed_cross_fwd_hm: B 4096, 26 x 1e6 x 16, 13 dense,
depth 3; diagnostic hook rs_diag_cross_set_dbg): median cycles since the
workgroup's first stamp, and the slowest wave's (median over workgroups).
Slots: 0 start, 1 rows + beta in LDS, 2 after the gather barrier, 3
contraction done, 4 after its barrier, 5 after the alpha barrier, 6 output
stores issued."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recommender_system_amd as rs  # noqa: E402
from recommender_system_amd import _lib  # noqa: E402
from pathlib import Path  # noqa: E402

# the CrossNet stamps exist only in the diagnostic build (scripts/build_diag.sh)
_lib._LIB_PATH = Path(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))) / "recommender_system_amd" / "librs_hip_diag.so"

B, F, V, k = 4096, 26, 1_000_000, 16
cols = [[{"feat": f"I{i}"} for i in range(13)],
        [{"feat": f"C{i}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
model = rs.DCN(cols, [256, 128, 64], 1, "relu", 3, embed_dim=k, seed=1, device=torch.device("cuda"))
ids = torch.randint(0, V, (B, F), dtype=torch.int32, device="cuda")
dense = torch.rand(B, 13, device="cuda")
lib = _lib.lib()
_lib.set_option(_lib.OPT_CROSS_KERNEL, int(os.environ.get("RS_CROSS_KERNEL", "0")))  # 0 register / 1 staged tile
lib.rs_diag_cross_set_dbg.argtypes = [C.c_void_p]
for _ in range(5):
    model.cross_fused((dense, ids), check_ids=False)
torch.cuda.synchronize()
nwg = (B + 15) // 16
dbg = torch.zeros(nwg * 16 * 8, dtype=torch.int64, device="cuda")
lib.rs_diag_cross_set_dbg(dbg.data_ptr())
model.cross_fused((dense, ids), check_ids=False)
torch.cuda.synchronize()
lib.rs_diag_cross_set_dbg(None)
d = dbg.cpu().numpy().reshape(-1, 16, 8)
d = d[d[:, :, 0].min(axis=1) > 0]
t0 = d[:, :, 0].min(axis=1, keepdims=True)
rel = d[:, :, :7] - t0[:, :, None]
for j, n in enumerate(["start", "rows_in_lds", "after_barrier", "contracted", "after_cs_barrier", "after_alpha",
                       "stores_issued"]):
    print(f"{n:16s} {int(np.median(rel[:, :, j])):8d} {int(np.median(rel[:, :, j].max(axis=1))):8d}")
