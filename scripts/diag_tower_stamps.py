"""Per-wave s_memtime stamps of the MLP tower (diagnostic hook
rs_diag_mlp_set_dbg): median cycles of each phase across workgroups."""
import ctypes as C
import os
from pathlib import Path
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from recommender_system_amd import DNNLayer, _lib  # noqa: E402

# the MLP stamps exist only in the diagnostic build (scripts/build_diag.sh)
_lib._LIB_PATH = Path(ROOT) / "recommender_system_amd" / "librs_hip_diag.so"

B = int(os.environ.get("TOWER_B", "4096"))
dims = [int(v) for v in os.environ.get("TOWER_DIMS", "429,256,128,64,1").split(",")]
dnn = DNNLayer(dims[1:-1], dims[-1], "relu", seed=1)
dnn.build(dims[0])
x = torch.rand(B, dims[0], device="cuda")
y = torch.empty(B, dims[-1], device="cuda")
nwg = (B + 15) // 16
dbg = torch.zeros(nwg * 16 * 16, dtype=torch.int64, device="cuda")
lib = _lib.lib()
lib.rs_diag_mlp_set_dbg.argtypes = [C.c_void_p]
for _ in range(5):
    dnn.tower(x, out=y)
torch.cuda.synchronize()
lib.rs_diag_mlp_set_dbg(dbg.data_ptr())
dnn.tower(x, out=y)
torch.cuda.synchronize()
lib.rs_diag_mlp_set_dbg(None)
d = dbg.cpu().numpy().reshape(nwg, 16, 16).astype(np.int64)
L = len(dims) - 1
t0 = d[:, :, 0].min(axis=1, keepdims=True)
names = ["start", "prologue"] + sum([[f"l{l}_barrier", f"l{l}_mac"] for l in range(L)], [])
idx = [0, 1] + sum([[2 + 2 * l, 3 + 2 * l] for l in range(L)], []) + [15]
names.append("end")
rel = d[:, :, idx] - t0[:, :, None]
print("B", B, "dims", dims, "workgroups", nwg)
print("phase: median over (wg, wave) of cycles since the workgroup's first stamp; max over waves (median over wgs)")
for j, n in enumerate(names):
    print(f"{n:12s} {int(np.median(rel[:, :, j])):8d} {int(np.median(rel[:, :, j].max(axis=1))):8d}")
kstart = d[:, :, 0].min()
print("kernel span cycles", int(d[:, :, 15].max() - kstart),
      "wg start spread", int(np.percentile(d[:, :, 0].min(axis=1) - kstart, 50)), int((d[:, :, 0].min(axis=1) - kstart).max()))
