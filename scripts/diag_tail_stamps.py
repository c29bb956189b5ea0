"""Every stamp slot (0..15) of the split-K tail's towers, diagnostic build:
median over workgroups of (median wave, slowest wave) cycles since the
workgroup's first stamp.  TAIL_WL=din_tower (PReLU 25-256-128-64-1, B 2048)
or deepfm (rs_deepfm_fwd_hm, B 4096, 26 x 1e6 x 16).  Slots: 0 entry, 1
layer 0 done (deepfm: FM done), 2/3 layer 0 barrier / mac (deepfm: bursts),
4/5 layer 1 barrier / mac, 10 partials written, 11 after the partials'
barrier, 12 epilogue done, 6/7 layer 2 barrier / mac, 13 partials written,
14 after their barrier, 8 head barrier, 15 end."""
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import recommender_system_amd as rs  # noqa: E402
from recommender_system_amd import _lib  # noqa: E402

_lib._LIB_PATH = Path(ROOT) / "recommender_system_amd" / "librs_hip_diag.so"
dev = torch.device("cuda")
wl = os.environ.get("TAIL_WL", "din_tower")
if wl == "din_tower":
    B = 2048
    dnn = rs.DNNLayer((256, 128, 64), 1, "prelu", seed=2, device=dev)
    dnn.build(25)
    x = torch.randn(16, B, 25, device=dev)
    run = lambda i: dnn.tower(x[i % 16])
else:
    B, F, nd, k, V = 4096, 26, 13, 16, int(1e6)
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    m = rs.DeepFM(cols, 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, seed=2, device=dev)
    ids = torch.randint(0, V, (16, B, F), device=dev, dtype=torch.int32)
    dense = torch.rand(16, B, nd, device=dev)
    run = lambda i: m.forward_fused((dense[i % 16], ids[i % 16]), check_ids=False)
nwg = (B + 15) // 16
dbg = torch.zeros(nwg * 16 * 16, dtype=torch.int64, device=dev)
lib = _lib.lib()
lib.rs_diag_mlp_set_dbg.argtypes = [C.c_void_p]
for i in range(40):
    run(i)
torch.cuda.synchronize()
lib.rs_diag_mlp_set_dbg(dbg.data_ptr())
run(0)
torch.cuda.synchronize()
lib.rs_diag_mlp_set_dbg(None)
d = dbg.cpu().numpy().reshape(nwg, 16, 16).astype(np.int64)
t0 = np.where(d[:, :, 0] > 0, d[:, :, 0], np.iinfo(np.int64).max).min(axis=1, keepdims=True)
out = {"workload": wl, "B": B, "slots": {}}
for j in range(16):
    ok = d[:, :, j] > 0
    if not ok.any():
        continue
    rel = np.where(ok, d[:, :, j] - t0, np.nan)
    out["slots"][j] = [int(np.nanmedian(rel)), int(np.nanmedian(np.nanmax(rel, axis=1)))]
print(json.dumps(out))
