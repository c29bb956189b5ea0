"""Per-wave s_memtime stamps of DIN.call as ONE launch (din_fused_tower,
rs_din_forward_ids) at the config-4 shape (B 2048, T 100, k 8, (80, 40),
random history lengths as bench.py): cycles from the workgroup's first
stamp, median over workgroups of the median wave and the slowest wave.
Attention slots (rs_diag_din_set_dbg): start, staged, item0 .. item3, merge
(tiles merged, tower row written); tower slots (rs_diag_mlp_set_dbg): 2 / 3
layer 0 barrier / mac, 4 / 5 layer 1, 10 / 11 / 12 partials / barrier /
epilogue, 6 / 7 layer 2, 13 / 14, 8 head barrier, 15 end.  Needs the
diagnostic build (scripts/build_diag.sh)."""
import ctypes as C
import json
import os
from pathlib import Path
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from recommender_system_amd import DIN, _lib  # noqa: E402

_lib._LIB_PATH = Path(ROOT) / "recommender_system_amd" / "librs_hip_diag.so"
B, T, k = 2048, 100, 8
dev = torch.device("cuda")
cols = [[{"feat": "price"}], [{"feat": "user_id", "feat_onehot_dim": 192404, "embed_dim": k},
                              {"feat": "movies_seq", "feat_onehot_dim": 63001, "embed_dim": k}]]
model = DIN(cols, ["movies_seq"], seed=1, device=dev)
g = torch.Generator(device=dev)
g.manual_seed(3)
lens = torch.randint(1, T + 1, (B, 1), generator=g, device=dev)
hist = torch.randint(1, 63001, (B, T), generator=g, device=dev)
hist = torch.where(torch.arange(T, device=dev)[None, :] < lens, hist, torch.zeros_like(hist))
inputs = {"price": torch.rand(B, 1, generator=g, device=dev),
          "user_id": torch.randint(0, 192404, (B, 1), generator=g, device=dev),
          "movies_seq": hist, "movie_id": torch.randint(1, 63001, (B, 1), generator=g, device=dev)}
lib = _lib.lib()
lib.rs_diag_din_set_dbg.argtypes = [C.c_void_p]
lib.rs_diag_mlp_set_dbg.argtypes = [C.c_void_p]
for _ in range(20):
    model(inputs, check_ids=False)
torch.cuda.synchronize()
nwg = (B + 7) // 8
dd = torch.zeros(nwg * 16 * 16, dtype=torch.int64, device=dev)
dm = torch.zeros(nwg * 16 * 16, dtype=torch.int64, device=dev)
lib.rs_diag_din_set_dbg(dd.data_ptr())
lib.rs_diag_mlp_set_dbg(dm.data_ptr())
model(inputs, check_ids=False)
torch.cuda.synchronize()
lib.rs_diag_din_set_dbg(None)
lib.rs_diag_mlp_set_dbg(None)
a = dd.cpu().numpy().reshape(nwg, 16, 16).astype(np.int64)
m = dm.cpu().numpy().reshape(nwg, 16, 16).astype(np.int64)
t0 = a[:, :, 0].min(axis=1, keepdims=True)
out = {"B": B, "T": T, "hist": "random", "phases_cycles": {}}
rows = [(a, j, n) for j, n in {0: "start", 1: "staged", 2: "item0", 3: "item1", 4: "item2", 5: "item3",
                                7: "merge"}.items()]
rows += [(m, j, f"tower_{j}") for j in (2, 3, 4, 5, 10, 11, 12, 6, 7, 13, 14, 8, 15)]
for d, j, n in rows:
    ok = d[:, :, j] > 0
    if not ok.any():
        continue
    rel = np.where(ok, d[:, :, j] - t0, np.nan)
    out["phases_cycles"][n] = {"median_wave": int(np.nanmedian(rel)),
                               "slowest_wave": int(np.nanmedian(np.nanmax(rel, axis=1))),
                               "max": int(np.nanmax(rel))}
print(json.dumps(out))
