"""Per-wave s_memtime stamps of the one-launch DIN attention unit (din_fused)
at the config-4 shape (B 2048, T 100, k 8, (80, 40)): cycles from the
workgroup's first stamp, median over workgroups of the median wave and the
slowest wave.  Slots: 0 start, 6 staging stores issued, 1 staged (after the
barrier), 8 / 9 / 10 item 0's MFMAs start / layer 1 done / layer 2 issued,
2..5 the wave's items 0..3 done, 7 end (tiles merged, output written).
Needs the diagnostic build (scripts/build_diag.sh).  --hist: history padding
(pad80: positions 80.. padded; random: lengths 1..T as bench.py's config 4;
full: none)."""
import argparse
import ctypes as C
import json
import os
from pathlib import Path
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from recommender_system_amd import Attention, _lib  # noqa: E402

_lib._LIB_PATH = Path(ROOT) / "recommender_system_amd" / "librs_hip_diag.so"

ap = argparse.ArgumentParser()
ap.add_argument("--hist", default="pad80", choices=["pad80", "random", "full"])
args = ap.parse_args()
B, T, k, V = 2048, 100, 8, 63001
layer = Attention((80, 40), "prelu", seed=1)
layer.build(T, k)
table = torch.randn(V, k, device="cuda")
hist = torch.randint(1, V, (B, T), device="cuda")
if args.hist == "pad80":
    hist[:, 80:] = 0
elif args.hist == "random":
    lens = torch.randint(1, T + 1, (B, 1), device="cuda")
    hist = torch.where(torch.arange(T, device="cuda")[None, :] < lens, hist, torch.zeros_like(hist))
cand = torch.randint(1, V, (B, 1), device="cuda")
lib = _lib.lib()
lib.rs_diag_din_set_dbg.argtypes = [C.c_void_p]
_lib.set_option(_lib.OPT_DIN_KERNEL, 0)
for _ in range(20):
    layer.forward_ids(table, V, hist, cand)
torch.cuda.synchronize()
nwg = (B + 7) // 8
dbg = torch.zeros(nwg * 16 * 16, dtype=torch.int64, device="cuda")
lib.rs_diag_din_set_dbg(dbg.data_ptr())
layer.forward_ids(table, V, hist, cand)
torch.cuda.synchronize()
lib.rs_diag_din_set_dbg(None)
d = dbg.cpu().numpy().reshape(nwg, 16, 16).astype(np.int64)
t0 = d[:, :, 0].min(axis=1, keepdims=True)
out = {"B": B, "T": T, "hist": args.hist, "phases_cycles": {}}
for j, n in {0: "start", 6: "staging_stored", 1: "staged", 8: "item0_mfma_start", 9: "item0_l1_done",
             10: "item0_l2_issued", 2: "item0", 3: "item1", 4: "item2", 5: "item3", 7: "end"}.items():
    ok = d[:, :, j] > 0
    if not ok.any():
        continue
    rel = np.where(ok, d[:, :, j] - t0, np.nan)
    out["phases_cycles"][n] = {"median_wave": int(np.nanmedian(rel)),
                               "slowest_wave": int(np.nanmedian(np.nanmax(rel, axis=1))),
                               "max": int(np.nanmax(rel))}
print(json.dumps(out))
