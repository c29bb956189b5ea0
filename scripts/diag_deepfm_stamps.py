"""Per-wave s_memtime stamps (shader cycles) of the fused DeepFM kernel
(rs_deepfm_fwd_hm: gather + FM + DNN tower + head, one launch; diagnostic hook
rs_diag_mlp_set_dbg, compiled into the product library behind a null check;
DIAG_DEEPFM_OPT = RS_OPT_DEEPFM_KERNEL, default 1 — the split-role form 0
stamps only the layers after its first):
  0 entry, 1 gather + FM combine done (tower about to start), 2+2l layer l
  after its barrier, 3+2l layer l's contraction done, 15 end.
Prints the median over workgroups of each phase (relative to the workgroup's
first stamp), for the median wave and the slowest wave, and the span."""
import ctypes as C
import json
import os
from pathlib import Path
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import recommender_system_amd as rs
    from recommender_system_amd import _lib
    # the MLP stamps exist only in the diagnostic build (scripts/build_diag.sh)
    _lib._LIB_PATH = Path(ROOT) / "recommender_system_amd" / "librs_hip_diag.so"
    dev = torch.device("cuda")
    B, F, nd, k = int(os.environ.get("DIAG_B", "4096")), 26, 13, 16
    V = int(float(os.environ.get("DIAG_V", "1e6")))
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    m = rs.DeepFM(cols, 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, seed=2, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    NP = 16
    ids = torch.randint(0, V, (NP, B, F), generator=g, device=dev, dtype=torch.int32)
    dense = torch.rand(NP, B, nd, generator=g, device=dev)
    nwg = (B + 15) // 16
    dbg = torch.zeros(nwg * 16 * 16, dtype=torch.int64, device=dev)
    lib = _lib.lib()
    lib.rs_diag_mlp_set_dbg.argtypes = [C.c_void_p]
    _lib.set_option(_lib.OPT_DEEPFM_KERNEL, int(os.environ.get("DIAG_DEEPFM_OPT", "1")))
    for i in range(40):
        m.forward_fused((dense[i % NP], ids[i % NP]), check_ids=False)
    torch.cuda.synchronize()
    lib.rs_diag_mlp_set_dbg(dbg.data_ptr())
    m.forward_fused((dense[0], ids[0]), check_ids=False)
    torch.cuda.synchronize()
    lib.rs_diag_mlp_set_dbg(None)
    d = dbg.cpu().numpy().reshape(nwg, 16, 16).astype(np.int64)
    t0 = d[:, :, 0].min(axis=1, keepdims=True)
    names = {0: "entry", 1: "fm_done"}
    for l in range(4):
        names[2 + 2 * l] = f"l{l}_start"
        names[3 + 2 * l] = f"l{l}_mac_done"
    if int(os.environ.get("DIAG_DEEPFM_OPT", "1")) == 0:  # split roles: slots 2 / 3 = burst 0 / 1 in
        names[2], names[3] = "burst0_in", "burst1_in"
    elif int(os.environ.get("DIAG_DEEPFM_OPT", "1")) == 2:  # every wave on layer 0: after barriers A / B
        names[2], names[3] = "after_A", "after_B"
    names[15] = "end"
    out = {"B": B, "V": V, "deepfm_kernel_option": int(os.environ.get("DIAG_DEEPFM_OPT", "1")), "phases_cycles": {}}
    for j, n in names.items():
        rel = d[:, :, j] - t0
        ok = d[:, :, j] > 0  # waves that wrote this slot
        if not ok.any():
            continue
        relm = np.where(ok, rel, np.nan)
        out["phases_cycles"][n] = {"median_wave": int(np.nanmedian(relm)),
                                   "slowest_wave": int(np.nanmedian(np.nanmax(relm, axis=1))),
                                   "loaders_median": int(np.nanmedian(relm[:, :8])) if ok[:, :8].any() else None,
                                   "compute_median": int(np.nanmedian(relm[:, 8:])) if ok[:, 8:].any() else None}
    st0 = np.where(d[:, :, 0] > 0, d[:, :, 0], np.iinfo(np.int64).max).min(axis=1)  # per-WG first stamp
    kstart = st0.min()
    out["kernel_span_cycles"] = int(d[:, :, 15].max() - kstart)
    out["wg_start_spread_cycles"] = [int(np.percentile(st0 - kstart, 50)), int((st0 - kstart).max())]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
