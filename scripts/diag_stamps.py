"""Phase timeline of one rs_embed_fm_fwd launch (diagnostic library with
s_memrealtime stamps, 100 MHz): per workgroup/wave
  t0 start -> t1 ids decoded -> t2 rows (+weights) arrived -> t3 MFMAs done -> t4 end (wave 0).
Prints percentiles (us) relative to the earliest t0 of the launch."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    lib = C.CDLL(os.path.join(ROOT, "recommender_system_amd", "librs_hip_diag.so"))
    P, L, I = C.c_void_p, C.c_int64, C.c_int
    lib.rs_diag_embed_fm_fwd.argtypes = [P, I, L, P, L, I, P, P, P, I, I, P, P, I, P, L, P, P]
    lib.rs_fm_prepare.argtypes = [P, P, I, I, I, I, P, P]
    lib.rs_fm_prepared_size.restype = L
    dev = torch.device("cuda")
    F, k, kfm, nd = 26, 16, 10, 13
    V = int(float(os.environ.get("DIAG_V", "1e7")))
    B = int(os.environ.get("DIAG_B", "4096"))
    table = torch.empty(F * V, k, device=dev).uniform_(-0.05, 0.05)
    d = nd + F * k
    w1 = torch.randn(d, 1, device=dev) * 0.05
    v = torch.randn(d, kfm, device=dev) * 0.05
    w0 = torch.zeros(1, device=dev)
    prep = torch.empty(lib.rs_fm_prepared_size(nd, F, k, kfm), device=dev)
    st = torch.cuda.current_stream().cuda_stream
    lib.rs_fm_prepare(w1.data_ptr(), v.data_ptr(), nd, F, k, kfm, prep.data_ptr(), st)
    offs = torch.arange(F, dtype=torch.int64, device=dev) * V
    voc = torch.full((F,), V, dtype=torch.int64, device=dev)
    NP = int(os.environ.get("DIAG_POOL", "8"))
    pool = [torch.randint(0, V, (B, F), dtype=torch.int32, device=dev) for _ in range(NP)]
    dense = torch.rand(B, nd, device=dev)
    logit = torch.empty(B, device=dev)
    nwg = (B + 15) // 16
    NW = 16
    dbg = torch.zeros(nwg * NW * 12, dtype=torch.int64, device=dev)
    for i in range(40):
        ids = pool[i % NP]
        dp = dbg.data_ptr() if i == 39 else None
        lib.rs_diag_embed_fm_fwd(ids.data_ptr(), 0, F, dense.data_ptr(), nd, nd, table.data_ptr(), offs.data_ptr(),
                                 voc.data_ptr(), F, k, prep.data_ptr(), w0.data_ptr(), kfm, logit.data_ptr(), B,
                                 dp, st)
    torch.cuda.synchronize()
    t = dbg.cpu().numpy().reshape(nwg, NW, 12).astype(np.float64) / 100.0  # us
    t8 = np.where(t[:, :, 8] > 0, t[:, :, 8], np.nan)
    base = t[:, :, 0].min()
    pct = lambda a: {p: round(float(np.percentile(a, p)), 3) for p in (0, 50, 90, 100)}
    out = {"V": V, "B": B, "pool": NP,
           "t0_start": pct(t[:, :, 0] - base),
           "kernarg (t5-t0)": pct(t[:, :, 5] - t[:, :, 0]),
           "issue (t6-t5)": pct(t[:, :, 6] - t[:, :, 5]),
           "ids wait (t1-t6)": pct(t[:, :, 1] - t[:, :, 6]),
           "id load return (t8-t5, loading lanes)": {p: round(float(np.nanpercentile(t8 - t[:, :, 5], p)), 3)
                                                     for p in (0, 50, 90, 100)},
           "barrier (t9-t8)": {p: round(float(np.nanpercentile(t[:, :, 9] - t8, p)), 3) for p in (0, 50, 90, 100)},
           "t9 after barrier": pct(t[:, :, 9] - base),
           "rows (t2-t1)": pct(t[:, :, 2] - t[:, :, 1]),
           "mfma (t3-t2)": pct(t[:, :, 3] - t[:, :, 2]),
           "barrier wait (t7-t3, wave0)": pct(t[:, 0, 7] - t[:, 0, 3]),
           "combine (t4-t7, wave0)": pct(t[:, 0, 4] - t[:, 0, 7]),
           "slowest wave t3 in WG": pct(t[:, :, 3].max(1) - base),
           "end (t4)": pct(t[:, 0, 4] - base),
           "span_us": round(float(t[:, 0, 4].max() - base), 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
