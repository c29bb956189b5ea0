"""Phase timeline of one rs_embed_fm_fwd launch through embed_fm_hot (diagnostic
library, s_memrealtime stamps at 100 MHz), per wave: t0 start, t6 first-trip
loads issued, t1 own ids decoded, t2 first field's MFMAs done, t3 all MFMAs
done, t7 after the combine barrier, t4 end.  Percentiles (us) vs the earliest t0."""
import ctypes as C
import json
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
    NP = 8
    pool = [torch.randint(0, V, (B, F), dtype=torch.int32, device=dev) for _ in range(NP)]
    dense = torch.rand(B, nd, device=dev)
    logit = torch.empty(B, device=dev)
    nwg, NW = (B + 15) // 16, 16
    dbg = torch.zeros(nwg * NW * 12, dtype=torch.int64, device=dev)
    for i in range(40):
        lib.rs_diag_embed_fm_fwd(pool[i % NP].data_ptr(), 0, F, dense.data_ptr(), nd, nd, table.data_ptr(),
                                 offs.data_ptr(), voc.data_ptr(), F, k, prep.data_ptr(), w0.data_ptr(), kfm,
                                 logit.data_ptr(), B, dbg.data_ptr() if i == 39 else None, st)
    torch.cuda.synchronize()
    t = dbg.cpu().numpy().reshape(nwg, NW, 12).astype(np.float64) / 100.0
    base = t[:, :, 0].min()
    pct = lambda a: {p: round(float(np.nanpercentile(a, p)), 3) for p in (0, 50, 90, 100)}
    has1 = np.arange(NW) + NW < F
    out = {"V": V, "B": B,
           "t0 start": pct(t[:, :, 0] - base),
           "issue (t6-t0)": pct(t[:, :, 6] - t[:, :, 0]),
           "ids (t1-t6)": pct(t[:, :, 1] - t[:, :, 6]),
           "t1 abs": pct(t[:, :, 1] - base),
           "row0+mfma (t2-t1)": pct(t[:, :, 2] - t[:, :, 1]),
           "row1+mfma (t3-t2), 2-field waves": pct((t[:, :, 3] - t[:, :, 2])[:, has1]),
           "t3 abs": pct(t[:, :, 3] - base),
           "slowest t3 in WG": pct(t[:, :, 3].max(1) - base),
           "barrier (t7 - slowest t3)": pct(t[:, :, 7].min(1) - t[:, :, 3].max(1)),
           "combine (t4-t7)": pct(t[:, :, 4] - t[:, :, 7]),
           "end (t4 max per WG)": pct(t[:, :, 4].max(1) - base),
           "span_us": round(float(t[:, :, 4].max() - base), 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
