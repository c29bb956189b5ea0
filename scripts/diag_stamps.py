"""Phase timeline of one rs_embed_fm_fwd launch (diagnostic library with
s_memrealtime stamps, 100 MHz, scripts/build_diag.sh): per workgroup / wave
  t0 start, t5 kernel arguments, per pass p (0: t6 row issue, t1 ids decoded,
  t2 rows arrived, t13 MFMAs done; 1: t10, t11, t12, t14), t3 wave's MFMAs
  done (dense included), t7 combine barrier released, t4 end (wave 0).
RS_DIAG_HM=1 runs the kernarg-metadata kernel (rs_embed_fm_fwd_hm's), DIAG_OPT
sets RS_OPT_EMBED_FM_KERNEL.  Prints percentiles (us) relative to the
earliest t0 of the launch."""
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
    lib.rs_set_option(0, int(os.environ.get("DIAG_OPT", "0")))
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
    NW, NS = 16, 16
    dbg = torch.zeros(nwg * NW * NS, dtype=torch.int64, device=dev)
    for i in range(40):
        ids = pool[i % NP]
        dp = dbg.data_ptr() if i == 39 else None
        lib.rs_diag_embed_fm_fwd(ids.data_ptr(), 0, F, dense.data_ptr(), nd, nd, table.data_ptr(), offs.data_ptr(),
                                 voc.data_ptr(), F, k, prep.data_ptr(), w0.data_ptr(), kfm, logit.data_ptr(), B,
                                 dp, st)
    torch.cuda.synchronize()
    t = dbg.cpu().numpy().reshape(nwg, NW, NS).astype(np.float64) / 100.0  # us
    t[t == 0] = np.nan
    base = np.nanmin(t[:, :, 0])
    pct = lambda a: {p: round(float(np.nanpercentile(a, p)), 3) for p in (0, 10, 50, 90, 100)}
    two = F - NW  # waves 0 .. two-1 carry a second field
    w2, w1 = slice(0, max(two, 0)), slice(max(two, 0), NW)
    out = {"V": V, "B": B, "pool": NP, "hm": bool(os.environ.get("RS_DIAG_HM")),
           "option": int(os.environ.get("DIAG_OPT", "0")),
           "start (t0)": pct(t[:, :, 0] - base),
           "kernarg (t5-t0)": pct(t[:, :, 5] - t[:, :, 0]),
           "p0 ids decoded (t1 - t0)": pct(t[:, :, 1] - t[:, :, 0]),
           "p0 rows arrived (t2 - t1)": pct(t[:, :, 2] - t[:, :, 1]),
           "p0 mfma (t13 - t2)": pct(t[:, :, 13] - t[:, :, 2]),
           "p1 ids decoded (t11 - t0)": pct(t[:, w2, 11] - t[:, w2, 0]),
           "p1 row issue after p0 rows (t10 - t2)": pct(t[:, w2, 10] - t[:, w2, 2]),
           "p1 rows arrived (t12 - t10)": pct(t[:, w2, 12] - t[:, w2, 10]),
           "p1 mfma (t14 - t12)": pct(t[:, w2, 14] - t[:, w2, 12]),
           "wave done (t3) 2-field waves": pct(t[:, w2, 3] - base),
           "wave done (t3) 1-field waves": pct(t[:, w1, 3] - base),
           "slowest wave t3 in WG": pct(np.nanmax(t[:, :, 3], 1) - base),
           "barrier released (t7)": pct(t[:, 0, 7] - base),
           "combine (t4 - t7, wave 0)": pct(t[:, 0, 4] - t[:, 0, 7]),
           "end (t4)": pct(t[:, 0, 4] - base),
           "span_us": round(float(np.nanmax(t[:, 0, 4]) - base), 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
