"""Per-layer timing of the tower builds in scripts/ab/librs_tower_{A..D}.so
(rs_mlp_fwd 429-256-128-64-1 with the sigmoid head, B 4096): each build's
diagnostic hook rs_diag_mlp_set_dbg gives per-wave s_memtime stamps (slot
2+2l: layer l after its barrier, 3+2l: its contraction done, 15: end); prints
per build the median over workgroups of each layer's span (barrier to the
slowest wave's contraction) and of the whole tile, as one JSON line."""
import ctypes as C
import json
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    dev = torch.device("cuda")
    P, L, I, F = C.c_void_p, C.c_int64, C.c_int, C.c_float
    B = int(os.environ.get("AB_B", "4096"))
    dims = [429, 256, 128, 64, 1]
    n = len(dims) - 1
    cd = (C.c_int * (n + 1))(*dims)
    acts = (C.c_int * n)(*([1] * (n - 1) + [0]))
    g = torch.Generator(device="cpu").manual_seed(0)
    Ws = [(torch.rand(dims[i], dims[i + 1], generator=g) * 0.1 - 0.05).to(dev) for i in range(n)]
    bs = [(torch.rand(dims[i + 1], generator=g) * 0.1).to(dev) for i in range(n)]
    x = torch.rand(B, dims[0], device=dev)
    nwg = (B + 15) // 16
    out = {}
    for name in "ABCD":
        path = os.path.join(ROOT, "scripts", "ab", f"librs_tower_{name}.so")
        if not os.path.exists(path):
            continue
        lib = C.CDLL(path)
        lib.rs_mlp_prepared_size.restype = L
        lib.rs_mlp_prepared_size.argtypes = [I, P]
        lib.rs_mlp_prepare.argtypes = [I, P, P, P, P, P, P, P]
        lib.rs_mlp_fwd.argtypes = [P, L, I, P, P, P, P, L, I, P, F, F, L, P]
        lib.rs_diag_mlp_set_dbg.argtypes = [P]
        prep = torch.empty(int(lib.rs_mlp_prepared_size(n, cd)), device=dev)
        Wp = (C.c_void_p * n)(*[w.data_ptr() for w in Ws])
        bp = (C.c_void_p * n)(*[b.data_ptr() for b in bs])
        assert lib.rs_mlp_prepare(n, cd, Wp, bp, None, None, prep.data_ptr(), None) == 0
        y = torch.empty(B, device=dev)
        run = lambda: lib.rs_mlp_fwd(x.data_ptr(), dims[0], n, cd, acts, prep.data_ptr(), y.data_ptr(), 1, 1, None,
                                     1.0, 0.0, B, torch.cuda.current_stream().cuda_stream)
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        dbg = torch.zeros(nwg * 256, dtype=torch.int64, device=dev)
        lib.rs_diag_mlp_set_dbg(dbg.data_ptr())
        run()
        torch.cuda.synchronize()
        lib.rs_diag_mlp_set_dbg(None)
        d = dbg.cpu().numpy().reshape(nwg, 16, 16).astype(np.float64)
        d[d == 0] = np.nan
        t0 = np.nanmin(d[:, :, 0], axis=1)
        res = {}
        for l in range(n):
            bar, mac = d[:, :, 2 + 2 * l], d[:, :, 3 + 2 * l]
            if np.isnan(bar).all():
                continue
            res[f"l{l}"] = int(np.nanmedian(np.nanmax(mac, axis=1) - np.nanmin(bar, axis=1))) \
                if not np.isnan(mac).all() else None
            res[f"l{l}_start"] = int(np.nanmedian(np.nanmin(bar, axis=1) - t0))
        res["end"] = int(np.nanmedian(np.nanmax(d[:, :, 15], axis=1) - t0))
        # what bounds the launch: workgroup start offsets and durations; the
        # s_memtime counters of different XCDs are not aligned, so offsets are
        # taken within each XCD (workgroup i runs on XCD i mod 8)
        xcd = np.arange(nwg) % 8
        start = np.empty(nwg)
        for xc in range(8):
            sel = xcd == xc
            start[sel] = t0[sel] - np.nanmin(t0[sel])
        dur = np.nanmax(d[:, :, 15], axis=1) - t0
        pct = lambda v: [int(np.nanpercentile(v, q)) for q in (0, 50, 90, 100)]
        res["wg_start_in_xcd_p0_50_90_100"] = pct(start)
        res["wg_duration_p0_50_90_100"] = pct(dur)
        res["span_in_xcd_max"] = int(np.nanmax(start + dur))
        out[name] = res
    print(json.dumps({"workload": f"rs_mlp_fwd {dims}, B {B}", "cycles": out}))


if __name__ == "__main__":
    main()
