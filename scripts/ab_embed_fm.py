"""A/B timing of rs_embed_fm_fwd from two builds (scripts/build_ab.sh) on the
same table and batches, graph-replayed, alternating A and B so drift on the
box hits both.  Prints one JSON line per round and the medians."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bind(path):
    lib = C.CDLL(path)
    P, L, I = C.c_void_p, C.c_int64, C.c_int
    lib.rs_embed_fm_fwd.argtypes = [P, I, L, P, L, I, P, P, P, I, I, P, P, I, P, P, L, P, P]
    lib.has_hm = hasattr(lib, "rs_embed_fm_fwd_hm")
    if lib.has_hm:  # the host-metadata entry (the product's headline path)
        lib.rs_embed_fm_fwd_hm.argtypes = [P, I, L, P, L, I, P, P, P, P, P, I, I, P, P, I, P, P, L, P, P]
    lib.rs_fm_prepare.argtypes = [P, P, I, I, I, I, P, P]
    lib.rs_fm_prepared_size.restype = L
    lib.rs_fm_prepared_size.argtypes = [I, I, I, I]
    return lib


def main():
    dev = torch.device("cuda")
    names = [n for n in "ABCD" if os.path.exists(os.path.join(ROOT, "scripts", "ab", f"librs_ab_{n}.so"))]
    libs = {n: bind(os.path.join(ROOT, "scripts", "ab", f"librs_ab_{n}.so")) for n in names}
    F, k, kfm, nd = 26, 16, 10, 13
    V = int(float(os.environ.get("DIAG_V", "1e7")))
    B = int(os.environ.get("DIAG_B", "4096"))
    table = torch.empty(F * V, k, device=dev).uniform_(-0.05, 0.05)
    d = nd + F * k
    w1 = torch.randn(d, 1, device=dev) * 0.05
    v = torch.randn(d, kfm, device=dev) * 0.05
    w0 = torch.zeros(1, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    offs = torch.arange(F, dtype=torch.int64, device=dev) * V
    voc = torch.full((F,), V, dtype=torch.int64, device=dev)
    hoff = (C.c_int64 * F)(*[c * V for c in range(F)])
    hvoc = (C.c_int64 * F)(*([V] * F))
    NP = 64
    pool = torch.randint(0, V, (NP, B, F), dtype=torch.int32, device=dev)
    dense = torch.rand(NP, B, nd, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    outs, graphs = {}, {}
    for n, lib in libs.items():
        prep = torch.empty(lib.rs_fm_prepared_size(nd, F, k, kfm), device=dev)
        lib.rs_fm_prepare(w1.data_ptr(), v.data_ptr(), nd, F, k, kfm, prep.data_ptr(), st)
        logit = torch.empty(NP, B, device=dev)

        def fn(i, lib=lib, prep=prep, logit=logit):
            j = i % NP
            if lib.has_hm and not os.environ.get("AB_NO_HM"):
                lib.rs_embed_fm_fwd_hm(pool[j].data_ptr(), 0, F, dense[j].data_ptr(), nd, nd, table.data_ptr(),
                                       offs.data_ptr(), voc.data_ptr(), C.addressof(hoff), C.addressof(hvoc), F, k,
                                       prep.data_ptr(), w0.data_ptr(), kfm, logit[j].data_ptr(), None, B,
                                       err.data_ptr(), torch.cuda.current_stream().cuda_stream)
                return
            lib.rs_embed_fm_fwd(pool[j].data_ptr(), 0, F, dense[j].data_ptr(), nd, nd, table.data_ptr(),
                                offs.data_ptr(), voc.data_ptr(), F, k, prep.data_ptr(), w0.data_ptr(), kfm,
                                logit[j].data_ptr(), None, B, err.data_ptr(), torch.cuda.current_stream().cuda_stream)

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            for i in range(NP):
                fn(i)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for i in range(NP):
                    fn(i)
        torch.cuda.synchronize()
        graphs[n], outs[n] = g, logit
    res = {n: [] for n in names}
    for r in range(8):
        for n in (names if r % 2 == 0 else names[::-1]):
            g = graphs[n]
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            res[n].append(e0.elapsed_time(e1) * 1e3 / (10 * NP))
    ref = outs["A"]
    rms = float(ref.pow(2).mean().sqrt())
    diff = {n: float(((outs[n] - ref).abs() / ref.abs().clamp_min(rms)).max()) for n in names}
    print(json.dumps({**{"us_per_launch_" + n: [round(x, 3) for x in res[n]] for n in names},
                      **{"median_" + n: round(float(np.median(res[n])), 3) for n in names},
                      "max_scaled_diff_vs_A": diff, "err": int(err.item())}))


if __name__ == "__main__":
    main()
