"""Times the gather-structure kernels of scripts/diag_gather_shapes.hip
(graph-replayed, 64-batch id pool, 26 x 1e7 x 16 table) next to the headline
kernel rs_embed_fm_fwd (RS_OPT_EMBED_FM_KERNEL 0) at B = 4096 and 16384.
Prints one JSON line per batch size: median us per launch slot."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from recommender_system_amd import _lib
    dev = torch.device("cuda")
    lib = _lib.lib()
    dg = C.CDLL(os.path.join(ROOT, "scripts", "ab", "libdiag_gather.so"))
    dg.diag_gather.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.c_void_p]
    F, k, kfm, nd, V = 26, 16, 10, 13, int(1e7)
    table = torch.empty(F * V, k, device=dev).uniform_(-0.05, 0.05)
    offs = torch.arange(F, dtype=torch.int64, device=dev) * V
    voc = torch.full((F,), V, dtype=torch.int64, device=dev)
    d = nd + F * k
    w1 = torch.randn(d, 1, device=dev) * 0.05
    v = torch.randn(d, kfm, device=dev) * 0.05
    w0 = torch.zeros(1, device=dev)
    prep = torch.empty(lib.rs_fm_prepared_size(nd, F, k, kfm), device=dev)
    _lib.call("rs_fm_prepare", w1.data_ptr(), v.data_ptr(), nd, F, k, kfm, prep.data_ptr(), _lib.stream())
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    prep32 = prep.repeat(32).contiguous()  # 32 copies (ablation bit 7)
    variants = [int(x) for x in os.environ.get("DIAG_VARIANTS", "0,1,2,3,4,5,6").split(",") if x]
    abls = [int(x) for x in os.environ.get("DIAG_ABL", "").split(",") if x]
    dg.diag_fm_abl.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int64,
                               C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                               C.c_int64, C.c_void_p]
    DB = (nd + 3) // 4
    dense_rec, field_rec = 64 + 4, 64 * 4 + 16
    field_base = DB * dense_rec
    NP = 64
    hmv = [int(x) for x in os.environ.get("DIAG_HM_VARIANTS", "").split(",") if x]
    hoff = (C.c_int64 * F)(*[c * V for c in range(F)])
    hvoc = (C.c_int64 * F)(*([V] * F))
    for B in [int(x) for x in os.environ.get("DIAG_BATCHES", "4096,16384").split(",")]:
        pool = torch.randint(0, V, (NP, B, F), dtype=torch.int32, device=dev)
        dense = torch.rand(NP, B, nd, device=dev)
        out = torch.empty(B * F, device=dev)
        logit = torch.empty(B, device=dev)
        fns = {}
        for vv in variants:
            fns[f"g{vv}"] = (lambda i, vv=vv: dg.diag_gather(vv, pool[i % NP].data_ptr(), table.data_ptr(),
                                                             offs.data_ptr(), F, B, out.data_ptr(),
                                                             torch.cuda.current_stream().cuda_stream))
        for ab in abls:
            fns[f"abl{ab}"] = (lambda i, ab=ab: dg.diag_fm_abl(ab, pool[i % NP].data_ptr(), table.data_ptr(),
                                                               offs.data_ptr(), voc.data_ptr(), F, kfm, B,
                                                               (prep32 if ab & 128 else prep).data_ptr(), dense_rec,
                                                               field_rec, field_base, nd, DB, dense[i % NP].data_ptr(),
                                                               logit.data_ptr(), prep.numel(),
                                                               torch.cuda.current_stream().cuda_stream))
        fns["embed_fm"] = lambda i: lib.rs_embed_fm_fwd(pool[i % NP].data_ptr(), 0, F, dense[i % NP].data_ptr(), nd,
                                                        nd, table.data_ptr(), offs.data_ptr(), voc.data_ptr(), F, k,
                                                        prep.data_ptr(), w0.data_ptr(), kfm, logit.data_ptr(), None, B,
                                                        err.data_ptr(), torch.cuda.current_stream().cuda_stream)
        for hv in hmv:  # the product's headline entry (kernarg metadata), RS_OPT_EMBED_FM_KERNEL = hv
            def hm_fn(i, hv=hv):
                _lib.set_option(_lib.OPT_EMBED_FM_KERNEL, hv)
                lib.rs_embed_fm_fwd_hm(pool[i % NP].data_ptr(), 0, F, dense[i % NP].data_ptr(), nd, nd,
                                       table.data_ptr(), offs.data_ptr(), voc.data_ptr(), C.addressof(hoff),
                                       C.addressof(hvoc), F, k, prep.data_ptr(), w0.data_ptr(), kfm, logit.data_ptr(),
                                       None, B, err.data_ptr(), torch.cuda.current_stream().cuda_stream)
                _lib.set_option(_lib.OPT_EMBED_FM_KERNEL, 0)
            fns[f"hm{hv}"] = hm_fn
        # correctness of the ablations that keep the arithmetic (bits 0, 4, 5 only)
        chk = {}
        fns["embed_fm"](0)
        ref = logit.clone()
        rms = float(ref.pow(2).mean().sqrt())
        for ab in abls:
            if ab & ~(1 | 16 | 32 | 64 | 128) == 0:
                fns[f"abl{ab}"](0)
                torch.cuda.synchronize()
                chk[f"abl{ab}"] = float(((logit - ref).abs() / ref.abs().clamp_min(rms)).max())
        graphs = {}
        for name, fn in fns.items():
            for i in range(NP):
                fn(i)
            torch.cuda.synchronize()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    for i in range(NP):
                        fn(i)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            graphs[name] = g
        res = {n: [] for n in graphs}
        names = list(graphs)
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
        print(json.dumps({"batch": B, "us_per_launch_median": {n: round(float(np.median(x)), 3) for n, x in res.items()},
                          "max_scaled_diff_vs_embed_fm": chk}), flush=True)


if __name__ == "__main__":
    main()
