"""Diagnostic sweep of rs_embed_fm_fwd / rs_embed_gather: kernel time (HIP
events, median of launches) vs vocab size, batch, id pattern.  Prints one
JSON line per point.  Usage: python scripts/sweep_embed_fm.py [--quick]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_system_amd import _lib  # noqa: E402


def time_launches(fn, n=50, warm=5):
    for i in range(warm):
        fn(i)
    torch.cuda.synchronize()
    ms = []
    for i in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn(i)
        e.record()
        ms.append((s, e))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ms]))


def main():
    quick = "--quick" in sys.argv
    dev = torch.device("cuda")
    F, k, kfm, nd = 26, 16, 10, 13
    big_rows = int(os.environ.get("SWEEP_ROWS", str(26 * 10_000_000)))
    table = torch.empty(big_rows, k, device=dev)
    table.uniform_(-0.05, 0.05)
    lib = _lib.lib()
    d = nd + F * k
    w1 = torch.randn(d, 1, device=dev) * 0.05
    v = torch.randn(d, kfm, device=dev) * 0.05
    w0 = torch.zeros(1, device=dev)
    prep = torch.empty(lib.rs_fm_prepared_size(nd, F, k, kfm), device=dev)
    _lib.call("rs_fm_prepare", w1.data_ptr(), v.data_ptr(), nd, F, k, kfm, prep.data_ptr(), 0)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    vocabs = [10_000, 100_000, 1_000_000, 10_000_000] if not quick else [100_000, 10_000_000]
    batches = [4096, 16384, 65536] if not quick else [4096, 65536]
    for V in vocabs:
        offs = torch.arange(F, dtype=torch.int64, device=dev) * V
        voc = torch.full((F,), V, dtype=torch.int64, device=dev)
        for B in batches:
            pool = [torch.randint(0, V, (B, F), dtype=torch.int32, device=dev) for _ in range(8)]
            dense = torch.rand(B, nd, device=dev)
            logit = torch.empty(B, device=dev)
            x = torch.empty(B, d, device=dev)

            def fm(i):
                ids = pool[i % 8]
                lib.rs_embed_fm_fwd(ids.data_ptr(), 0, F, dense.data_ptr(), nd, nd, table.data_ptr(),
                                    offs.data_ptr(), voc.data_ptr(), F, k, prep.data_ptr(), w0.data_ptr(), kfm,
                                    logit.data_ptr(), None, B, err.data_ptr(), 0)

            def gat(i):
                ids = pool[i % 8]
                lib.rs_embed_gather(ids.data_ptr(), 0, F, dense.data_ptr(), nd, nd, table.data_ptr(),
                                    offs.data_ptr(), voc.data_ptr(), F, k, x.data_ptr(), d, B, err.data_ptr(), 0)

            t_fm = time_launches(fm)
            t_g = time_launches(gat)
            alg = B * 1824
            print(json.dumps({"V": V, "table_GB": F * V * k * 4 / 1e9, "B": B, "nw": os.environ.get("RS_FM_NW", "8"),
                              "fm_us": t_fm * 1e3, "fm_GBps": alg / t_fm / 1e6, "gather_us": t_g * 1e3,
                              "gather_GBps": B * (F * 68 + nd * 8 + d * 4) / t_g / 1e6}), flush=True)
    assert int(err.item()) == 0


if __name__ == "__main__":
    main()
