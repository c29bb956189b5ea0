"""Launch-regime diagnostics for the headline kernel: per-launch time when
launched back to back from the host, when replayed from a HIP graph, and the
floor set by a near-empty kernel.  Prints JSON lines."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_system_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda")
    F, k, kfm, nd = 26, 16, 10, 13
    V = int(float(os.environ.get("DIAG_V", "1e7")))
    lib = _lib.lib()
    table = torch.empty(F * V, k, device=dev)
    table.uniform_(-0.05, 0.05)
    d = nd + F * k
    w1 = torch.randn(d, 1, device=dev) * 0.05
    v = torch.randn(d, kfm, device=dev) * 0.05
    w0 = torch.zeros(1, device=dev)
    prep = torch.empty(lib.rs_fm_prepared_size(nd, F, k, kfm), device=dev)
    _lib.call("rs_fm_prepare", w1.data_ptr(), v.data_ptr(), nd, F, k, kfm, prep.data_ptr(), _lib.stream())
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    offs = torch.arange(F, dtype=torch.int64, device=dev) * V
    voc = torch.full((F,), V, dtype=torch.int64, device=dev)
    one = torch.zeros(1, device=dev)
    for B in (4096, 65536):
        pool = [torch.randint(0, V, (B, F), dtype=torch.int32, device=dev) for _ in range(16)]
        dense = torch.rand(B, nd, device=dev)
        logit = torch.empty(B, device=dev)

        def fm(i):
            ids = pool[i % 16]
            lib.rs_embed_fm_fwd(ids.data_ptr(), 0, F, dense.data_ptr(), nd, nd, table.data_ptr(), offs.data_ptr(),
                                voc.data_ptr(), F, k, prep.data_ptr(), w0.data_ptr(), kfm, logit.data_ptr(), None,
                                B, err.data_ptr(), _lib.stream())

        def empty(i):
            lib.rs_sigmoid_combine(one.data_ptr(), None, 1.0, 0.0, one.data_ptr(), 1, _lib.stream())

        for name, fn in (("embed_fm", fm), ("empty", empty)):
            # back to back from the host
            for i in range(200):
                fn(i)
            torch.cuda.synchronize()
            n = 2000
            t0 = time.perf_counter()
            for i in range(n):
                fn(i)
            torch.cuda.synchronize()
            host_us = (time.perf_counter() - t0) / n * 1e6
            # graph replay
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            per = 64
            with torch.cuda.stream(s):
                for i in range(3):
                    fn(i)
                torch.cuda.synchronize()
                with torch.cuda.graph(g, stream=s):
                    for i in range(per):
                        fn(i)
            torch.cuda.synchronize()
            for _ in range(5):
                g.replay()
            torch.cuda.synchronize()
            reps = 50
            t0 = time.perf_counter()
            for _ in range(reps):
                g.replay()
            torch.cuda.synchronize()
            graph_us = (time.perf_counter() - t0) / (reps * per) * 1e6
            print(json.dumps({"kernel": name, "V": V, "B": B, "host_loop_us_per_launch": host_us,
                              "graph_us_per_launch": graph_us,
                              "graph_GBps": (B * 1824 / graph_us / 1e3) if name == "embed_fm" else None}),
                  flush=True)
    assert int(err.item()) == 0


if __name__ == "__main__":
    main()
