"""Same-box timing of tower build variants (scripts/ab/librs_tower_{A..D}.so,
each `hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include
-I recommender_system_amd/csrc <flags> csrc/mlp.hip csrc/capi.cpp`): the
DeepFM DNN tower 429-256-128-64-1 with the sigmoid head (rs_mlp_fwd) at
B 4096, graph-replayed (64 launches per replay), variants alternated, outputs
compared bitwise with A.  Prints one JSON line."""
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
    acts = (C.c_int * n)(*([1] * (n - 1) + [0]))  # relu hidden, linear last (RS_ACT_RELU = 1)
    g = torch.Generator(device="cpu").manual_seed(0)
    Ws = [(torch.rand(dims[i], dims[i + 1], generator=g) * 0.1 - 0.05).to(dev) for i in range(n)]
    bs = [(torch.rand(dims[i + 1], generator=g) * 0.1).to(dev) for i in range(n)]
    NP = 64
    x = torch.rand(NP, B, dims[0], device=dev)
    names = [v for v in "ABCD" if os.path.exists(os.path.join(ROOT, "scripts", "ab", f"librs_tower_{v}.so"))]
    graphs, outs, res = {}, {}, {}
    for name in names:
        lib = C.CDLL(os.path.join(ROOT, "scripts", "ab", f"librs_tower_{name}.so"))
        lib.rs_mlp_prepared_size.restype = L
        lib.rs_mlp_prepared_size.argtypes = [I, P]
        lib.rs_mlp_prepare.argtypes = [I, P, P, P, P, P, P, P]
        lib.rs_mlp_fwd.argtypes = [P, L, I, P, P, P, P, L, I, P, F, F, L, P]
        prep = torch.empty(int(lib.rs_mlp_prepared_size(n, cd)), device=dev)
        Wp = (C.c_void_p * n)(*[w.data_ptr() for w in Ws])
        bp = (C.c_void_p * n)(*[b.data_ptr() for b in bs])
        assert lib.rs_mlp_prepare(n, cd, Wp, bp, None, None, prep.data_ptr(), None) == 0
        y = torch.empty(NP, B, device=dev)

        def fn(i, lib=lib, prep=prep, y=y):
            j = i % NP
            lib.rs_mlp_fwd(x[j].data_ptr(), dims[0], n, cd, acts, prep.data_ptr(), y[j].data_ptr(), 1, 1, None,
                           1.0, 0.0, B, torch.cuda.current_stream().cuda_stream)

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            for i in range(NP):
                fn(i)
            torch.cuda.synchronize()
            with torch.cuda.graph(gr, stream=s):
                for i in range(NP):
                    fn(i)
        torch.cuda.synchronize()
        graphs[name], outs[name], res[name] = gr, (y, prep), []
    for r in range(8):
        for name in (names if r % 2 == 0 else names[::-1]):
            graphs[name].replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                graphs[name].replay()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / (10 * NP))
    ref = outs["A"][0]
    print(json.dumps({"workload": f"rs_mlp_fwd 429-256-128-64-1 head, B {B}",
                      **{f"median_us_{k}": round(float(np.median(v)), 3) for k, v in res.items()},
                      **{f"us_{k}": [round(t, 3) for t in v] for k, v in res.items()},
                      "bit_identical_to_A": {k: bool(torch.equal(o[0], ref)) for k, o in outs.items()}}))


if __name__ == "__main__":
    main()
