"""A/B of the DCN / PNN kernels' front ends on one box:
the cooperative id tile (rs_embed_cross_fwd, rs_dcn_fwd, rs_embed_inner_fwd)
against the headline kernel's kernel-argument front end (the _hm entries),
config-3 shapes: 26 fields x 1e6 rows x 16, 13 dense, B 4096, CrossNet depth
3, DNN 256-128-64.  Graph-replayed, arms alternated over rounds; prints one
JSON line of medians (us per launch slot) and whether each pair is bit-equal."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import recommender_system_amd as rs
    from recommender_system_amd import _lib
    dev = torch.device("cuda")
    B, F, V, k, nd = int(os.environ.get("DIAG_B", "4096")), 26, int(1e6), 16, 13
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    m = rs.DCN(cols, [256, 128, 64], 1, "relu", layer_num=3, embed_dim=k, seed=1, device=dev)
    p = rs.PNN(cols, "inner", [256, 128, 64], 1, embed_dim=k, seed=1, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    NP = 64
    ids = torch.randint(0, V, (NP, B, F), generator=g, device=dev, dtype=torch.int32)
    dense = torch.rand(NP, B, nd, generator=g, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    d = m.d
    e, pe = m.embed_layer, p.embed_layer
    prep = m.cross_layer.prepared(d)
    cross, mlp, dims, acts, _ = m._fused_params()
    n = len(dims) - 1
    cd, ca = (C.c_int * (n + 1))(*dims), (C.c_int * n)(*acts)
    P = F * (F - 1) // 2
    outs = {name: torch.empty(NP, B, w, device=dev) for name, w in (("cross", d), ("dcn", 1), ("inner", F * k + P))}
    st = lambda: torch.cuda.current_stream().cuda_stream

    def cross_fn(hm):
        def fn(i):
            j = i % NP
            head = (ids[j].data_ptr(), 0, F, dense[j].data_ptr(), nd, nd, e.table.data_ptr(), e.field_offsets.data_ptr(),
                    e.field_vocab.data_ptr())
            tail = (F, k, 3, prep.data_ptr(), outs["cross"][j].data_ptr(), d, B, err.data_ptr(), st())
            if hm:
                _lib.call("rs_embed_cross_fwd_hm", *head, *e.host_meta(), *tail)
            else:
                _lib.call("rs_embed_cross_fwd", *head, *tail)
        return fn

    def dcn_fn(hm):
        def fn(i):
            j = i % NP
            head = (ids[j].data_ptr(), 0, F, dense[j].data_ptr(), nd, nd, e.table.data_ptr(), e.field_offsets.data_ptr(),
                    e.field_vocab.data_ptr())
            tail = (F, k, 3, cross.data_ptr(), n, cd, ca, mlp.data_ptr(), outs["dcn"][j].data_ptr(), B,
                    err.data_ptr(), st())
            if hm:
                _lib.call("rs_dcn_fwd_hm", *head, *e.host_meta(), *tail)
            else:
                _lib.call("rs_dcn_fwd", *head, *tail)
        return fn

    def inner_fn(hm):
        def fn(i):
            j = i % NP
            head = (ids[j].data_ptr(), 0, F, pe.table.data_ptr(), pe.field_offsets.data_ptr(), pe.field_vocab.data_ptr())
            tail = (F, k, outs["inner"][j].data_ptr(), F * k + P, B, err.data_ptr(), st())
            if hm:
                _lib.call("rs_embed_inner_fwd_hm", *head, *pe.host_meta(), *tail)
            else:
                _lib.call("rs_embed_inner_fwd", *head, *tail)
        return fn

    arms = {f"{name}_{'hm' if hm else 'tile'}": mk(hm) for name, mk in (("cross", cross_fn), ("dcn", dcn_fn),
                                                                          ("inner", inner_fn)) for hm in (False, True)}
    graphs, first = {}, {}
    for name, fn in arms.items():
        for i in range(NP):
            fn(i)
        torch.cuda.synchronize()
        first[name] = outs[name.split("_")[0]].clone()
        gr = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(gr, stream=s):
                for i in range(NP):
                    fn(i)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graphs[name] = gr
    res = {nm: [] for nm in graphs}
    names = list(graphs)
    for r in range(8):
        for nm in (names if r % 2 == 0 else names[::-1]):
            gr = graphs[nm]
            gr.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                gr.replay()
            e1.record()
            torch.cuda.synchronize()
            res[nm].append(e0.elapsed_time(e1) * 1e3 / (10 * NP))
    assert int(err.item()) == 0
    print(json.dumps({"batch": B, "us_per_launch_median": {nm: round(float(np.median(v)), 3) for nm, v in res.items()},
                      "bit_equal": {nm: bool(torch.equal(first[f"{nm}_tile"], first[f"{nm}_hm"]))
                                    for nm in ("cross", "dcn", "inner")}}))


if __name__ == "__main__":
    main()
