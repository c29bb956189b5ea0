"""A/B timing of a runtime option (rs_set_option) on one workload, values
alternated in rounds so drift on the box hits every arm; each arm is
graph-replayed (the option is read at capture time).

  python scripts/ab_options.py --option mlp_flow --workload deepfm
  python scripts/ab_options.py --option embed_fm_kernel --workload embed_fm --batch 16384

Prints one JSON line: per value the median us per launch and the max scaled
difference of its output against value 0's.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

OPTS = {"embed_fm_kernel": 0, "mlp_unroll": 1, "deepfm_kernel": 2, "din_kernel": 3, "cross_kernel": 5}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--option", default="embed_fm_kernel", choices=sorted(OPTS))
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--workload", default="deepfm",
                    choices=["deepfm", "dcn", "cross", "embed_fm", "din", "mlp", "din_tower", "shard_pipe", "peer_gather", "din_forward",
                             "gather_rows", "pnn", "embed_x"])
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--vocab", type=float, default=1e7)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--pool", type=int, default=64)
    ap.add_argument("--save", default=None, help="save the first value's outputs here (.pt)")
    ap.add_argument("--compare", default=None, help="compare the first value's outputs with a saved .pt")
    ap.add_argument("--hist", default="pad80", choices=["pad80", "random", "full"],
                    help="din: history padding (from position 80 / random lengths 1..T as bench.py / none)")
    ap.add_argument("--vocab-all", action="store_true", help="use --vocab for every workload (default: embed_fm only)")
    ap.add_argument("--lib", default=None, help="another build of librs_hip.so (build A/B: one process per build)")
    args = ap.parse_args()
    import recommender_system_amd as rs
    from recommender_system_amd import _lib
    if args.lib:
        from pathlib import Path
        _lib._LIB_PATH = Path(args.lib).resolve()
        _lib._ALLOW_MISSING = True

    dev = torch.device("cuda")
    B, F, k, nd = args.batch, 26, 16, 13
    V = int(args.vocab) if args.workload == "embed_fm" or args.vocab_all else int(1e6)
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    NP = args.pool
    ids = torch.randint(0, V, (NP, B, F), generator=g, device=dev, dtype=torch.int32)
    dense = torch.rand(NP, B, nd, generator=g, device=dev)
    if args.workload == "din":  # config 4: the attention unit from ids, B 2048, T 100, k 8, (80, 40)
        Bd, T, kd, Vd = 2048 if args.batch == 4096 else args.batch, 100, 8, 63001
        B = Bd
        layer = rs.Attention((80, 40), "prelu", seed=1)
        layer.build(T, kd)
        table = torch.randn(Vd, kd, device=dev, generator=g)
        hist_p = torch.randint(1, Vd, (NP, Bd, T), generator=g, device=dev)
        if args.hist == "pad80":
            hist_p[:, :, 80:] = 0  # padded tails, as Amazon-Electronics histories
        elif args.hist == "random":  # bench.py's config-4 lengths
            lens = torch.randint(1, T + 1, (NP, Bd, 1), generator=g, device=dev)
            hist_p = torch.where(torch.arange(T, device=dev)[None, None, :] < lens, hist_p, torch.zeros_like(hist_p))
        cand_p = torch.randint(1, Vd, (NP, Bd, 1), generator=g, device=dev)

        def fn(i):
            outs[i % NP] = layer.forward_ids(table, Vd, hist_p[i % NP], cand_p[i % NP])
    elif args.workload == "shard_pipe":  # the sharded FM's pipe launch at world 1 (no exchange), 26 x 1e7
        from recommender_system_amd.sharded import ShardedEmbeddingFM
        V = int(args.vocab)
        sh = ShardedEmbeddingFM([V] * F, k, nd, 10, device=dev, seed=3, world=1, rank=0)
        idsv = torch.randint(0, V, (NP, B, F), generator=g, device=dev, dtype=torch.int32)
        souts = [torch.empty(B, 1, device=dev) for _ in range(NP)]
        sh.pipe_route(idsv[0])

        def fn(i):
            j, jp, jn = i % NP, (i - 1) % NP, (i + 1) % NP
            sh.pipe_step(prev=(dense[jp], souts[jp]), cur=idsv[j], nxt=(dense[jn], idsv[jn]))
            outs[i % NP] = souts[jp]
    elif args.workload == "din_forward":  # config 4's DIN.call (random history lengths as bench.py)
        Bd, T, kd = 2048 if args.batch == 4096 else args.batch, 100, 8
        B = Bd
        dcols = [[{"feat": "price"}], [{"feat": "user_id", "feat_onehot_dim": 192404, "embed_dim": kd},
                                       {"feat": "movies_seq", "feat_onehot_dim": 63001, "embed_dim": kd}]]
        dm = rs.DIN(dcols, ["movies_seq"], seed=1, device=dev)
        lens = torch.randint(1, T + 1, (NP, Bd, 1), generator=g, device=dev)
        hs = torch.randint(1, 63001, (NP, Bd, T), generator=g, device=dev)
        hs = torch.where(torch.arange(T, device=dev)[None, None, :] < lens, hs, torch.zeros_like(hs))
        dpool = [{"price": torch.rand(Bd, 1, generator=g, device=dev),
                  "user_id": torch.randint(0, 192404, (Bd, 1), generator=g, device=dev),
                  "movies_seq": hs[j], "movie_id": torch.randint(1, 63001, (Bd, 1), generator=g, device=dev)}
                 for j in range(NP)]

        def fn(i):
            outs[i % NP] = dm(dpool[i % NP], check_ids=False)
    elif args.workload == "peer_gather":  # config 5's owner row service at world 1: rs_peer_gather_a2a, B x F rows
        import torch.distributed as dist
        from recommender_system_amd.sharded import PeerExchange
        if not dist.is_initialized():
            dist.init_process_group("gloo", init_method="tcp://127.0.0.1:29533", rank=0, world_size=1)
        V = int(args.vocab)
        table = torch.randn(V, k, device=dev, generator=g)
        nw = B * F
        idsp = torch.randint(0, V, (NP, nw), generator=g, device=dev, dtype=torch.int32)
        ex = PeerExchange(nw * 64, world=1, rank=0, device=dev)

        def fn(i):
            outs[i % NP] = ex.gather_all_to_all(idsp[i % NP], nw, table).view(torch.float32)
    elif args.workload == "gather_rows":  # config 5's owner gather (rs_gather_rows, k 16) on the 1e8-row shard
        from recommender_system_amd.sharded import ShardedEmbeddingFM  # noqa: F401  (library handle only)
        from recommender_system_amd._lib import call, ptr
        V = int(1e8)
        table = torch.empty(V, k, device=dev).uniform_(-1, 1, generator=g)
        nw = B * F
        rowsp = torch.randint(0, V, (NP, nw), generator=g, device=dev, dtype=torch.int32)
        gouts = [torch.empty(nw, k, device=dev) for _ in range(NP)]
        errf = torch.zeros(1, dtype=torch.int32, device=dev)

        def fn(i):
            call("rs_gather_rows", ptr(table), V, k, ptr(rowsp[i % NP]), nw, ptr(gouts[i % NP]), ptr(errf),
                 _lib.stream())
            outs[i % NP] = gouts[i % NP]
    elif args.workload == "pnn":  # PNN's product inputs [flat_emb | inner] (rs_embed_inner_fwd_hm), 26 x 1e6
        pm = rs.PNN(cols, "inner", [256, 128, 64], 1, embed_dim=k, seed=3, device=dev)

        def fn(i):
            outs[i % NP] = pm.product_inputs((dense[i % NP], ids[i % NP]), check_ids=False)
    elif args.workload == "embed_x":  # x = [dense | EmbedLayer(ids)] (rs_embed_gather), 26 x 1e6
        dm = rs.DeepFM(cols, 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, seed=3, device=dev)

        def fn(i):
            outs[i % NP] = dm.embed_layer.gather(ids[i % NP], dense[i % NP], check_ids=False)
    elif args.workload == "din_tower":  # DIN's tower shape: PReLU 25 -> 256 -> 128 -> 64 -> 1 at B 2048
        Bt = 2048 if args.batch == 4096 else args.batch
        B = Bt
        dnn = rs.DNNLayer((256, 128, 64), 1, "prelu", seed=2, device=dev)
        dnn.build(25)
        xs = torch.randn(NP, Bt, 25, generator=g, device=dev)

        def fn(i):
            outs[i % NP] = dnn.tower(xs[i % NP])
    elif args.workload == "mlp":  # rs_mlp_fwd: DNNLayer((256, 128, 64), 1) on [B, 429] (the DeepFM tower alone)
        dnn = rs.DNNLayer((256, 128, 64), 1, "relu", seed=2, device=dev)
        dnn.build(429)
        xs = torch.randn(NP, B, 429, generator=g, device=dev)

        def fn(i):
            outs[i % NP] = dnn.tower(xs[i % NP])
    elif args.workload in ("dcn", "cross"):
        m = rs.DCN(cols, [256, 128, 64], 1, "relu", layer_num=3, embed_dim=k, seed=3, device=dev)

        def fn(i):
            if args.workload == "dcn":
                outs[i % NP] = m.forward_fused((dense[i % NP], ids[i % NP]), check_ids=False)
            else:  # the CrossNet output x_L (embed_cross)
                outs[i % NP] = m.cross_fused((dense[i % NP], ids[i % NP]), check_ids=False)
    else:
        m = rs.DeepFM(cols, 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, seed=3, device=dev)
        if args.workload == "deepfm":
            def fn(i):
                outs[i % NP] = m.forward_fused((dense[i % NP], ids[i % NP]), check_ids=False)
        else:
            def fn(i):
                outs[i % NP] = m.fm_logit((dense[i % NP], ids[i % NP]), check_ids=False)
    outs = {}  # step -> output tensor of the last call (graph memory after capture)
    opt = OPTS[args.option]
    values = [int(v) for v in args.values.split(",")]
    graphs, res = {}, {}
    for v in values:
        _lib.set_option(opt, v)
        for i in range(NP):
            fn(i)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(gr, stream=s):
                for i in range(args.chunk):
                    fn(i)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        gr.replay()
        torch.cuda.synchronize()
        res[v] = {"out": torch.cat([outs[i % NP] for i in range(max(0, args.chunk - NP), args.chunk)]).clone(), "us": []}
        graphs[v] = gr
    _lib.set_option(opt, 0)
    for r in range(args.rounds):
        for v in (values if r % 2 == 0 else values[::-1]):
            gr = graphs[v]
            gr.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                gr.replay()
            e1.record()
            torch.cuda.synchronize()
            res[v]["us"].append(e0.elapsed_time(e1) * 1e3 / (10 * args.chunk))
    base = res[values[0]]["out"]
    rms = float(base.pow(2).mean().sqrt())
    line = {"option": args.option, "workload": args.workload, "batch": B, "lib": args.lib,
            "us_per_launch_median": {v: float(np.median(res[v]["us"])) for v in values},
            "us_per_launch_all": {v: [round(x, 3) for x in res[v]["us"]] for v in values},
            "max_scaled_diff_vs_first": {v: float(((res[v]["out"] - base).abs() / base.abs().clamp_min(rms)).max())
                                         for v in values}}
    if args.save:
        torch.save(base.cpu(), args.save)
    if args.compare:
        ref = torch.load(args.compare, weights_only=True)
        cur = base.cpu()
        line["vs_saved"] = {"bit_identical": bool(torch.equal(ref, cur)),
                            "max_abs_diff": float((ref - cur).abs().max())}
    line["hist"] = args.hist if args.workload == "din" else None
    print(json.dumps(line))


if __name__ == "__main__":
    main()
