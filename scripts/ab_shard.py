"""A/B of config 5's local kernels on one box: the row route
(rs_shard_row_route, RS_OPT_SHARD_ROUTE 0 / 1) and the owner's row gather
(rs_gather_rows, RS_OPT_GATHER_ROWS 0..3) at config 5's shapes — 26 fields x
3,846,154 rows (1e8 rows, 6.4 GB), B 4096, world 1 (every lookup local:
106,496 rows) — plus the route of the sharded FM (rs_shard_field_route) on
the 26 x 1e7 table at the N > 1 shapes of world 8 (rank 0's records).  Each
arm is graph-replayed (options are read at capture), arms alternated over
rounds; prints one JSON line of medians (us per launch slot)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed_arms(arms, rounds=8, chunk=64):
    from recommender_system_amd import _lib
    graphs = {}
    for name, (opt, val, fn) in arms.items():
        _lib.set_option(opt, val)
        for i in range(chunk):
            fn(i)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for i in range(chunk):
                    fn(i)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graphs[name] = g
        _lib.set_option(opt, 0)
    res = {n: [] for n in graphs}
    names = list(graphs)
    for r in range(rounds):
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
            res[n].append(e0.elapsed_time(e1) * 1e3 / (10 * chunk))
    return {n: round(float(np.median(v)), 3) for n, v in res.items()}


def main():
    from recommender_system_amd import _lib
    from recommender_system_amd.sharded import ShardedEmbeddingFM
    dev = torch.device("cuda")
    B, F, k = 4096, 26, 16
    V5 = 3846154
    sh = ShardedEmbeddingFM([V5] * F, k, 13, 10, device=dev, seed=1, world=1, rank=0)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    NP = 16
    ids = torch.randint(0, V5, (NP, B, F), generator=g, device=dev, dtype=torch.int32)
    S = sh.slot_stride
    send = torch.empty(B * S, dtype=torch.int32, device=dev)
    slot_of = torch.empty(B * F, dtype=torch.int32, device=dev)
    reply = torch.empty(B * S, k, device=dev)
    rows = [torch.randint(0, sh.table_shard.shape[0], (B * S,), generator=g, device=dev, dtype=torch.int32)
            for _ in range(NP)]
    arms = {}
    for v in (0, 1):
        arms[f"row_route_opt{v}"] = (_lib.OPT_SHARD_ROUTE, v,
                                     lambda i: sh.ops.row_route(sh, ids[i % NP], send, slot_of))
    for v in (0, 1, 2, 3):
        arms[f"gather_opt{v}"] = (_lib.OPT_GATHER_ROWS, v,
                                  lambda i: sh.ops.gather_rows_into(sh.table_shard, rows[i % NP], reply))
    out = {"config5": timed_arms(arms)}
    del sh, reply
    torch.cuda.empty_cache()
    # the sharded FM's route at the world-8 shape (rank 0: 8 owners x 4 fields)
    V = int(1e7)
    s8 = ShardedEmbeddingFM([V] * F, k, 13, 10, device=dev, seed=1, world=8, rank=0, table_init=False)
    ids8 = torch.randint(0, V, (NP, B, F), generator=g, device=dev, dtype=torch.int32)
    R = s8.slot_stride + s8.partial_width
    send8 = torch.empty(8 * B * R, dtype=torch.int32, device=dev)
    arms = {f"field_route_w8_opt{v}": (_lib.OPT_SHARD_ROUTE, v,
                                       lambda i: s8.ops.field_route(s8, ids8[i % NP], send8, rec=R))
            for v in (0, 1)}
    out["fm_world8"] = timed_arms(arms)
    assert int(s8.ops.err.item()) == 0
    print(json.dumps(out))


if __name__ == "__main__":
    main()
