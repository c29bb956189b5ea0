"""Profile target: the config-5 Zipf(1.2) step at world 1 with the exchange
forced, field-range records vs the deduplicated route, eager and replayed from
a HIP graph.  Run under rocprofv3 --kernel-trace --stats for the per-kernel
split of the dedup route (dedup_field_sort / dedup_field_meta / scatter).
Prints one JSON line of wall-clock ms per step."""
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402
from recommender_system_amd import _lib  # noqa: E402
from recommender_system_amd.sharded import ShardedDeepFM  # noqa: E402

if os.environ.get("PD_LIB"):  # A/B: another build of the library (scripts/ab)
    from pathlib import Path
    _lib._LIB_PATH = Path(os.environ["PD_LIB"]).resolve()


def main():
    B, F, k, nd = 4096, 26, 16, 13
    V = int(os.environ.get("PD_VOCAB", 3846154))
    steps = int(os.environ.get("PD_STEPS", 50))
    bench._world1_group()
    dev = torch.device("cuda")
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    rng = np.random.default_rng(17)
    npool = 8
    zipf = torch.as_tensor(np.minimum(rng.zipf(1.2, size=(npool, B, F)) - 1, V - 1).astype(np.int32), device=dev)
    dense = torch.rand(npool, B, nd, device=dev)
    out = torch.empty(B, 1, device=dev)
    res = {}
    base = None
    for name, dd in (("records", None), ("dedup", 0.5)):
        m = ShardedDeepFM(cols, 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, device=dev, seed=1,
                          dedup=dd, table_init=base is None)
        m.emb._force_exchange = True
        if base is None:
            base = m.emb.table_shard
        else:
            m.emb.table_shard = base

        def st(i, m=m):
            j = i % npool
            m.forward((dense[j], zipf[j]), check=False, out=out)

        for i in range(5):
            st(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            st(i)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / steps * 1e3
        ok, why = bench._graph_capturable(st, 0)
        graph = None
        if ok:
            dt, _ = bench._timed_graph(st, steps, 2, 1, chunk=16)
            graph = dt / steps * 1e3
        res[name] = {"eager_ms": eager, "graph_ms": graph, "graph_note": why}
    print(json.dumps(res))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
