"""Local per-rank cost of the pipelined sharded step at a SIMULATED world
size (default 8) on one GPU: rs_shard_fm_pipe (combine | owner partials |
route) on buffers shaped as rank 0 of an 8-rank job would hold them after the
all-to-all (B = 4096 per rank, 26 x 1e7 table split in 8 blocks).  Graph-
replayed; prints one JSON line.  The all-to-all itself (2.1 MB per rank each
way) is what the driver's 8-GPU run adds."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_system_amd.sharded import ShardedEmbeddingFM  # noqa: E402


def main():
    world = int(os.environ.get("SIM_WORLD", "8"))
    B, F, V, k = 4096, 26, 10_000_000, 16
    dev = torch.device("cuda")
    sims = [ShardedEmbeddingFM([V] * F, k, 13, 10, device=dev, seed=1, world=world, rank=r, table_init=(r == 0))
            for r in range(world)]
    sh = sims[0]
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    ids = [torch.randint(0, V, (B, F), generator=g, device=dev, dtype=torch.int32) for _ in range(world)]
    dense = torch.rand(B, 13, device=dev)
    S, P = sh.slot_stride, sh.partial_width
    R = S + P
    # rank 0's received records: block q = what rank q routed to owner 0
    recv = torch.zeros(world * B * R, dtype=torch.int32, device=dev)
    for q in range(world):
        buf = torch.zeros(world * B * R, dtype=torch.int32, device=dev)
        sims[q].ops.field_route(sims[q], ids[q], buf, rec=R)
        recv.view(world, B * R)[q] = buf.view(world, B * R)[0]
    send = torch.zeros_like(recv)
    out = torch.empty(B, 1, device=dev)

    def step():
        sh.ops.pipe(sh, recv, send, prev=(dense, out), cur=ids[0], nxt=(dense, ids[0]))

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.cuda.graph(gr, stream=s):
        for _ in range(32):
            step()
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 640 * 1e3
    sh.ops.check()
    print(json.dumps({"sim_world": world, "owner_fields": sh.owner_field_ranges[0], "slot_stride": S,
                      "record_words": R, "pipe_kernel_us": round(us, 3),
                      "a2a_bytes_per_rank_each_way": world * B * R * 4}), flush=True)


if __name__ == "__main__":
    main()
