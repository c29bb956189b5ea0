"""PipeLanes parity check (run by tests/test_sharded_gloo.py::test_gpu_pipe_lanes_equal_forward).

Batches spread over 2 / 3 lanes (sharded.PipeLanes: all-to-alls on one hub
stream in batch order, launches on per-lane HIP streams) must give every batch
exactly the logit the one-lane stream gives it, eagerly and replayed from a
HIP graph (the bench's timed form).  With ``exchange`` the steps run the RCCL
self-exchange of a 1-rank nccl group (bench.py --sharded at N=1); that case
runs in its own process, which exits without tearing the group down (RCCL
shutdown after captured collectives can block)."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def check(exchange):
    from recommender_system_amd.sharded import PipeLanes, ShardedEmbeddingFM
    dev = torch.device("cuda")
    if exchange:
        s_ = socket.socket()
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
        s_.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    vocabs = [1000, 50, 3000, 7] * 6 + [11, 12]
    sh = ShardedEmbeddingFM(vocabs, 16, 13, 10, device=dev, seed=5)
    sh._force_exchange = exchange
    rng = np.random.default_rng(1)
    B, n = 260, 7
    batches = [(torch.as_tensor(rng.random((B, 13)), dtype=torch.float32, device=dev),
                torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1), dtype=torch.int32,
                                device=dev)) for _ in range(n)]
    ref = [o.cpu().numpy() for o in sh.forward_stream(batches)]
    fused = [sh.forward(d, i).cpu().numpy() for d, i in batches]
    for r, f in zip(ref, fused):
        np.testing.assert_allclose(r, f, rtol=1e-6, atol=1e-7)
    for lanes in (2, 3):
        got = sh.forward_stream(batches, lanes=lanes)
        torch.cuda.synchronize()
        for o, r in zip(got, ref):
            np.testing.assert_array_equal(o.cpu().numpy(), r)
    # graph-captured lanes: prologue routes, then every step in one graph
    L = 2
    pl = PipeLanes(sh, L)
    outs = [torch.full((B, 1), float("nan"), device=dev) for _ in range(n)]
    pl.begin()
    for lane in range(L):
        pl.route(lane, batches[lane][1])
    pl.end()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            pl.begin()
            for i in range(n + L):  # batch i on lane i % L; steps past n only combine
                prev = (batches[i - L][0], outs[i - L]) if i >= L else None
                cur = batches[i][1] if i < n else None
                nxt = batches[i + L] if i + L < n else None
                pl.step(i % L, prev, cur, nxt)
            pl.end()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    for o, r in zip(outs, ref):
        np.testing.assert_array_equal(o.cpu().numpy(), r)
    assert int(sh.ops.bad_flag().item()) == 0


if __name__ == "__main__":
    check(len(sys.argv) > 1 and sys.argv[1] == "exchange")
    print("LANES OK", flush=True)
    sys.stdout.flush()
    os._exit(0)  # no process-group teardown (see the module docstring)
