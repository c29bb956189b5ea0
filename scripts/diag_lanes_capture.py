"""Diagnostic: which cross-stream dependency form survives HIP graph capture
for the two-lane pipelined sharded stream (sharded.PipeLanes).
usage: python scripts/diag_lanes_capture.py MODE [exchange]
  MODE reuse  : one event re-recorded every step (chain)
       fresh  : a new event per step, kept alive until capture end
       nochain: fork/join only, no cross-lane chain
       single : one stream, no lanes (control)"""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from recommender_system_amd.sharded import ShardedEmbeddingFM  # noqa: E402


def main():
    mode = sys.argv[1]
    exchange = len(sys.argv) > 2 and sys.argv[2] == "exchange"
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
    B, n, L = 260, 7, 2
    batches = [(torch.rand(B, 13, device=dev),
                torch.as_tensor(np.stack([rng.integers(0, v, B) for v in vocabs], 1), dtype=torch.int32,
                                device=dev)) for _ in range(n)]
    ref = [o.cpu().numpy() for o in sh.forward_stream(batches)]
    outs = [torch.full((B, 1), float("nan"), device=dev) for _ in range(n)]
    streams = [torch.cuda.Stream() for _ in range(L)]
    keep = []
    if mode == "single":
        L = 1
    for lane in range(L):
        with torch.cuda.stream(streams[lane]):
            sh.pipe_route(batches[lane][1], lane=lane)
    torch.cuda.synchronize()
    coll = torch.cuda.Event()
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    print(mode, "exchange" if exchange else "local", "capturing", flush=True)
    with torch.cuda.stream(cs):
        with torch.cuda.graph(g, stream=cs):
            for st in streams[:L]:
                st.wait_stream(cs)
            last = None
            for i in range(n + L):
                lane = i % L
                st = streams[lane]
                prev = (batches[i - L][0], outs[i - L]) if i >= L else None
                cur = batches[i][1] if i < n else None
                nxt = batches[i + L] if i + L < n else None
                if mode == "hub" and last is not None:
                    cs.wait_event(last)  # chain through the capture stream (star topology)
                    st.wait_stream(cs)
                with torch.cuda.stream(st):
                    if mode in ("reuse", "fresh") and last is not None:
                        st.wait_event(last)
                    sh.pipe_step(prev, cur, nxt, lane=lane)
                    if mode == "reuse":
                        coll.record(st)
                        last = coll
                    elif mode in ("fresh", "hub"):
                        ev = torch.cuda.Event()
                        ev.record(st)
                        keep.append(ev)
                        last = ev
            for st in streams[:L]:
                cs.wait_stream(st)
    print("captured", flush=True)
    torch.cuda.current_stream().wait_stream(cs)
    g.replay()
    torch.cuda.synchronize()
    ok = all(np.array_equal(o.cpu().numpy(), r) for o, r in zip(outs, ref))
    print(mode, "replay equal:", ok, flush=True)
    if exchange:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
