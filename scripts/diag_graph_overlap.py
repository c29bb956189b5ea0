"""Do two branches of one replayed HIP graph run concurrently when one of
them holds RCCL kernels?  World-1 RCCL group (127.0.0.1), config-5 shapes:
branch R = N RCCL all-to-all self-exchanges of the 6.8 MB row message,
branch K = N fused DeepFM launches from an exchange buffer (rs_deepfm_fwd via
ShardedDeepFM.finish), and C = N device copies of the same 6.8 MB (the
exchange without RCCL).  Times (us per item, graph-replayed):
  R, K, C alone; R || K and C || K as two long branches (one fork, one join);
  R | K and C | K forked and joined every item (the pipelined step's shape).
Prints one JSON line."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402
from recommender_system_amd.sharded import ShardedDeepFM  # noqa: E402


def graph_time(build, reps=5):
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):
        with torch.cuda.graph(g, stream=cap):
            build(cap)
    torch.cuda.current_stream().wait_stream(cap)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    N = int(os.environ.get("GO_N", 32))
    bench._world1_group()
    dev = torch.device("cuda")
    B, F, k, nd, V = 4096, 26, 16, 13, 100000
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    m = ShardedDeepFM(cols, 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, device=dev, seed=1)
    m.emb._force_exchange = True
    ids = torch.randint(0, V, (B, F), dtype=torch.int32, device=dev)
    dense = torch.rand(B, nd, device=dev)
    out = torch.empty(B, 1, device=dev)
    rb = m._rbufs(B)
    m.forward((dense, ids), check=False, out=out)  # fills rb (route, exchange)
    torch.cuda.synchronize()
    n = rb["n"]
    src = torch.randn(n * k, device=dev)
    dst = torch.empty_like(src)
    dst2 = torch.empty_like(src)

    def R(i):
        dist.all_to_all_single(dst, src)

    def C(i):
        dst2.copy_(src)

    def K(i):
        m.finish(dense, rb["got"], rb, out)

    side = torch.cuda.Stream()

    def alone(f):
        return lambda cap: [f(i) for i in range(N)]

    def long_branches(f, g):
        def build(cap):
            side.wait_stream(cap)
            for i in range(N):
                f(i)
            with torch.cuda.stream(side):
                for i in range(N):
                    g(i)
            cap.wait_stream(side)
        return build

    def per_item(f, g):
        def build(cap):
            for i in range(N):
                side.wait_stream(cap)
                with torch.cuda.stream(side):
                    g(i)
                f(i)
                cap.wait_stream(side)
        return build

    res = {"items": N}
    for name, b in (("R", alone(R)), ("K", alone(K)), ("C", alone(C)),
                    ("R||K", long_branches(R, K)), ("C||K", long_branches(C, K)),
                    ("R|K per item", per_item(R, K)), ("C|K per item", per_item(C, K))):
        res[name] = graph_time(b) / N
    print(json.dumps(res))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
