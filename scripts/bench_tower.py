"""Graph-replayed timing of the fused MLP tower (rs_mlp_fwd) alone, for a few
batch sizes and tower shapes; prints achieved fp32 MFMA TFLOP/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_system_amd import DNNLayer  # noqa: E402


def time_graph(fn, n=64, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (n * reps) * 1e3  # us


def main():
    shapes = [(429, [256, 128, 64], 1), (429, [256], 1), (741, [256, 128, 64], 1)]
    for K, hidden, out in shapes:
        dnn = DNNLayer(hidden, out, "relu", seed=1)
        dnn.build(K)
        dims = [K] + hidden + [out]
        flop = 2 * sum(a * b for a, b in zip(dims[:-1], dims[1:]))
        for B in (4096, 16384, 65536):
            x = torch.rand(B, K, device="cuda")
            y = torch.empty(B, out, device="cuda")
            us = time_graph(lambda: dnn.tower(x, out=y))
            print(json.dumps({"dims": dims, "B": B, "us": round(us, 2),
                              "tflops": round(flop * B / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
