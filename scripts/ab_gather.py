"""A/B of the config-5 owner gather (rs_gather_rows, k = 16) on its shape:
106,496 uniform rows of a 1e8-row table (6.4 GB), graph-replayed, one JSON
line: us per launch and a checksum of the output (compare builds with
--lib).

  python scripts/ab_gather.py [--lib other/librs_hip.so]
"""
import argparse
import json
import os
import sys
from pathlib import Path

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--rounds", type=int, default=6)
    args = ap.parse_args()
    from recommender_system_amd import _lib
    if args.lib:
        _lib._LIB_PATH = Path(args.lib).resolve()
        _lib._ALLOW_MISSING = True
    from recommender_system_amd._lib import call, ptr
    dev = torch.device("cuda")
    V, k, n, NP = 100_000_000, 16, 106_496, 16
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    table = torch.empty(V, k, device=dev)
    table.normal_(generator=g)
    rows = torch.randint(0, V, (NP, n), generator=g, device=dev, dtype=torch.int32)
    out = torch.empty(NP, n, k, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)

    def fn(i):
        call("rs_gather_rows", ptr(table), V, k, ptr(rows[i % NP]), n, ptr(out[i % NP]), ptr(err), _lib.stream())

    for i in range(NP):
        fn(i)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    chunk = 64
    with torch.cuda.stream(s):
        with torch.cuda.graph(gr, stream=s):
            for i in range(chunk):
                fn(i)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    us = []
    for _ in range(args.rounds):
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        us.append(e0.elapsed_time(e1) * 1e3 / (10 * chunk))
    ref = table[rows[0].long()]
    ok = bool(torch.equal(out[0], ref)) and int(err.item()) == 0
    us.sort()
    print(json.dumps({"lib": args.lib, "us_per_launch_median": us[len(us) // 2], "us_all": [round(x, 3) for x in us],
                      "exact": ok}))


if __name__ == "__main__":
    main()
