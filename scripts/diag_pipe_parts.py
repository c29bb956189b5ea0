"""What the pipelined sharded FM step's one launch (rs_shard_fm_pipe) spends
on each of its parts, at world 1 on the headline workload (26 x 1e7 x 16,
B 4096): graph-replayed launches of the full pipe (combine t-1 | owner t |
route t+1), the owner part alone, combine + route alone, and the unsharded
headline kernel for reference.  Prints one JSON line (us per launch; the
parts without an owner tile include a memset of the partial words, so only
`full` vs `owner_only` compare launch for launch)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from recommender_system_amd import _lib  # noqa: E402


def main():
    import argparse
    args = argparse.Namespace(gpus=1, steps=64, warmup=5, batch=4096, vocab=1e7, config="hotpath",
                              cpu_baseline=False, cpu_budget=0.0, extras=False, config5_pipelined=False,
                              no_config5=True, sharded=True)
    bench._dist_setup(args)
    dev = torch.device("cuda")
    B, F, k, nd, V = 4096, 26, 16, 13, int(1e7)
    ids_pool, dense_pool = bench._pool(B, [V] * F, nd, 64, dev)
    bench._world1_group()
    _, sh, _ = bench.bench_sharded_fm(args, 1, 0, [V] * F, dense_pool, lite=True)
    sb = sh._sbufs(B)
    outs = [torch.empty(B, 1, device=dev) for _ in range(2)]
    sh.pipe_route(ids_pool[0])
    sb["recv"].copy_(sb["send"])  # world 1: the records as the exchange would deliver them
    j = 0

    def full(i):
        sh.ops.pipe(sh, sb["recv"], sb["send"], prev=(dense_pool[j], outs[0]), cur=ids_pool[j],
                    nxt=(dense_pool[j], ids_pool[j]))

    def owner(i):
        sh.ops.pipe(sh, sb["recv"], sb["send"], prev=None, cur=ids_pool[j], nxt=None)

    def others(i):
        sh.ops.pipe(sh, sb["recv"], sb["send"], prev=(dense_pool[j], outs[0]), cur=None,
                    nxt=(dense_pool[j], ids_pool[j]))

    def route(i):
        sh.ops.pipe(sh, sb["recv"], sb["send"], prev=None, cur=None, nxt=(dense_pool[j], ids_pool[j]))

    def combine(i):
        sh.ops.pipe(sh, sb["recv"], sb["send"], prev=(dense_pool[j], outs[0]), cur=None, nxt=None)

    res = {}
    for name, fn in (("full", full), ("owner_only", owner), ("combine_and_route", others), ("route_only", route),
                     ("combine_only", combine), ("full_again", full)):
        _, slot = bench._timed_graph(fn, 256, 5, 1, chunk=64)
        res[name] = round(slot * 1e3, 3)
    print(json.dumps({"world": 1, "B": B, "us_per_launch": res}))


if __name__ == "__main__":
    main()
