"""Graph-replayed timing of rs_shard_slot_bucketize (one-pass slotted kernel)
under its diagnostic modes (rs_diag_shard_set_mode: bit0 blockIdx instead of
the ticket, bit1 no look-back, bit2 no finish counter — timing only, results
of modes 2/3 are wrong), beside the three-kernel exact rs_shard_bucketize."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_system_amd import _lib  # noqa: E402
from recommender_system_amd.sharded import ShardedEmbeddingFM  # noqa: E402

B, F, V, k = 4096, 26, 10_000_000, 16
world = int(os.environ.get("SH_WORLD", "8"))
lib = _lib.lib()
lib.rs_diag_shard_set_mode.argtypes = [C.c_int]
sh = ShardedEmbeddingFM([V] * F, k, 13, 10, device="cuda", seed=1, table_init=False)
sh.world, sh.rows_per_rank = world, -(-sh.total_rows // world)
bufs = sh._bufs(B)
ids = [torch.randint(0, V, (B, F), dtype=torch.int32, device="cuda") for _ in range(8)]


def graph_us(fn, n=100):
    for i in range(5):
        fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        for i in range(n):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


for mode in (0, 1, 2, 3):
    lib.rs_diag_shard_set_mode(mode)
    us = graph_us(lambda i: sh.ops.slot_bucketize(ids[i % 8], sh.offsets, sh.vocab, sh.rows_per_rank, world,
                                                  bufs["cap"], bufs))
    print(f"slot one-pass mode {mode}: {us:.2f} us/launch (world {world}, cap {bufs['cap']})")
lib.rs_diag_shard_set_mode(0)
us = graph_us(lambda i: sh.ops.bucketize(ids[i % 8], sh.offsets, sh.vocab, sh.rows_per_rank, world))
print(f"exact three-kernel bucketize: {us:.2f} us/launch")
# owner-side gather of the exchanged slot requests (world*cap rows, k = 16)
shard = torch.empty(sh.rows_per_rank, k, device="cuda")
sh.ops.slot_bucketize(ids[0], sh.offsets, sh.vocab, sh.rows_per_rank, world, bufs["cap"], bufs)
req = bufs["send"].clone()
req[req >= 0] = torch.randint(0, sh.rows_per_rank, (int((req >= 0).sum()),), dtype=torch.int32, device="cuda")
us = graph_us(lambda i: sh.ops.gather_rows_into(shard, req, bufs["reply"]))
print(f"gather_rows: {us:.2f} us/launch ({req.numel()} slots, {int((req >= 0).sum())} live)")
