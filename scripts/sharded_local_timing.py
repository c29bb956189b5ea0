"""world=1 timing of the sharded step's local part — eager, no collectives:
the partial protocol (field route, owner FM partials, combine) and the row
exchange (slot bucketize, gather, FM from the exchange buffer); for the
step-overhead estimate of the N>1 path (which adds two RCCL all-to-alls)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_system_amd.sharded import ShardedEmbeddingFM  # noqa: E402

B, F, V, k = 4096, 26, 10_000_000, 16
sh = ShardedEmbeddingFM([V] * F, k, 13, 10, device="cuda", seed=1)
ids = [torch.randint(0, V, (B, F), dtype=torch.int32, device="cuda") for _ in range(8)]
dense = torch.rand(B, 13, device="cuda")
for i in range(20):
    sh.forward(dense, ids[i % 8], check=False)
torch.cuda.synchronize()
n = 200
t0 = time.perf_counter()
for i in range(n):
    sh.forward(dense, ids[i % 8], check=False)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / n
print(f"world=1 partial-protocol step (eager, no check): {dt * 1e6:.1f} us/step")
t0 = time.perf_counter()
for i in range(n):
    sh.forward_slots(dense, ids[i % 8], check=False)
torch.cuda.synchronize()
print(f"world=1 row-slot step (eager, no check): {(time.perf_counter() - t0) / n * 1e6:.1f} us/step")
t0 = time.perf_counter()
for i in range(50):
    sh.forward(dense, ids[i % 8], check=True)
torch.cuda.synchronize()
print(f"with per-step check (1 sync): {(time.perf_counter() - t0) / 50 * 1e6:.1f} us/step")
