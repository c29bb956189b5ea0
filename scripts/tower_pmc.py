"""Driver for PMC passes on the fused MLP tower: 20 launches of one shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommender_system_amd import DNNLayer  # noqa: E402

B = int(os.environ.get("TOWER_B", "65536"))
dims = [int(v) for v in os.environ.get("TOWER_DIMS", "429,256,1").split(",")]
dnn = DNNLayer(dims[1:-1], dims[-1], "relu", seed=1)
dnn.build(dims[0])
x = torch.rand(B, dims[0], device="cuda")
y = torch.empty(B, dims[-1], device="cuda")
for _ in range(20):
    dnn.tower(x, out=y)
torch.cuda.synchronize()
print("ok")
