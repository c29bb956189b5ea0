"""Driver for PMC passes on the fused DeepFM kernel (rs_deepfm_fwd_hm ->
deepfm_ws, RS_OPT_DEEPFM_KERNEL 0) at the Criteo shape: B 4096, 26 x 1e6 x 16,
13 dense, 429-256-128-64-1; 40 launches over a 16-batch pool.  Run under
`rocprofv3 --pmc ...` (one pass per run); the summary is taken per dispatch
of the kernel named deepfm_ws."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recommender_system_amd as rs  # noqa: E402

dev = torch.device("cuda")
B, F, nd, k, V = int(os.environ.get("DIAG_B", "4096")), 26, 13, 16, int(1e6)
cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
        [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
m = rs.DeepFM(cols, 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, seed=2, device=dev)
g = torch.Generator(device=dev)
g.manual_seed(5)
ids = torch.randint(0, V, (16, B, F), generator=g, device=dev, dtype=torch.int32)
dense = torch.rand(16, B, nd, generator=g, device=dev)
for i in range(40):
    m.forward_fused((dense[i % 16], ids[i % 16]), check_ids=False)
torch.cuda.synchronize()
print("ok")
