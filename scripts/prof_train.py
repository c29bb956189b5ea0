"""Kernel profile of DeepFM.train_step / DCN.train_step at the config-2
shape (B 4096, 26 x 1e6 x 16): run under rocprofv3 --kernel-trace."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import recommender_system_amd as rs  # noqa: E402
from tests.helpers import criteo_columns  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "deepfm"
    B, F, V, k = 4096, 26, 1_000_000, 16
    dev = torch.device("cuda")
    cols = criteo_columns([V] * F, embed_dim=k)
    if which == "deepfm":
        m = rs.DeepFM(cols, 10, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, seed=1)
    else:
        m = rs.DCN(cols, [256, 128, 64], 1, "relu", layer_num=3, embed_dim=k, seed=1)
    rng = np.random.default_rng(0)
    ids = torch.as_tensor(rng.integers(0, V, (B, F)).astype(np.int32), device=dev)
    dense = torch.rand(B, 13, device=dev)
    lab = (torch.rand(B, device=dev) < 0.25).float()
    for i in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.train_step((dense, ids), lab, lr=0.01, check_ids=False, dropout=False)
        torch.cuda.synchronize()
        print(f"step {i}: {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
