"""Kernel profile of DIN.train_step at the config-4 shape (B 2048, T 100,
k 8, behaviour vocab 63,001): run under rocprofv3 --kernel-trace --stats."""
import sys
import time

import torch

sys.path.insert(0, ".")
import recommender_system_amd as rs  # noqa: E402


def main():
    B, T, k = 2048, 100, 8
    dev = torch.device("cuda")
    cols = [[{"feat": "age"}],
            [{"feat": "user_id", "feat_onehot_dim": 192404, "embed_dim": k},
             {"feat": "movies_seq", "feat_onehot_dim": 63001, "embed_dim": k}]]
    model = rs.DIN(cols, ["movies_seq"], seed=1, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    lens = torch.randint(1, T + 1, (B,), generator=g, device=dev)
    hist = torch.randint(1, 63001, (B, T), generator=g, device=dev)
    hist = torch.where(torch.arange(T, device=dev)[None, :] < lens[:, None], hist, torch.zeros_like(hist))
    inp = {"age": torch.rand(B, 1, generator=g, device=dev),
           "user_id": torch.randint(0, 192404, (B, 1), generator=g, device=dev),
           "movie_id": torch.randint(1, 63001, (B, 1), generator=g, device=dev), "movies_seq": hist}
    labels = (torch.rand(B, generator=g, device=dev) < 0.25).to(torch.float32)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    for i in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model.train_step(inp, labels, lr=0.01, check_ids=False)
        torch.cuda.synchronize()
        print(f"step {i}: {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
