"""Concurrent-stream diagnostic: independent headline batches
spread over 1 / 2 / 4 parallel branches of ONE hipGraph, for the two entry
points of the headline kernel — rs_embed_fm_fwd_hm (field metadata as 512 B
of kernel arguments) and rs_embed_fm_fwd (metadata in device memory) —
alternated over rounds on one box.  Prints one JSON line of medians (us per
batch) plus the empty-kernel slot and the device state."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import recommender_system_amd as rs  # noqa: E402
from recommender_system_amd import _lib  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda")
    B, F, V, k, kfm, nd = 4096, 26, int(float(os.environ.get("DIAG_V", "1e7"))), 16, 10, 13
    cols = [[{"feat": f"I{i + 1}"} for i in range(nd)],
            [{"feat": f"C{i + 1}", "feat_onehot_dim": V, "embed_dim": k} for i in range(F)]]
    model = rs.DeepFM(cols, kfm, 1e-4, 1e-4, [256, 128, 64], 1, "relu", embed_dim=k, seed=1, device=dev)
    e = model.embed_layer
    prep = model.fm.prepared(nd, F, k)
    ids_pool, dense_pool = bench._pool(B, [V] * F, nd, 64, dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    lib = _lib.lib()
    hoff, hvoc = e.host_meta()
    outs = [torch.empty(B, 1, device=dev) for _ in range(4)]

    def make(entry, ns):
        def step(i):
            j = i % 64
            args0 = (ids_pool[j].data_ptr(), 0, F, dense_pool[j].data_ptr(), nd, nd, e.table.data_ptr(),
                     e.field_offsets.data_ptr(), e.field_vocab.data_ptr())
            tail = (F, k, prep.data_ptr(), model.fm.w0.data_ptr(), kfm, outs[i % ns].data_ptr(), None, B,
                    err.data_ptr(), _lib.stream())
            if entry == "hm":
                st = lib.rs_embed_fm_fwd_hm(*args0, hoff, hvoc, *tail)
            else:
                st = lib.rs_embed_fm_fwd(*args0, *tail)
            _lib.check(st, entry)
        return step

    res = {}
    for r in range(5):
        for entry in (("hm", "dev") if r % 2 == 0 else ("dev", "hm")):
            for ns in (1, 2, 4):
                n = 256
                t = bench._timed_graph_streams(make(entry, ns), n, ns, 1)
                res.setdefault(f"{entry}_{ns}", []).append(t / n * 1e6)
    out = {key: round(float(np.median(v)), 3) for key, v in res.items()}
    out["all"] = {key: [round(x, 3) for x in v] for key, v in res.items()}
    out["empty_kernel_slot_us"] = bench._empty_kernel_slot(1)
    out["device_state"] = bench._device_state()
    assert int(err.item()) == 0
    print(json.dumps(out))


if __name__ == "__main__":
    main()
