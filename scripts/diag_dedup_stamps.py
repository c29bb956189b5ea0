"""Phase timeline of the dedup route's per-field hash kernel (diagnostic
build scripts/ab/librs_dhstamp.so, -DRS_DH_STAMPS): thread 0 of every
workgroup stamps s_memrealtime (100 MHz) at the phase ends into the
workspace's incl slab.  Config-5 shape: B 4096, 26 fields x 3,846,154 rows,
Zipf(1.2) (or uniform with DD_UNIFORM=1) ids, world DD_WORLD (default 1).
Prints one JSON line: median over workgroups of each phase's end (us from the
workgroup's start) and the kernel's HIP-event time."""
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from recommender_system_amd import _lib  # noqa: E402

_lib._LIB_PATH = Path(os.environ.get("DD_LIB", "scripts/ab/librs_dhstamp.so")).resolve()

PHASES = ["start", "loaded", "inserted", "numbered", "written"]


def main():
    lib = _lib.lib()
    B, F, V = 4096, 26, 3846154
    world = int(os.environ.get("DD_WORLD", 1))
    dev = torch.device("cuda")
    rng = np.random.default_rng(7)
    if os.environ.get("DD_UNIFORM"):
        ids_h = rng.integers(0, V, size=(B, F)).astype(np.int32)
    else:
        ids_h = np.minimum(rng.zipf(1.2, size=(B, F)) - 1, V - 1).astype(np.int32)
    ids = torch.as_tensor(ids_h, device=dev)
    offs = torch.arange(F, dtype=torch.int64, device=dev) * V
    voc = torch.full((F,), V, dtype=torch.int64, device=dev)
    rows = F * V
    rpr = (rows + world - 1) // world
    cap = ((B * F // 2 + 63) // 64) * 64
    send = torch.empty(world * cap, dtype=torch.int32, device=dev)
    slot = torch.empty(B, F, dtype=torch.int32, device=dev)
    wsz = lib.rs_shard_dedup_workspace_size(B * F, world)
    ws = torch.zeros(wsz, dtype=torch.uint8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    over = torch.zeros(1, dtype=torch.int32, device=dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run():
        s = lib.rs_shard_dedup_route(C.c_void_p(ids.data_ptr()), 0, F, C.c_void_p(offs.data_ptr()),
                                     C.c_void_p(voc.data_ptr()), F, B, rpr, world, cap, C.c_void_p(send.data_ptr()),
                                     C.c_void_p(slot.data_ptr()), C.c_void_p(ws.data_ptr()), C.c_void_p(err.data_ptr()),
                                     C.c_void_p(over.data_ptr()), st)
        assert s == 0, s

    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 50
    for _ in range(n):
        run()
    e1.record()
    torch.cuda.synchronize()
    # the incl slab: the workspace layout of shard_dedup.hip (dd_al = 256-B rounding)
    al = lambda x: (x + 255) // 256 * 256
    nb = B * F * 4
    o = 0
    offs_ws = {}
    for name in ("key_in", "key_out", "val_in", "val_out", "head", "incl"):
        offs_ws[name] = o
        o = al(o + nb)
    st_h = ws[offs_ws["incl"]:offs_ws["incl"] + F * 16 * 8].cpu().numpy().view(np.uint64).reshape(F, 16)
    t0 = st_h[:, 0].astype(np.int64)
    res = {"us_per_route_incl_scatter": e0.elapsed_time(e1) / n * 1e3, "world": world,
           "ids": "uniform" if os.environ.get("DD_UNIFORM") else "zipf1.2",
           "distinct_fraction": float(np.mean([np.unique(ids_h[:, c]).size for c in range(F)]) / B),
           "err": int(err.item()), "overflow": int(over.item())}
    for k, name in enumerate(PHASES[1:], 1):
        v = (st_h[:, k].astype(np.int64) - t0) / 100.0  # 100 MHz ticks -> us
        res[name] = float(np.median(v))
    res["slowest_workgroup_us"] = float(((st_h[:, 4].astype(np.int64) - t0) / 100.0).max())
    res["start_spread_us"] = float((t0.max() - t0.min()) / 100.0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
