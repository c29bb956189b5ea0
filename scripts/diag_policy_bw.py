"""Random 64-B row read rate by load cache policy (diagnostic library):
mode 0 plain, 1 nt, 2 sc1, 3 sc0 sc1, 4 sc0 sc1 nt, 5 sc1 nt, 6 sc0, 7 sc0 nt.
4 loads in flight per lane, inline-asm loads.  Prints TB/s of 64-B rows for
uniformly random rows of the 16.6 GB table, both halves of random lines,
and sequential rows."""
import ctypes as C
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = C.CDLL(os.path.join(ROOT, "recommender_system_amd", "librs_hip_diag.so"))
lib.rs_diag_policy_sum.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
dev = torch.device("cuda")
total_rows = 26 * 10_000_000
table = torch.empty(total_rows, 16, device=dev).uniform_(-1, 1)
out = torch.zeros(1 << 16, device=dev)
st = torch.cuda.current_stream().cuda_stream


def bench(rows, grid, mode):
    for _ in range(3):
        lib.rs_diag_policy_sum(table.data_ptr(), rows.data_ptr(), rows.numel(), grid, out.data_ptr(), mode, st)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    s.record()
    for _ in range(reps):
        lib.rs_diag_policy_sum(table.data_ptr(), rows.data_ptr(), rows.numel(), grid, out.data_ptr(), mode, st)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


n = 16 * 1_703_936
g = torch.Generator(device=dev)
g.manual_seed(1)
rows = torch.randint(0, total_rows, (n,), generator=g, device=dev)
pairs = (rows // 2) * 2
pairs = torch.stack([pairs[: n // 2], pairs[: n // 2] + 1], 1).reshape(-1)
seq = torch.arange(n, device=dev)
for mode in range(8):
    res = {"mode": mode}
    for name, r in (("random", rows), ("line_pairs", pairs), ("seq", seq)):
        t = bench(r, 8192, mode)
        res[name + "_TBps"] = round(n * 64 / t / 1e12, 3)
    print(json.dumps(res), flush=True)
