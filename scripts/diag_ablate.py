"""Ablation of the headline kernel at B=4096 (diagnostic library): graph-replayed
per-launch time with parts removed (RS_ABLATE bits: 1 no MFMA, 2 no B-fragment
loads, 4 no cross-wave combine) plus the pure random-gather probe of the same
106,496 rows (2 dependent round trips, nothing else)."""
import ctypes as C
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_one(ablate):
    lib = C.CDLL(os.path.join(ROOT, "recommender_system_amd", "librs_hip_diag.so"))
    P, L, I = C.c_void_p, C.c_int64, C.c_int
    lib.rs_diag_embed_fm_fwd.argtypes = [P, I, L, P, L, I, P, P, P, I, I, P, P, I, P, L, P, P]
    lib.rs_fm_prepare.argtypes = [P, P, I, I, I, I, P, P]
    lib.rs_fm_prepared_size.restype = L
    lib.rs_diag_gather_sum.argtypes = [P, P, L, I, P, I, P]
    dev = torch.device("cuda")
    F, k, kfm, nd, V, B = 26, 16, 10, 13, 10_000_000, 4096
    table = torch.empty(F * V, k, device=dev).uniform_(-0.05, 0.05)
    d = nd + F * k
    w1 = torch.randn(d, 1, device=dev) * 0.05
    v = torch.randn(d, kfm, device=dev) * 0.05
    w0 = torch.zeros(1, device=dev)
    prep = torch.empty(lib.rs_fm_prepared_size(nd, F, k, kfm), device=dev)
    lib.rs_fm_prepare(w1.data_ptr(), v.data_ptr(), nd, F, k, kfm, prep.data_ptr(), torch.cuda.current_stream().cuda_stream)
    offs = torch.arange(F, dtype=torch.int64, device=dev) * V
    voc = torch.full((F,), V, dtype=torch.int64, device=dev)
    pool = [torch.randint(0, V, (B, F), dtype=torch.int32, device=dev) for _ in range(64)]
    rows = [(offs[None, :] + p.long()).reshape(-1).contiguous() for p in pool]
    dense = torch.rand(B, nd, device=dev)
    logit = torch.empty(B, device=dev)
    out = torch.zeros(8192, device=dev)

    def fm(i):
        ids = pool[i % 64]
        lib.rs_diag_embed_fm_fwd(ids.data_ptr(), 0, F, dense.data_ptr(), nd, nd, table.data_ptr(), offs.data_ptr(),
                                 voc.data_ptr(), F, k, prep.data_ptr(), w0.data_ptr(), kfm, logit.data_ptr(), B,
                                 None, torch.cuda.current_stream().cuda_stream)

    def probe(i):
        r = rows[i % 64]
        lib.rs_diag_gather_sum(table.data_ptr(), r.data_ptr(), r.numel(), 1024, out.data_ptr(), 1,
                               torch.cuda.current_stream().cuda_stream)

    def probe_mfma_layout(i):
        r = rows[i % 64]
        lib.rs_diag_gather_sum(table.data_ptr(), r.data_ptr(), r.numel(), 1024, out.data_ptr(), 5,
                               torch.cuda.current_stream().cuda_stream)

    res = {}
    for name, fn in (("embed_fm", fm), ("probe_gather", probe), ("probe_mfma_layout", probe_mfma_layout)):
        for i in range(8):
            fn(i)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for i in range(64):
                    fn(i)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name + "_us"] = round(e0.elapsed_time(e1) / 640 * 1e3, 3)
    print(json.dumps({"ablate": ablate, **res}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run_one(int(sys.argv[1]))
    else:
        runs = [(a, None) for a in (0, 4, 7)]
        for ab, nw in runs:
            env = dict(os.environ, RS_ABLATE=str(ab))
            if nw:
                env["RS_FM_NW"] = nw
            print("RS_FM_NW", nw or 16, end=" ")
            r = subprocess.run([sys.executable, __file__, str(ab)], env=env, capture_output=True, text=True, timeout=120)
            print(r.stdout.strip() or r.stderr[-500:], flush=True)
            if r.returncode != 0:
                sys.exit(r.returncode)
