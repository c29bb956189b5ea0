"""Does the memory type of the embedding table change the random-row rate?

The round-2/3 policy sweep (scripts/diag_policy_bw.py) varied the load's cache
bits on ordinary (coarse-grained, cached) device memory: every random 64-B row
cost a 128-B line fill, ~3.3 TB/s of row bytes.  This probe allocates the same
16.6 GB table with hipExtMallocWithFlags under each device-memory flag
(0 default, 1 fine-grained, 3 uncached) and measures
  * random 64-B rows through rs_diag_policy_sum (diagnostic library; modes
    0 plain, 1 nt), and
  * the product headline kernel (rs_embed_fm_fwd_hm, B 4096 and 16384,
    graph-replayed, 64-batch id pool) on a bit-identical copy of the table,
alternating the allocations so box drift hits all of them.  Prints JSON lines.
"""
import ctypes as C
import json
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def hip_runtime():
    # the libamdhip64 torch already loaded (one HIP runtime per process)
    with open("/proc/self/maps") as f:
        for line in f:
            p = line.split()[-1]
            if "libamdhip64.so" in p:
                return C.CDLL(p)
    raise RuntimeError("libamdhip64 not loaded")


def main():
    dev = torch.device("cuda")
    torch.zeros(1, device=dev)
    hip = hip_runtime()
    hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipFree.argtypes = [C.c_void_p]
    diag = C.CDLL(os.path.join(ROOT, "recommender_system_amd", "librs_hip_diag.so"))
    diag.rs_diag_policy_sum.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
    lib = C.CDLL(os.path.join(ROOT, "recommender_system_amd", "librs_hip.so"))
    P, L, I = C.c_void_p, C.c_int64, C.c_int
    lib.rs_embed_fm_fwd_hm.argtypes = [P, I, L, P, L, I, P, P, P, P, P, I, I, P, P, I, P, P, L, P, P]
    lib.rs_fm_prepare.argtypes = [P, P, I, I, I, I, P, P]
    lib.rs_fm_prepared_size.restype = L
    lib.rs_fm_prepared_size.argtypes = [I, I, I, I]

    F, k, kfm, nd, V = 26, 16, 10, 13, 10_000_000
    nbytes = F * V * k * 4
    src = torch.empty(F * V, k, device=dev).uniform_(-0.05, 0.05)
    flags = [int(x) for x in os.environ.get("MTYPE_FLAGS", "0,1,3").split(",")]
    tabs = {}
    for fl in flags:
        p = C.c_void_p()
        rc = hip.hipExtMallocWithFlags(C.byref(p), nbytes, fl)
        if rc != 0:
            print(json.dumps({"flag": fl, "alloc_rc": rc}), flush=True)
            continue
        assert hip.hipMemcpy(p, C.c_void_p(src.data_ptr()), nbytes, 3) == 0  # device to device
        tabs[fl] = p.value
    del src
    torch.cuda.synchronize()
    st = torch.cuda.current_stream().cuda_stream
    out = torch.zeros(1 << 16, device=dev)

    def time_it(fn, reps=10):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps * 1e-3

    # ---- random-row probe
    n = 16 * 1_703_936
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    rows = torch.randint(0, F * V, (n,), generator=g, device=dev)
    pairs = (rows // 2) * 2
    pairs = torch.stack([pairs[: n // 2], pairs[: n // 2] + 1], 1).reshape(-1)
    for mode in (0, 1):
        for fl, tp in tabs.items():
            res = {"probe": "random_rows", "flag": fl, "mode": mode}
            for name, r in (("random", rows), ("line_pairs", pairs)):
                t = time_it(lambda: diag.rs_diag_policy_sum(tp, r.data_ptr(), r.numel(), 8192, out.data_ptr(), mode, st))
                res[name + "_TBps"] = round(n * 64 / t / 1e12, 3)
            print(json.dumps(res), flush=True)
    del rows, pairs

    # ---- the product headline kernel on each allocation
    d = nd + F * k
    w1 = torch.randn(d, 1, device=dev) * 0.05
    v = torch.randn(d, kfm, device=dev) * 0.05
    w0 = torch.zeros(1, device=dev)
    prep = torch.empty(lib.rs_fm_prepared_size(nd, F, k, kfm), device=dev)
    lib.rs_fm_prepare(w1.data_ptr(), v.data_ptr(), nd, F, k, kfm, prep.data_ptr(), st)
    offs = torch.arange(F, dtype=torch.int64, device=dev) * V
    voc = torch.full((F,), V, dtype=torch.int64, device=dev)
    hoff = (C.c_int64 * F)(*[c * V for c in range(F)])
    hvoc = (C.c_int64 * F)(*([V] * F))
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    NP = 64
    for B in [int(x) for x in os.environ.get("MTYPE_BATCHES", "4096,16384").split(",")]:
        pool = torch.randint(0, V, (NP, B, F), dtype=torch.int32, device=dev)
        dense = torch.rand(NP, B, nd, device=dev)
        graphs, outs = {}, {}
        for fl, tp in tabs.items():
            logit = torch.empty(NP, B, device=dev)

            def fn(i, tp=tp, logit=logit):
                j = i % NP
                lib.rs_embed_fm_fwd_hm(pool[j].data_ptr(), 0, F, dense[j].data_ptr(), nd, nd, tp,
                                       offs.data_ptr(), voc.data_ptr(), C.addressof(hoff), C.addressof(hvoc), F, k,
                                       prep.data_ptr(), w0.data_ptr(), kfm, logit[j].data_ptr(), None, B,
                                       err.data_ptr(), torch.cuda.current_stream().cuda_stream)

            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                for i in range(NP):
                    fn(i)
                torch.cuda.synchronize()
                with torch.cuda.graph(gr, stream=s):
                    for i in range(NP):
                        fn(i)
            torch.cuda.synchronize()
            graphs[fl], outs[fl] = gr, logit
        res = {fl: [] for fl in tabs}
        names = list(tabs)
        for r in range(8):
            for fl in (names if r % 2 == 0 else names[::-1]):
                res[fl].append(time_it(graphs[fl].replay, 10) * 1e6 / NP)
        ref = outs[names[0]]
        print(json.dumps({"probe": "embed_fm_hm", "batch": B,
                          **{f"median_us_flag{fl}": round(float(np.median(res[fl])), 3) for fl in names},
                          **{f"us_flag{fl}": [round(x, 3) for x in res[fl]] for fl in names},
                          "bit_identical": {fl: bool(torch.equal(outs[fl], ref)) for fl in names},
                          "err": int(err.item())}), flush=True)
    for tp in tabs.values():
        hip.hipFree(C.c_void_p(tp))


if __name__ == "__main__":
    main()
