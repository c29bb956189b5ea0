"""Same-box timing of the stable (row, lookup) sort: the hand-written variants
(scripts/build_ab_sort.sh: tile sizes) and the
hipCUB radix sort (H), graph-replayed (20 sorts per replay),
uniform and Zipf keys; outputs compared with a stable numpy argsort.  Prints one JSON line per case."""
import ctypes as C
import json
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    dev = torch.device("cuda")
    P, L, I = C.c_void_p, C.c_int64, C.c_int
    libs = {}
    for n in "ADEH":
        lib = C.CDLL(os.path.join(ROOT, "scripts", "ab", f"librs_sort_{n}.so"))
        if n == "H":
            lib.diag_hipcub_sort_bytes.restype = L
            lib.diag_hipcub_sort_bytes.argtypes = [L]
            lib.diag_hipcub_sort.argtypes = [P, P, P, P, L, I, P, L, P]
        else:
            lib.rs_sort_pairs_workspace_size.restype = L
            lib.rs_sort_pairs_workspace_size.argtypes = [L]
            lib.rs_sort_pairs_u32.argtypes = [P, P, P, P, L, I, P, P]
        libs[n] = lib
    rng = np.random.default_rng(0)
    for case, n, rows in (("uniform_B4096", 106_496, 26_000_000), ("zipf_B4096", 106_496, 26_000_000),
                          ("uniform_B65536", 1_703_936, 26_000_000)):
        if case.startswith("zipf"):
            keys = np.minimum(rng.zipf(1.05, size=n) - 1, rows - 1).astype(np.uint32)
        else:
            keys = rng.integers(0, rows, size=n).astype(np.uint32)
        bits = int(np.ceil(np.log2(rows + 1)))
        kin = torch.from_numpy(keys.view(np.int32)).to(dev)
        vin = torch.arange(n, dtype=torch.int32, device=dev)
        res, outs, graphs, keep = {}, {}, {}, []
        expect_k = keys[np.argsort(keys, kind="stable")]
        expect_v = np.argsort(keys, kind="stable").astype(np.int32)
        for name, lib in libs.items():
            kout, vout = torch.empty_like(kin), torch.empty_like(vin)
            if name == "H":
                wsb = int(lib.diag_hipcub_sort_bytes(n))
                ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
                fn = lambda lib=lib, ws=ws, wsb=wsb, kout=kout, vout=vout: lib.diag_hipcub_sort(
                    kin.data_ptr(), vin.data_ptr(), kout.data_ptr(), vout.data_ptr(), n, bits, ws.data_ptr(), wsb,
                    torch.cuda.current_stream().cuda_stream)
            else:
                ws = torch.empty(int(lib.rs_sort_pairs_workspace_size(n)), dtype=torch.uint8, device=dev)
                fn = lambda lib=lib, ws=ws, kout=kout, vout=vout: lib.rs_sort_pairs_u32(
                    kin.data_ptr(), vin.data_ptr(), kout.data_ptr(), vout.data_ptr(), n, bits, ws.data_ptr(),
                    torch.cuda.current_stream().cuda_stream)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                fn()
                torch.cuda.synchronize()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(20):
                        fn()
            torch.cuda.synchronize()
            graphs[name], outs[name], res[name] = g, (kout, vout), []
            keep.append(ws)  # the graph writes it: keep it allocated
        names = list(graphs)
        for r in range(6):
            for name in (names if r % 2 == 0 else names[::-1]):
                graphs[name].replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    graphs[name].replay()
                e1.record()
                torch.cuda.synchronize()
                res[name].append(e0.elapsed_time(e1) * 1e3 / 100)
        print(json.dumps({"case": case, "n": n, "bits": bits,
                          **{f"median_us_{k}": round(float(np.median(v)), 2) for k, v in res.items()},
                          "equal_to_stable_argsort": {
                              k: bool(np.array_equal(o[0].cpu().numpy().view(np.uint32), expect_k)
                                      and np.array_equal(o[1].cpu().numpy(), expect_v))
                              for k, o in outs.items()}}), flush=True)


if __name__ == "__main__":
    main()
