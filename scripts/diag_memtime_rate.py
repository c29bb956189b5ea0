"""Rate of the s_memtime counter: one long MFMA-chain kernel per SIMD
(rs_diag_mfma_chain, 4 waves of 8192 MFMAs), its s_memtime cycles against
its HIP-event duration, at 1 and 256 workgroups.  Prints one JSON line:
counter ticks per microsecond (= the shader clock in MHz if s_memtime counts
shader cycles)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from recommender_system_amd import _lib
    res = {}
    for grid in (1, 256):
        n, nw = 65536, 4
        cyc = torch.zeros(grid * nw, dtype=torch.int64, device="cuda")
        sink = torch.zeros(grid * nw * 64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        for _ in range(2):
            _lib.call("rs_diag_mfma_chain", grid, 64 * nw, n, 4, cyc.data_ptr(), sink.data_ptr(), st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("rs_diag_mfma_chain", grid, 64 * nw, n, 4, cyc.data_ptr(), sink.data_ptr(), st)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3
        c = float(np.max(cyc.cpu().numpy()))
        res[f"grid_{grid}"] = {"kernel_us": round(us, 2), "memtime_cycles_max": int(c), "ticks_per_us": round(c / us, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
