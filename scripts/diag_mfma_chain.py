"""Cycles per v_mfma_f32_16x16x4_f32 (s_memtime) as one, two or four
independent accumulation chains per wave, with 1, 2 and 4 waves per SIMD
(workgroups of 4 / 8 / 16 waves: wave w runs on SIMD perm(w mod 4)).
Prints one JSON line: median cycles per MFMA per wave, and per SIMD."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from recommender_system_amd import _lib
    n, grid = 512, 256
    res = {}
    for nw in (4, 8, 16):
        for ch in (1, 2, 4):
            cyc = torch.zeros(grid * nw, dtype=torch.int64, device="cuda")
            sink = torch.zeros(grid * nw * 64, device="cuda")
            for _ in range(3):
                _lib.call("rs_diag_mfma_chain", grid, 64 * nw, n, ch, cyc.data_ptr(), sink.data_ptr(),
                          torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            c = float(np.median(cyc.cpu().numpy()))
            res[f"waves_per_simd_{nw // 4}_chains_{ch}"] = {"cycles_per_mfma_per_wave": round(c / n, 2),
                                                            "cycles_per_mfma_per_simd": round(c / n / (nw // 4), 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
