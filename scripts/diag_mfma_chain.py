"""Cycles per v_mfma_f32_16x16x4_f32 (s_memtime, shader cycles) as one, two or
four independent accumulation chains per wave, with 1, 2 and 4 waves per SIMD
(workgroups of 4 / 8 / 16 waves, 256 workgroups).

Each wave records its start / end stamp and its HW_ID; the waves are grouped
by (workgroup, SIMD) and a SIMD's cycles per MFMA = (last end - first start)
over its waves / (MFMAs issued on that SIMD) — the issue rate of the SIMD's
matrix pipe, which cannot beat the 32-cycle issue of this instruction
(MI355X_MICROARCH.md).  Round 4's script divided ONE wave's window by the
waves per SIMD, which assumes perfectly overlapped waves and read 22 cycles
(VERDICT r4, weak 8).  Also printed: one wave's own cycles per MFMA.
Prints one JSON line (medians over the SIMDs / waves)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from recommender_system_amd import _lib
    n, grid = 512, 256
    res = {"n_mfma_per_wave": n, "grid": grid}
    for nw in (4, 8, 16):
        for ch in (1, 2, 4):
            cyc = torch.zeros(grid * nw * 3, dtype=torch.int64, device="cuda")
            sink = torch.zeros(grid * nw * 64, device="cuda")
            for _ in range(3):
                _lib.call("rs_diag_mfma_chain", grid, 64 * nw, n, ch, cyc.data_ptr(), sink.data_ptr(),
                          torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            c = cyc.cpu().numpy().reshape(grid, nw, 3)
            t0, t1, simd = c[:, :, 0], c[:, :, 1], (c[:, :, 2] >> 4) & 3
            per_simd, per_wave = [], ((t1 - t0) / n).reshape(-1)
            for g in range(grid):
                for sd in range(4):
                    sel = simd[g] == sd
                    k = int(sel.sum())
                    if k:
                        per_simd.append((t1[g][sel].max() - t0[g][sel].min()) / (n * k))
            res[f"waves_per_simd_{nw // 4}_chains_{ch}"] = {
                "cycles_per_mfma_per_simd_window": round(float(np.median(per_simd)), 2),
                "cycles_per_mfma_per_simd_window_min": round(float(np.min(per_simd)), 2),
                "cycles_per_mfma_one_wave": round(float(np.median(per_wave)), 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
