"""Which SIMD each wave of a 1024-thread workgroup runs on (rs_diag_wave_slots:
HW_ID per wave), at the tower's occupancy (one workgroup per CU through its
LDS) and at a small one.  Prints one JSON line: per LDS size, the SIMD of
waves 0..15 in the first workgroups and how often each wave -> SIMD pattern
occurs."""
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from recommender_system_amd import _lib
    grid = 256
    res = {}
    for nw, lds in ((16, 4096), (16, 80 * 1024), (8, 4096), (8, 80 * 1024), (4, 4096)):
        out = torch.zeros(grid * nw, dtype=torch.int32, device="cuda")
        _lib.call("rs_diag_wave_slots", grid, 64 * nw, lds, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        hw = out.cpu().numpy().astype("uint32").reshape(grid, nw)
        simd = (hw >> 4) & 3
        slot = hw & 15
        pats = collections.Counter(tuple(int(x) for x in r) for r in simd)
        res[f"waves_{nw}_lds_{lds}"] = {"simd_of_wave_wg0": [int(x) for x in simd[0]], "slot_of_wave_wg0": [int(x) for x in slot[0]],
                             "patterns": {",".join(map(str, k)): v for k, v in pats.most_common(4)},
                             "waves_per_simd_wg0": [int((simd[0] == s).sum()) for s in range(4)],
                             "cu_of_wg0_1": [int((hw[0, 0] >> 8) & 15), int((hw[1, 0] >> 8) & 15)]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
