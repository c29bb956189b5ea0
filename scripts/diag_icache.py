"""Instruction-fetch cost (rs_diag_icache): 2048 FMAs per wave as a loop or
as straight-line code, each run twice in one launch (first pass: cold
instruction cache after the dispatch; second: warm), 256 workgroups of 1024
threads, and the launch repeated (does the code stay cached across
launches?).  Prints one JSON line: median s_memtime cycles per pass."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from recommender_system_amd import _lib
    grid, block = 256, 1024
    nw = grid * block // 64
    res = {}
    for unroll in (0, 1):
        cyc = torch.zeros(2 * nw, dtype=torch.int64, device="cuda")
        sink = torch.zeros(grid * block, device="cuda")
        runs = []
        for _ in range(3):
            _lib.call("rs_diag_icache", grid, block, unroll, cyc.data_ptr(), sink.data_ptr(),
                      torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            c = cyc.cpu().numpy().reshape(nw, 2)
            runs.append([int(np.median(c[:, 0])), int(np.median(c[:, 1])), int(c[:, 0].max())])
        res["straight_line" if unroll else "loop"] = {"first_pass_second_pass_firstmax_per_launch": runs}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
