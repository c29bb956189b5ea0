"""Minimal reproducer: HIP graph capture of cross-stream event chains (no
librs_hip, no RCCL — torch ops only).  usage: python capture_repro.py MODE
  single : one stream (control)
  hub    : two side streams, every cross dependency through the origin
           (capture) stream: origin waits lane, lane waits origin
  chain  : two side streams, lane i%2 waits an event recorded on the OTHER
           side stream in the previous step (fresh event per step)
  chain1 : as chain, but each side stream's first op waits the origin first
Prints 'captured' and 'replay equal: True' on success."""
import sys

import torch


def main():
    mode = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    x = [torch.zeros(1024, device="cuda") for _ in range(2)]
    side = [torch.cuda.Stream() for _ in range(2)]
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    keep = []
    print(mode, "capturing", flush=True)
    with torch.cuda.stream(cs):
        with torch.cuda.graph(g, stream=cs):
            if mode != "single":
                for s in side:
                    s.wait_stream(cs)
            last = None
            for i in range(n):
                if mode == "single":
                    x[i % 2].add_(1.0)
                    continue
                st = side[i % 2]
                if mode == "hub":
                    if last is not None:
                        cs.wait_event(last)
                        st.wait_stream(cs)
                elif last is not None:
                    st.wait_event(last)
                with torch.cuda.stream(st):
                    x[i % 2].add_(1.0)
                ev = torch.cuda.Event()
                ev.record(st)
                keep.append(ev)
                last = ev
            if mode != "single":
                for s in side:
                    cs.wait_stream(s)
    print("captured", flush=True)
    torch.cuda.current_stream().wait_stream(cs)
    g.replay()
    torch.cuda.synchronize()
    want = (n + 1) // 2, n // 2
    print(mode, "replay equal:", float(x[0][0]) == want[0] and float(x[1][0]) == want[1], flush=True)


if __name__ == "__main__":
    main()
