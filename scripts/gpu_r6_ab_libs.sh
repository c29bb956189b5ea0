#!/bin/bash
# Alternate scripts/ab/librs_ab_cross_{0,1}.so per process over $WORKLOADS
# (ab_options.py, 3 rounds each), then print medians and bit-identity.
WORKLOADS=${WORKLOADS:-embed_fm}
OUT=${OUT:-gpurun_out/ab_libs.jsonl}
for wl in $WORKLOADS; do for r in 1 2 3; do for i in 0 1; do
  timeout -k 10 120 python scripts/ab_options.py --option cross_kernel --values 0 --workload $wl --rounds 6 \
      --lib scripts/ab/librs_ab_cross_$i.so --save /tmp/ab_${wl}_$i.pt ${AB_ARGS:-} || exit 9
done; done; done > $OUT
WORKLOADS="$WORKLOADS" OUT=$OUT python - <<EOF2
import json, os, torch
for l in open(os.environ["OUT"]): d=json.loads(l); print(d["workload"], d["lib"][-20:], d["us_per_launch_median"])
for wl in os.environ["WORKLOADS"].split():
    print(wl, "bit-identical", torch.equal(torch.load(f"/tmp/ab_{wl}_0.pt"), torch.load(f"/tmp/ab_{wl}_1.pt")))
EOF2
