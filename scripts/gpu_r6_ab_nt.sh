for wl in pnn gather_rows embed_x; do for r in 1 2 3; do for i in 0 1; do
  timeout -k 10 120 python scripts/ab_options.py --option cross_kernel --values 0 --workload $wl --rounds 6 --lib scripts/ab/librs_ab_cross_$i.so --save /tmp/ab_${wl}_$i.pt || exit 9
done; done; done > gpurun_out/ab_nt_out.jsonl
python - <<EOF2
import json, torch
for l in open("gpurun_out/ab_nt_out.jsonl"): d=json.loads(l); print(d["workload"], d["lib"][-20:], d["us_per_launch_median"])
for wl in ["pnn", "gather_rows", "embed_x"]:
    print(wl, "bit-identical", torch.equal(torch.load(f"/tmp/ab_{wl}_0.pt"), torch.load(f"/tmp/ab_{wl}_1.pt")))
EOF2
