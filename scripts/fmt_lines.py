"""Print a compact summary of bench JSON lines (file argument or stdin)."""
import json
import sys

src = open(sys.argv[1]) if len(sys.argv) > 1 else sys.stdin
for line in src:
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    r = d.get("roofline") or {}
    extra = {k: v for k, v in d.items() if isinstance(v, dict) and k not in ("config", "roofline", "cpu_baseline")}
    print(d["metric"][:48], f"{d['value'] / 1e6:.1f} M/s", f"{d['ms_per_step'] * 1e3:.2f} us/step",
          f"kern {1e3 * (r.get('kernel_ms') or r.get('kernel_ms_avg') or 0):.2f} us", f"frac {r.get('frac') or 0:.3f}",
          json.dumps(extra)[:600])
