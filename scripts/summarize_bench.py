"""One-screen summary of a bench.py N = 1 line (the nested legs' headline numbers)."""
import json
import sys


def main():
    d = json.load(open(sys.argv[1]))
    r = d["roofline"]
    print(f"headline {d['value'] / 1e6:.1f} M/s  ms_per_step {d['ms_per_step'] * 1e3:.2f} us  kernel {r['kernel_ms'] * 1e3:.2f} us"
          f"  frac {r['frac']:.3f}")
    g = lambda k, f: (f(d[k]) if k in d and d[k] else None)
    print("deepfm_forward us", g("deepfm_forward", lambda x: round(x["ms_per_step"] * 1e3, 2)))
    print("config5_n1 us", g("config5_n1", lambda x: round(x["ms_per_step"] * 1e3, 2)),
          "kernel", g("config5_n1", lambda x: round(x["roofline"]["kernel_ms"] * 1e3, 2)),
          "frac", g("config5_n1", lambda x: round(x["roofline"]["frac"], 3)))
    print("sharded_n1 us", g("fm_hotpath_sharded_n1", lambda x: round(x["ms_per_step"] * 1e3, 2)))
    print("streamed S8/S32 us", g("streamed", lambda x: (round(x["S8"]["us_per_batch"], 2), round(x["S32"]["us_per_batch"], 2))))
    print("config3 kernel us", g("config3_n1", lambda x: round(x["ms_per_step"] * 1e3, 2)),
          "dcn_forward", g("config3_n1", lambda x: round(x["dcn_forward"]["ms_per_step"] * 1e3, 2)))
    print("config4 kernel us", g("config4_n1", lambda x: round(x["ms_per_step"] * 1e3, 2)),
          "din_forward", g("config4_n1", lambda x: round(x["din_forward"]["ms_per_step"] * 1e3, 2)))


if __name__ == "__main__":
    main()
