"""profiles/pmc_traffic.json -> profiles/r1_pmc_summary.csv: PMC HBM bytes per launch vs the
algorithmic bytes of each kernel (A streamed once + the X/R/G operands).

    python scripts/pmc_summary.py [--json profiles/pmc_traffic.json] [--out profiles/r1_pmc_summary.csv]
"""
import argparse
import csv
import json
import re


def algorithmic(kind, key, nsrc):
    m = re.search(r"_(f64|f32)_(\d+)x(\d+)x(\d+)_g", key)
    s = 8 if m.group(1) == "f64" else 4
    M, N, L = int(m.group(2)), int(m.group(3)), int(m.group(4))
    if kind == "ax":
        return s * (M * N + (M + N) * L * nsrc)
    return s * (M * N + (M + N) * L)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="profiles/pmc_traffic.json")
    ap.add_argument("--out", default="profiles/r1_pmc_summary.csv")
    a = ap.parse_args()
    d = json.load(open(a.json))
    with open(a.out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["config", "kernel", "launches", "FETCH_SIZE_KB", "WRITE_SIZE_KB",
                     "hbm_bytes_per_launch(2*FETCH+WRITE)", "algorithmic_bytes", "ratio"])
        for key, v in d.items():
            if not isinstance(v, dict) or "detail" not in v:
                continue
            for kind, e in v["detail"].items():
                nsrc = 1 if "SGD" in key else 2   # batched A@X: 2 RHS (SGD: l = 1, operands negligible)
                alg = algorithmic(kind, key, nsrc)
                w.writerow([key, "%s: %s" % (kind, e["kernel"][:80]), e["launches"],
                            round(e["FETCH_SIZE_KB"]), round(e["WRITE_SIZE_KB"]),
                            round(e["bytes_per_launch"]), alg, round(e["bytes_per_launch"] / alg, 3)])


if __name__ == "__main__":
    main()
