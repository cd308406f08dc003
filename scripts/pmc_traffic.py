"""Turn rocprofv3 PMC passes into per-launch HBM traffic for the dominant kernels.

    python scripts/pmc_traffic.py --fetch DIR_FETCH --write DIR_WRITE --key CFG_KEY \
        [--out profiles/pmc_traffic.json]

DIR_FETCH / DIR_WRITE are the output directories of two separate passes (FETCH_SIZE costs 3
TCC slots and WRITE_SIZE 2, so they cannot share one):

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d DIR_FETCH -o run -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d DIR_WRITE -o run -- python bench.py ...

Per MI355X_MICROARCH.md §HBM, gfx950's FETCH_SIZE reports half the bytes of a wide coalesced
streaming read, so traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes (both counters in KB),
averaged over the launches of each kernel. CFG_KEY matches bench.py's
"<method>_<dtype>_<m>x<n>x<l>_g<N>|<A@X tile description>" (bench.py prints it as
roofline.pmc_key).
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = collections.defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--tag", default="round 3")
    args = ap.parse_args()
    fetch = load(args.fetch, "FETCH_SIZE")
    write = load(args.write, "WRITE_SIZE")
    summary = {}
    for name in fetch:
        # (round 6) the fused A e form of k_ax_dma (its last template flag, EG) is a different
        # kernel from the plain dense pass the bench's key names: not an "ax" candidate
        if "k_ax_dma" in name and name.split(">(")[0].replace(" ", "").endswith(",true"):
            continue
        short = ("ax" if ("k_ax_" in name or "k_gemv_" in name) else
                 ("atr" if "k_atr_" in name else
                  ("gather" if ("k_at_gather" in name or "k_e_lists" in name or "k_at_rows" in name) else None)))
        if short is None:
            continue
        f = sum(fetch[name]) / len(fetch[name])
        w = sum(write.get(name, [0.0])) / max(1, len(write.get(name, [])))
        summary.setdefault(short, []).append({"kernel": name[:120], "launches": len(fetch[name]),
                                              "FETCH_SIZE_KB": f, "WRITE_SIZE_KB": w,
                                              "bytes_per_launch": (2 * f + w) * 1024})
    # dominant kernel = the A@x launch with the most dispatches
    entry = {}
    for k, v in summary.items():
        if k == "gather":   # split-candidate A e: the column lists and the gather, both per trial
            entry[k] = {"kernels": v, "bytes_per_launch": sum(e["bytes_per_launch"] for e in v)}
            continue
        best = max(v, key=lambda e: e["launches"])
        entry[k] = best
    out = {}
    if os.path.exists(args.out):
        out = json.load(open(args.out))
    if "ax" in entry:
        # the dense A@X kernel (bench.py's roofline kernel); the split-candidate gather is timed
        # and reported apart since round 3
        out[args.key] = {"bytes_per_launch": entry["ax"]["bytes_per_launch"],
                         "gather_bytes_per_launch": entry.get("gather", {}).get("bytes_per_launch"),
                         "detail": entry,
                         "correction": "traffic = (2*FETCH_SIZE + WRITE_SIZE) KB * 1024 (gfx950)",
                         "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, " + args.tag}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1, sort_keys=True)
    print(json.dumps(out.get(args.key), indent=1))


if __name__ == "__main__":
    main()
