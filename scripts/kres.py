"""Compact kernel resource table (VGPRs, AGPRs, spills, LDS, occupancy) of one HIP source.

    python scripts/kres.py convex-optimization_amd/csrc/kernels_atr.hip [regex]

Compiles the file for gfx950 with -Rpass-analysis=kernel-resource-usage (the library's flags)
and prints one line per kernel whose demangled name matches the regex.
"""
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
           "-ffp-contract=off", "-Iinclude", "-Iconvex-optimization_amd/csrc", "-x", "hip", "-c", src,
           "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr.splitlines()
    rows, cur = [], None
    for ln in out:
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s+(\d+)", ln)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    for r, dn in zip(rows, names):
        short = re.sub(r"\(.*", "", dn)
        if pat and not pat.search(short):
            continue
        print("%-70s vgpr %3s agpr %3s vspill %3s sspill %3s lds %6s occ %s" % (
            short[:70], r.get("VGPRs"), r.get("AGPRs"), r.get("VGPRs Spill"), r.get("SGPRs Spill"),
            r.get("LDS Size [bytes/block]"), r.get("Occupancy [waves/SIMD]")))


if __name__ == "__main__":
    main()
