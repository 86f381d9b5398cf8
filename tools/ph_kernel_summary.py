"""Per-phase kernel times of the phase-per-kernel IPM from a rocprofv3 --kernel-trace run.

usage: python tools/ph_kernel_summary.py OUTDIR   (OUTDIR: rocprofv3 -d directory)
Prints, per phase kernel (k_ph<Model, PH>), launches, total and mean duration; per solve (the
launches between two k_tree launches) the summed time of all phase kernels; keeps the
*_kernel_stats.csv (copied to OUTDIR/kernel_stats.csv), deletes the raw trace.
"""
import csv
import glob
import os
import re
import shutil
import sys
from collections import defaultdict

PH = ["INIT1", "INIT2", "INIT3", "RES", "FAC", "CPL", "BKP", "RFP0", "RFP1", "AFF", "CMB", "RFC0", "RFC1", "UPD",
      "FIN"]


def name(k):
    m = re.search(r"k_ph<[^,]*,\s*(\d+)>", k)
    if m:
        return "ph_" + PH[int(m.group(1))]
    for s in ("k_ipm", "k_tree", "k_qp", "k_env"):
        if s in k:
            return s
    return k[:40]


def main(out):
    for st in glob.glob(os.path.join(out, "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(st, os.path.join(out, "kernel_stats.csv"))
    rows = []
    for kt in glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True):
        with open(kt, newline="") as f:
            rows += list(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    per = defaultdict(list)
    solves, cur = [], None
    for r in rows:
        n = name(r["Kernel_Name"])
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per[n].append(d)
        if n == "k_tree":
            cur = {"start": int(r["Start_Timestamp"]), "ipm_busy": 0, "end": int(r["End_Timestamp"])}
            solves.append(cur)
        elif cur is not None and (n.startswith("ph_") or n == "k_ipm"):
            cur["ipm_busy"] += d
            cur["end"] = int(r["End_Timestamp"])
    print("%-10s %8s %12s %10s" % ("kernel", "launches", "total ms", "mean us"))
    tot = 0
    for n in sorted(per, key=lambda k: -sum(per[k])):
        v = per[n]
        tot += sum(v)
        print("%-10s %8d %12.3f %10.2f" % (n, len(v), sum(v) / 1e6, sum(v) / len(v) / 1e3))
    print("all kernels %.3f ms" % (tot / 1e6))
    for i, s in enumerate(solves):
        print("solve %d: IPM kernels busy %.3f ms, tree start -> last IPM kernel end %.3f ms"
              % (i, s["ipm_busy"] / 1e6, (s["end"] - s["start"]) / 1e6))
    for d in glob.glob(os.path.join(out, "*")):
        if os.path.isdir(d):
            shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main(sys.argv[1])
