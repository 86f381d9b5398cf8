"""HBM traffic per IPM kernel (and per phase kernel of the phase-per-kernel mode) from rocprofv3
--pmc FETCH_SIZE / WRITE_SIZE passes of tools/quick_bench.py (4 solves of 4096 egos).

usage: python tools/ph_pmc_summary.py OUTDIR MODE...   (OUTDIR/pmc_<mode>_<counter>/ from ab_phased.sh)
bytes = 2 x FETCH_SIZE + WRITE_SIZE: on gfx950 FETCH_SIZE reports half of the bytes of coalesced
8 B / 16 B per lane reads (calibrated by tools/mb_calib.hip: 1 GiB read -> 0.524 GB FETCH_SIZE at
both widths; WRITE_SIZE exact).  Writes OUTDIR/pmc_summary.json; deletes the raw CSVs.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ph_kernel_summary import name  # noqa: E402


def main(out, modes):
    res = {}
    for m in modes:
        per = defaultdict(lambda: {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0, "dispatches": 0, "ns": 0})
        nsolve = 0
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            for f in glob.glob(os.path.join(out, f"pmc_{m}_{c}", "**", "*counter_collection.csv"), recursive=True):
                seen = set()
                with open(f, newline="") as fh:
                    for r in csv.DictReader(fh):
                        if r["Counter_Name"] != c:
                            continue
                        k = name(r["Kernel_Name"])
                        per[k][c] += float(r["Counter_Value"]) * 1024.0   # kB -> bytes
                        if c == "FETCH_SIZE" and r["Dispatch_Id"] not in seen:
                            seen.add(r["Dispatch_Id"])
                            per[k]["dispatches"] += 1
                            if k == "k_tree":
                                nsolve += 1
        nsolve = max(nsolve, 1)
        rows = {}
        for k, v in per.items():
            if not (k.startswith("ph_") or k in ("k_ipm", "k_ipm_g", "k_tree")):
                continue
            byt = 2.0 * v["FETCH_SIZE"] + v["WRITE_SIZE"]
            rows[k] = {"GB_per_solve": byt / nsolve / 1e9, "read_GB_per_solve": 2.0 * v["FETCH_SIZE"] / nsolve / 1e9,
                       "write_GB_per_solve": v["WRITE_SIZE"] / nsolve / 1e9, "dispatches": v["dispatches"]}
        ipm = sum(r["GB_per_solve"] for k, r in rows.items() if k != "k_tree")
        res[m] = {"solves": nsolve, "ipm_GB_per_solve": ipm, "kernels": rows}
        print(f"mode {m}: {nsolve} solves, IPM kernels {ipm:.1f} GB per solve (2 x FETCH_SIZE + WRITE_SIZE)")
        for k in sorted(rows, key=lambda k: -rows[k]["GB_per_solve"]):
            r = rows[k]
            print("   %-10s %8.2f GB/solve  (read %7.2f, write %7.2f)  %d dispatches"
                  % (k, r["GB_per_solve"], r["read_GB_per_solve"], r["write_GB_per_solve"], r["dispatches"]))
    with open(os.path.join(out, "pmc_summary.json"), "w") as f:
        json.dump(res, f, indent=1)
    for d in glob.glob(os.path.join(out, "pmc_*")):
        if os.path.isdir(d):
            shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
