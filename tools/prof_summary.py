"""Condense rocprofv3 output directories (kernel stats + PMC passes) into small files.

usage: python tools/prof_summary.py OUTDIR   (OUTDIR from tools/gpu_prof.sh)
Writes OUTDIR/summary.json and copies every *_stats.csv next to it; deletes raw traces.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def short(name):
    for k in ("k_ipm", "k_tree", "k_loop", "k_gather", "k_scatter", "k_reset", "k_model"):
        if k in name:
            return k
    return name[:60]


def main(out):
    summ = {}
    for st in glob.glob(os.path.join(out, "stats", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(st, os.path.join(out, "kernel_stats.csv"))
        summ["kernel_stats"] = [{k: r[k] for k in r} for r in rows(st)]
    for kt in glob.glob(os.path.join(out, "stats", "**", "*kernel_trace.csv"), recursive=True):
        dur = defaultdict(list)
        for r in sorted(rows(kt), key=lambda r: int(r["Start_Timestamp"])):
            dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        # launches in submission order: the first solve of a run is the cold one (inittree), so
        # the warm figures drop it; bench.py's HIP-event kernel_ms covers the timed steps only
        summ["kernel_durations_ns"] = {k: {"count": len(v), "avg": sum(v) / len(v), "min": min(v), "max": max(v),
                                           "median": sorted(v)[len(v) // 2],
                                           "warm_avg": sum(v[1:]) / max(len(v) - 1, 1),
                                           "warm_median": sorted(v[1:])[(len(v) - 1) // 2] if len(v) > 1 else v[0],
                                           "last20_avg": sum(v[-20:]) / len(v[-20:])}
                                       for k, v in dur.items() if k.startswith("k_")}
    pmc = defaultdict(lambda: defaultdict(list))
    for cc in glob.glob(os.path.join(out, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in rows(cc):
            k = short(r["Kernel_Name"])
            if not k.startswith("k_"):
                continue
            pmc[k][r["Counter_Name"]].append((r.get("Dispatch_Id"), float(r["Counter_Value"])))
    agg = {}
    for k, cs in pmc.items():
        agg[k] = {}
        for c, vals in cs.items():
            per = defaultdict(float)
            for d, v in vals:
                per[d] += v
            vs = list(per.values())
            agg[k][c] = {"dispatches": len(vs), "avg_per_dispatch": sum(vs) / len(vs)}
    summ["pmc"] = agg
    # the fused closed loop (bench.py --loop fused): one k_loop dispatch per region; the last
    # dispatch is the timed one, LOOP_STEPS steps long -- per-step figures from it
    loop_steps = int(os.environ.get("LOOP_STEPS", "20"))
    if "k_loop" in pmc:
        for c, vals in pmc["k_loop"].items():
            per = defaultdict(float)
            for d, v in vals:
                per[int(d)] += v
            last = per[max(per)]
            agg["k_loop"][c]["timed_dispatch_per_step"] = last / loop_steps
        kd = summ.get("kernel_durations_ns", {}).get("k_loop")
        if kd:
            kd["timed_dispatch_per_step"] = kd["max"] / loop_steps
    with open(os.path.join(out, "summary.json"), "w") as f:
        json.dump(summ, f, indent=1)
    # per-launch HBM bytes of the IPM kernel (the figure bench.py reports as roofline.traffic)
    for k in ("k_ipm", "k_qp", "k_loop"):
        a = agg.get(k, {})
        if "FETCH_SIZE" in a and "WRITE_SIZE" in a:
            sel = "timed_dispatch_per_step" if k == "k_loop" else "avg_per_dispatch"   # k_loop: per step
            fk = a["FETCH_SIZE"][sel]
            wk = a["WRITE_SIZE"][sel]
            byt = (2.0 * fk + wk) * 1024.0
            dur = summ.get("kernel_durations_ns", {}).get(k, {}).get("timed_dispatch_per_step" if k == "k_loop" else "avg")
            tj = {"kernel": k, "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes (" + os.path.basename(out) + ")",
                  "FETCH_SIZE_kB_per_dispatch": fk, "WRITE_SIZE_kB_per_dispatch": wk,
                  "correction": "gfx950: FETCH_SIZE counts half of the bytes of wide streaming reads "
                                "(MI355X_MICROARCH.md, HBM section); doubled here. Our loads are mostly 8 B/lane "
                                "(uncalibrated width), so the read figure is an upper estimate.",
                  f"{k}_bytes_per_launch": byt, "avg_dispatch_ns": dur,
                  "hbm_GBps": byt / dur if dur else None}
            with open(os.path.join(out, f"{k}_pmc_traffic.json"), "w") as f:
                json.dump(tj, f, indent=1)
            if KEY:   # entry for profiles/pmc_traffic.json (bench.py looks it up by key + source hash)
                sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                "belief-planning_amd"))
                from bmpc import _lib
                ent = {"key": KEY, "source_hash": _lib.source_hash(), "kernel": k, "bytes_per_launch": byt,
                       "fetch_kB": fk, "write_kB": wk, "avg_dispatch_ns": dur,
                       "profile": os.path.basename(out) + " (rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE; "
                                  "bytes = 2 x FETCH_SIZE + WRITE_SIZE)"}
                with open(os.path.join(out, "pmc_entry.json"), "w") as f:
                    json.dump(ent, f, indent=1)
    for d in ("stats", "fetch", "write", "sq", "tcc"):
        shutil.rmtree(os.path.join(out, d), ignore_errors=True)
    print(json.dumps(summ.get("kernel_durations_ns", {}), indent=1))
    print(json.dumps(agg, indent=1))


KEY = sys.argv[2] if len(sys.argv) > 2 else None

if __name__ == "__main__":
    main(sys.argv[1])
