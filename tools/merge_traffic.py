"""Merge gpurun_out/prof_*/pmc_entry.json files into profiles/pmc_traffic.json (the table
bench.py reads roofline.traffic from; one entry per workload key and source hash)."""
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(REPO, "profiles", "pmc_traffic.json")
entries = json.load(open(dst)) if os.path.exists(dst) else []
for f in sys.argv[1:] or glob.glob(os.path.join(REPO, "gpurun_out", "prof_*", "pmc_entry.json")):
    e = json.load(open(f))
    entries = [x for x in entries if not (x["key"] == e["key"] and x["source_hash"] == e["source_hash"])] + [e]
json.dump(entries, open(dst, "w"), indent=1)
print(f"{len(entries)} entries -> {dst}")
