"""Instruction mix per device function of an hipcc -S listing (development helper).
usage: python tools/isa_mix.py listing.s [substring ...]"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().splitlines()
want = sys.argv[2:]
funcs, cur = {}, None
for ln in src:
    m = re.match(r"^(_Z\S+):\s*(;.*)?$", ln)
    if m:
        cur = m.group(1)
        funcs[cur] = Counter()
        continue
    if cur is None:
        continue
    t = ln.strip()
    if not t or t.startswith((".", ";")):
        continue
    op = t.split()[0]
    c = funcs[cur]
    c["total"] += 1
    if op.startswith("v_"):
        c["valu"] += 1
        if "f64" in op:
            c["f64"] += 1
        if op.startswith("v_rcp_iflag") or op.startswith("v_cvt_f32_u32"):
            c["intdiv"] += 1
        if "_dpp" in t or "dpp" in op:
            c["dpp"] += 1
    elif op.startswith("s_"):
        c["salu"] += 1
        if op == "s_waitcnt":
            c["waitcnt"] += 1
    if op.startswith("global_load"):
        c["gload"] += 1
    if op.startswith("global_store"):
        c["gstore"] += 1
    if op.startswith("scratch_"):
        c["scratch"] += 1
    if op.startswith("ds_"):
        c["lds"] += 1
for name, c in funcs.items():
    if want and not any(w in name for w in want):
        continue
    print(f"{name[:70]:70s} " + " ".join(f"{k}={c[k]}" for k in
          ("total", "valu", "f64", "intdiv", "dpp", "salu", "waitcnt", "gload", "gstore", "scratch", "lds")))
