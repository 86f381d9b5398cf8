"""Line up two IPM iteration traces (tools/trace_replay.py, host build vs device) and report, per
replayed step, the first iteration and quantity where they differ beyond a relative tolerance,
and how the difference grows (development helper).

    python tools/trace_diff.py A.log B.log [rtol=1e-13]"""
import re
import sys


def parse(path):
    """{(name, step): dict(iters=[{field: value}], tail=str)}"""
    out, cur, key = {}, None, None
    for line in open(path, errors="replace"):
        m = re.match(r"== begin (\S+) (\d+)", line)
        if m:
            key = (m.group(1), int(m.group(2)))
            cur = out[key] = dict(iters=[], tail="")
            continue
        if cur is None:
            continue
        m = re.match(r"== (\S+) (\d+) status", line)
        if m:
            cur["tail"] = line.strip()
            continue
        s = line.strip()
        if s.startswith("it "):
            toks = s.split()
            rec = {"it": int(toks[1])}
            for k, v in zip(toks[2::2], toks[3::2]):
                try:
                    rec[k] = float(v)
                except ValueError:
                    pass
            cur["iters"].append(rec)
        elif s.startswith("step ") and cur["iters"]:
            toks = s.split()
            for k, v in zip(toks[1::2], toks[2::2]):
                try:
                    cur["iters"][-1]["step_" + k] = float(v)
                except ValueError:
                    pass
        elif s.startswith("code") or s.startswith("backtrack"):
            cur["iters"][-1]["end"] = s if cur["iters"] else s
    return out


def rel(a, b):
    return abs(a - b) / max(abs(a), abs(b), 1e-300)


def main():
    A, B = parse(sys.argv[1]), parse(sys.argv[2])
    rtol = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-13
    for key in sorted(set(A) & set(B)):
        a, b = A[key], B[key]
        print(f"### {key[0]} step {key[1]}")
        print(f"  A: {a['tail']}\n  B: {b['tail']}")
        first = None
        for ia, ib in zip(a["iters"], b["iters"]):
            worst = max(((rel(ia[k], ib[k]), k) for k in ia if k in ib and isinstance(ia[k], float)
                         and k not in ("best",)), default=(0.0, ""))
            if first is None and worst[0] > rtol:
                first = (ia["it"], worst[1], worst[0])
            if first is not None:
                print(f"  it {ia['it']:3d} worst rel diff {worst[0]:.2e} ({worst[1]})  "
                      f"pres {ia.get('pres', 0):.3e}/{ib.get('pres', 0):.3e} dres {ia.get('dres', 0):.3e}/"
                      f"{ib.get('dres', 0):.3e} gap {ia.get('gap', 0):.3e}/{ib.get('gap', 0):.3e} "
                      f"alpha {ia.get('step_alpha', 0):.4f}/{ib.get('step_alpha', 0):.4f} "
                      f"{ia.get('end', '')}|{ib.get('end', '')}")
        print(f"  first divergence beyond {rtol:g}: {first}; iterations {len(a['iters'])} / {len(b['iters'])}")


if __name__ == "__main__":
    main()
