"""Per-phase HBM byte budget of the CVaR IPM for one ego-iteration (round-4 verdict item 1):
for each phase of the phase-per-kernel build (csrc/experimental/bmpc_ipm_ph.h, the same
arithmetic as k_ipm), the bytes of the slab arrays it reads and writes counted ONCE each
(operands and results; arrays that live only inside the phase -- the tree solve's q0 / l / kf,
tA of the residuals, the KKT scratch k_r0 -- count as zero: the ideal fused phase), next to the
measured 2 x FETCH_SIZE + WRITE_SIZE per ego-iteration of that phase's kernel (rocprofv3 passes of
tools/ab_phased.sh, pmc_summary.json).  The array lists are read off the phase bodies
(bmpc_ipm_ph.h ph_* and the functions they call); sizes from the plan (default: the headline,
highway N=20 NB=1 m=3).
    python tools/byte_budget.py [ab_phased output dir] [N NB]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "belief-planning_amd")]


def sizes(N, NB):
    import hostsim_lib as H
    from bmpc.scenarios import highway_desc
    hs = H.HostSim(highway_desc(N=N, NB=NB), 1)
    lay = hs.layout()
    T, U, bd, nv = hs.T, hs.U, hs.bdim, hs.nv
    n, d, Nc, m = 4, 2, 5, 3
    nc = bd * m + 1
    # rows from the layout's slices: nr = |z|, nlp = |dl|, neq = |y| (64-byte aligned slices, within 7)
    nr = lay["s"] - lay["z"]
    neq = lay["z"] - lay["y"]
    nlp = lay["dli"] - lay["dl"]
    ncr = 2 * nc + N * (n + d) * (nc - 1) + d   # cone rows (2 + N(n+d) per child cone, 2 + d root)
    gks = (nc - 1) * (N * (n + d + Nc) + 4) + (d + Nc + 2)   # g_k supports
    z = dict(nv=nv, nr=nr, neq=neq, nlp=nlp, ncr=ncr, nc=nc, T=T, U=U, Ad=U * n * n, Bd=U * n * d, dh=T * n,
             sd=T * Nc * 2, P=T * n * n, Kg=U * d * n, Luu=U * d * d, gk=gks)
    return z


def phases(z):
    nv, nr, neq, nlp, ncr, nc = (z[k] for k in ("nv", "nr", "neq", "nlp", "ncr", "nc"))
    node = z["Ad"] + z["Bd"]
    fac = z["sd"] + z["P"] + z["Kg"] + z["Luu"]   # the factorisation's results
    W = 2 * nlp + 2 * ncr                         # dl, dli (LP), wbar / vnt (cone rows)
    tree = fac + node + z["dh"]                   # what a tree solve reads besides its right-hand sides
    cols = nc * nv + nc * neq                     # Woodbury columns (colk, colnu)
    return {
        # residuals, exit tests, best iterate, NT scaling: x y z s h b + the factors, A / G data
        "RES": (3 * nv + 2 * neq + 4 * nr + node + z["dh"] + neq,              # x xeq (bestx src) y bvec aeq z s hvec geq
                nv + neq + nr + nv + W + nr),                                  # rx ry rz bestx, W, lam
        # node Hessians + Riccati + g_k, the pair's right-hand sides
        "FAC": (W + z["dh"] + node + nv + 2 * nr + nr,                         # W, dh, A/B, rx, lam rz, hvec
                fac + z["gk"] + 2 * nv + nr + 2 * nr + 2 * nv),               # sd P K Luu, g_k, tA tA2, rb, k_t3 k_t3b, tzc tza
        # Woodbury columns + both directions in one tree solve, coupling products
        "CPL": (z["gk"] + 2 * nv + 2 * neq + tree,                             # g_k, tzc tza, bvec ry, tree data
                cols + 2 * nv + 2 * neq),                                      # columns, x1 x2, y1 y2
        # the pair's back halves: g_k'dx, column corrections, W^-1 G dx - r3h
        "BKP": (z["gk"] + 2 * nv + 2 * neq + cols + 2 * nr + W + z["dh"],      # g_k, x1 x2, y1 y2, columns, r3h x2, W, dh
                2 * nv + 2 * neq + 2 * nr),                                    # x1 x2 y1 y2 z1 z2
        # affine step, combined right-hand side and its G'W^-1 r3h + r1
        "AFF": (2 * nv + 2 * neq + 2 * nr + neq + nr + nr + W + 2 * nr + nv + neq + z["dh"],
                nr + nr + nv + nv + neq),                                      # ds (xi), k_t3, k_nv0, tA, ya
        # the combined solve: tree solve + back half
        "CMB": (nv + neq + tree + z["gk"] + cols + nr + W,
                nv + neq + nr),
        # combined step, step length, update
        "UPD": (2 * nv + 2 * neq + 2 * nr + nr + nr + W + nv + neq + 2 * nr + neq + nr,
                nv + neq + 2 * nr),
    }


def main():
    # argument: the tools/ab_phased.sh output directory (pmc_summary.json of mode 1, vc_1.npz for the
    # batch's iteration counts), then optionally N NB
    d = sys.argv[1] if len(sys.argv) > 1 and os.path.isdir(sys.argv[1]) else None
    rest = [a for a in sys.argv[1:] if a != d]
    N, NB = (int(rest[0]), int(rest[1])) if len(rest) >= 2 else (20, 1)
    z = sizes(N, NB)
    meas = {}
    if d and os.path.exists(os.path.join(d, "pmc_summary.json")):
        import re
        j = json.load(open(os.path.join(d, "pmc_summary.json")))["1"]
        # the PMC passes run tools/quick_bench.py (4 closed-loop solves of 4096 egos): its mode-1
        # lines give the iterations per ego of each solve (ab.log)
        its, cur = [], None
        for ln in open(os.path.join(d, "ab.log")):
            m = re.match(r"== mode=(\S+) run", ln)
            if m:
                cur = m.group(1)
                continue
            m = re.search(r"iters ([\d.]+)", ln)
            if m and cur == "1":
                its.append(float(m.group(1)))
        egos, iters = 4096, sum(its) / max(len(its), 1)
        ks = {k: v["GB_per_solve"] * 1e9 / egos / iters / 1e3 for k, v in j["kernels"].items()}
        meas = {k[3:]: v for k, v in ks.items() if k.startswith("ph_")}
        print(f"measured: mode-1 phase kernels, {egos} egos, {iters:.2f} iterations per ego (mean of the quick_bench "
              f"steps); refinement kernels: " + ", ".join(f"{k} {v:.1f} KB" for k, v in meas.items() if k.startswith("RF")))
    print(f"plan N={N} NB={NB}: nv {z['nv']}, rows {z['nr']} (LP {z['nlp']}, cone {z['ncr']}), eq {z['neq']}, "
          f"T {z['T']}, U {z['U']}, cones {z['nc']}")
    print(f"{'phase':>5s} {'read KB':>9s} {'write KB':>9s} {'once KB':>9s} {'measured KB':>12s} {'ratio':>6s}")
    tot_o = tot_m = 0.0
    for ph, (r, w) in phases(z).items():
        o = 8 * (r + w) / 1e3
        mv = meas.get(ph)
        tot_o += o
        tot_m += mv or 0.0
        print(f"{ph:>5s} {8 * r / 1e3:9.1f} {8 * w / 1e3:9.1f} {o:9.1f} {mv if mv else float('nan'):12.1f} "
              f"{(mv / o) if mv else float('nan'):6.2f}")
    print(f"{'sum':>5s} {'':9s} {'':9s} {tot_o:9.1f} {tot_m if meas else float('nan'):12.1f} "
          f"{(tot_m / tot_o) if meas else float('nan'):6.2f}   (refinement rounds and the initial point not included)")


if __name__ == "__main__":
    main()
