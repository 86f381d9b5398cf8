#!/bin/bash
# GPU box: tools/mb_riccati (Riccati + backward sweep, 4096 headline egos, aos / soa / mfma, with and
# without prefetch): timings, then per-variant FETCH_SIZE, WRITE_SIZE and SQ counters from separate
# rocprofv3 passes.  usage: bash tools/mb_riccati.sh TAG
set -o pipefail
tag=${1:-mbr}
R=$PWD
out=$R/gpurun_out/$tag
mkdir -p $out
timeout -k 10 120 $R/tools/mb_riccati all 50 > $out/time.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for v in aos aos_pf soa soa_pf mfma mfma_pf; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/f_$v -o run --output-format csv -- $R/tools/mb_riccati $v 5 > $out/f_$v.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/w_$v -o run --output-format csv -- $R/tools/mb_riccati $v 5 > $out/w_$v.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace -d $out/s_$v -o run --output-format csv -- $R/tools/mb_riccati $v 5 > $out/s_$v.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $out/t_$v -o run --output-format csv -- $R/tools/mb_riccati $v 5 > $out/t_$v.log 2>&1 || exit $?
done
python3 - $out <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
def per_kernel(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_aos" in k or "k_soa" in k or "k_mfma<" in k:
                acc[r["Counter_Name"]][r["Dispatch_Id"]].append(float(r["Counter_Value"]))
    res = {}
    for c, disp in acc.items():
        vals = [sum(v) for _, v in sorted(disp.items(), key=lambda t: int(t[0]))][1:]   # drop the warm launch
        res[c] = sum(vals) / max(len(vals), 1)
    return res
print("variant   2F+W MB   FETCH MB  WRITE MB   L2hit   WAVE_CYC  WAIT_ANY%  VALU_inst  VMEM_RD  VMEM_WR  LDS")
for v in ("aos", "aos_pf", "soa", "soa_pf", "mfma", "mfma_pf"):
    f, w, s, t = (per_kernel(f"{out}/{p}_{v}") for p in "fwst")
    F, W = f.get("FETCH_SIZE", 0) * 1024 / 1e6, w.get("WRITE_SIZE", 0) * 1024 / 1e6
    hit = t.get("TCC_HIT_sum", 0) / max(t.get("TCC_HIT_sum", 0) + t.get("TCC_MISS_sum", 0), 1)
    wc = s.get("SQ_WAVE_CYCLES", 0)
    print(f"{v:8s} {2*F+W:9.1f} {F:9.1f} {W:9.1f} {hit:7.3f} {wc:10.3e} {100*s.get('SQ_WAIT_ANY',0)/max(wc,1):9.1f} "
          f"{s.get('SQ_INSTS_VALU',0):10.3e} {s.get('SQ_INSTS_VMEM_RD',0):8.3e} {s.get('SQ_INSTS_VMEM_WR',0):8.3e} {s.get('SQ_INSTS_LDS',0):8.3e}")
PY
find $out -name "*.csv" -delete
cat $out/time.log
