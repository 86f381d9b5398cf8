set -e
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*\|TCP_[A-Z_0-9]*\|TA_[A-Z_0-9]*\|TCC_EA0*_[A-Z_0-9]*" $O/avail.txt | sort -u > $O/names.txt || true
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES --kernel-trace -d $O/pmc1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/quick_bench.py 4096 > $O/pmc1.log 2>&1
