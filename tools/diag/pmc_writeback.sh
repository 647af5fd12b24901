#!/bin/bash
# L2 write-back / eviction counters of one config-3 backward dispatch
# (tools/diag/bwd_once.py), the default build vs variant builds
# (build/<name>/libirlmx.so from tools/diag/build_variant.sh; default list:
# gran_pad0 = IRLMX_GRAN_PAR_PAD = IRLMX_GRAN_INST_PAD = 0).  Each counter set
# is its own rocprofv3 pass (at most 4 TCC counters per pass).
#   VARIANTS="default resc16" tools/diag/pmc_writeback.sh [SIZE B [OUTDIR]]
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${3:-pmc_wb}
VARIANTS=${VARIANTS:-default gran_pad0}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="${1:-128} ${2:-64}"
i=0
for v in $VARIANTS; do
  lib=""
  [ $v != default ] && lib=$ROOT/build/$v/libirlmx.so
  for set in "TCC_NORMAL_WRITEBACK_sum TCC_ALL_TC_OP_WB_WRITEBACK_sum TCC_NORMAL_EVICT_sum TCC_PROBE_EVICT_sum" \
             "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum TCC_WRITE_sum" \
             "TCC_HIT_sum TCC_MISS_sum TCC_STREAMING_REQ_sum TCC_ALL_TC_OP_INV_EVICT_sum"; do
    i=$((i+1))
    (cd /tmp && if [ -n "$lib" ]; then export IRLMX_LIB=$lib; else unset IRLMX_LIB; fi && timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT/${v}_p$i -o p -- python3 $ROOT/tools/diag/bwd_once.py $ARGS > $OUT/${v}_p$i.log 2>&1)
    rc=$?
    echo "pass $v $i rc=$rc"
    [ $rc -ne 0 ] && tail -5 $OUT/${v}_p$i.log && exit $rc
  done
done
python3 - "$OUT" $VARIANTS <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for v in sys.argv[2:]:
    vals = {}
    for path in glob.glob(f"{out}/{v}_p*/**/*counter_collection.csv", recursive=True):
        rows = [r for r in csv.DictReader(open(path)) if "cluster_kernel<1" in r["Kernel_Name"]]
        if not rows:
            continue
        last = max(int(r["Dispatch_Id"]) for r in rows)
        acc = collections.defaultdict(float)
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
        vals.update(acc)
    print(f"[{v}] " + ", ".join(f"{k} {val:.4g}" for k, val in sorted(vals.items())), flush=True)
    wb = vals.get("TCC_NORMAL_WRITEBACK_sum", 0.0)
    req, r64 = vals.get("TCC_EA0_WRREQ_sum", 0.0), vals.get("TCC_EA0_WRREQ_64B_sum", 0.0)
    print(f"[{v}] WRITE_SIZE = {((req - r64) * 32 + r64 * 64) / 1e9:.3f} GB; normal writebacks x 128 B = "
          f"{wb * 128 / 1e9:.3f} GB; TC_OP writebacks x 128 B = {vals.get('TCC_ALL_TC_OP_WB_WRITEBACK_sum', 0) * 128 / 1e9:.3f} GB",
          flush=True)
PY
