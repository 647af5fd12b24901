#!/bin/bash
# Halo granule layout variants (cluster.h IRLMX_GRAN_*_PAD): backward wall time
# (tools/diag/ab_passes.py, c4_variants.py) and HBM WRITE_SIZE of one backward
# dispatch (rocprofv3 --pmc, own pass) at configs 3 and 4.  Variants are built
# beforehand into build/gran_<name>/ (tools/diag/build_variant.sh).
#   tools/diag/gran_layout_ab.sh name1 name2 ...
set -e
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/gran_ab
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  lib=$ROOT/build/gran_$v/libirlmx.so
  for cfg in "128 64" "256 32"; do
    tag=${v}_${cfg// /_}
    (cd /tmp && IRLMX_LIB=$lib timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$tag -o w -- python3 $ROOT/tools/diag/bwd_once.py $cfg > $OUT/$tag.log 2>&1)
    python3 - "$OUT/$tag" "$v" "$cfg" <<'PY'
import csv, glob, sys
rows = [r for p in glob.glob(sys.argv[1] + "/*counter_collection.csv") for r in csv.DictReader(open(p))
        if "cluster_kernel<1" in r["Kernel_Name"]]
last = max(int(r["Dispatch_Id"]) for r in rows)
w = sum(float(r["Counter_Value"]) for r in rows if int(r["Dispatch_Id"]) == last) * 1024
print(f"[{sys.argv[2]}] {sys.argv[3]}: backward WRITE_SIZE {w / 1e9:.2f} GB per launch", flush=True)
PY
  done
  IRLMX_LIB=$lib timeout -k 10 200 python3 $ROOT/tools/diag/ab_passes.py $v
  IRLMX_LIB=$lib timeout -k 10 200 python3 $ROOT/tools/diag/c4_variants.py 2>&1 | grep -E "^cw-default|stamps.*R=32 G=4" || true
done
