#!/bin/bash
# Profile the bench workload on the GPU box (run via gpurun from the repo root).
#   1. rocprofv3 --kernel-trace --stats      -> per-kernel durations
#   2. rocprofv3 --pmc FETCH_SIZE (own pass) -> HBM read bytes per dispatch
#   3. rocprofv3 --pmc WRITE_SIZE (own pass) -> HBM write bytes per dispatch
# Output under gpurun_out/prof_<tag>/; condensed by tools/parse_rocprof.py.
set -e
TAG=${1:-r01}
shift || true
ARGS=${@:-"--steps 2 --warmup 1 --no-cpu-baseline --no-config1 --first-steps 0 --no-full-run"}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $ROOT/bench.py $ARGS > $OUT/bench_kt.json 2> $OUT/kt.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $ROOT/bench.py $ARGS > $OUT/bench_fetch.json 2> $OUT/fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $ROOT/bench.py $ARGS > $OUT/bench_write.json 2> $OUT/write.err
# keep the merged-back tree small: the per-dispatch traces are not needed
rm -f $OUT/kt/*kernel_trace* $OUT/kt/*memory_copy* 2>/dev/null || true
find $OUT -name "*.csv"
