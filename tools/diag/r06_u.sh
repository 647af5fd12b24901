#!/bin/bash
# final build: smoke and the default bench (config 3)
tools/gpu_steps.sh \
  "r06u/smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "r06u/bench|400|python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06u/bench.json"
