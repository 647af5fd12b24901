#!/bin/bash
# Config 2 vs config 2s backward on one box, with in-kernel phase stamps
# (3.95 vs 3.38 ms on the identical plan).
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-config1 --first-steps 0 --no-full-run"
tools/gpu_steps.sh "c2a|120|IRLMX_STAMPS=1 $B --config c2" "c2sa|120|IRLMX_STAMPS=1 $B --config c2s" \
  "c2b|120|IRLMX_STAMPS=1 $B --config c2" "c2sb|120|IRLMX_STAMPS=1 $B --config c2s" \
  "c2n|120|$B --config c2" "c2sn|120|$B --config c2s"
