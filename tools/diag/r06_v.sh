#!/bin/bash
# config 5's whole irl_causal run on the final build (soft VI with numpy's exp / log)
tools/gpu_steps.sh \
  "r06v/full_c5|300|python -u bench.py --config c5 --steps 2 --warmup 1 --full-run --no-cpu-baseline --no-config1 --first-steps 0 > gpurun_out/r06v/full_c5.json"
