#!/bin/bash
# Config 2 backward: solo-tile block length (IRLMX_SOLO_T) sweep on one box, then the bit-identity tests.
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-config1 --first-steps 0 --no-full-run --config c2"
tools/gpu_steps.sh "t16|120|IRLMX_SOLO_T=16 $B" "t64|120|$B" "t128|120|IRLMX_SOLO_T=128 $B" "t256|120|IRLMX_SOLO_T=256 $B" "t16b|120|IRLMX_SOLO_T=16 $B" "t64b|120|$B" \
  "bitid|300|python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu -k 'pair_layout or shapes_bit or maxent_small or config1' -p no:cacheprovider"
