#!/bin/bash
# A/B of the config-4 backward on one box: the in-tree library against a variant
# built by tools/diag/build_variant.sh (usage: tools/diag/ab_c4.sh VARIANT)
v=${1:-lazy}
B="python bench.py --config c4 --steps 4 --warmup 1 --no-cpu-baseline --no-config1 --first-steps 0"
tools/gpu_steps.sh "base1|120|$B" "${v}1|120|IRLMX_LIB=build/$v/libirlmx.so $B" "base2|120|$B" "${v}2|120|IRLMX_LIB=build/$v/libirlmx.so $B"
