#!/bin/bash
# Round-6 A/B: round-5 library (build/r05) vs the current one, backward at configs 3/4 and the forward passes.
tools/gpu_steps.sh \
  "r06k/bwd_ab|400|for k in 1 2 3; do python -u tools/diag/bwd_ab.py cur && IRLMX_LIB=build/r05/libirlmx.so python -u tools/diag/bwd_ab.py r05; done" \
  "r06k/fwd_ab|300|for k in 1 2; do python -u tools/diag/ab_passes.py cur && IRLMX_LIB=build/r05/libirlmx.so python -u tools/diag/ab_passes.py r05; done" \
  "r06k/stamps|200|python -u tools/diag/c4_variants.py 128 64 2>&1 | grep -E 'cw-default|lds-cols' && IRLMX_LIB=build/r05/libirlmx.so python -u tools/diag/c4_variants.py 128 64 2>&1 | grep -E 'cw-default|lds-cols'"
