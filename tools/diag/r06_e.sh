#!/bin/bash
# Round-6 probe 5: forward with no bookkeeping (timing bound), granule padding A/B at configs 3/4.
tools/gpu_steps.sh \
  "r06e/fwd_ab|300|for k in 1 2; do python -u tools/diag/ab_passes.py default && IRLMX_LIB=build/fwdnoacct/libirlmx.so python -u tools/diag/ab_passes.py noacct; done" \
  "r06e/fwd_stamps|300|IRLMX_LIB=build/fwdnoacct/libirlmx.so python -u tools/diag/fwd_stamps.py" \
  "r06e/pad_ab|500|for k in 1 2 3; do python -u tools/diag/bwd_ab.py pad && IRLMX_LIB=build/gran_pad0/libirlmx.so python -u tools/diag/bwd_ab.py pad0; done" \
  "r06e/pad_stamps|300|python -u tools/diag/c4_variants.py 128 64 && IRLMX_LIB=build/gran_pad0/libirlmx.so python -u tools/diag/c4_variants.py 128 64"
