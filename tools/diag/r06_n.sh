#!/bin/bash
tools/gpu_steps.sh \
  "r06n/resc_ab|400|for k in 1 2 3; do python -u tools/diag/bwd_ab.py resc16 && IRLMX_LIB=build/resc32/libirlmx.so python -u tools/diag/bwd_ab.py resc32; done"
