#!/bin/bash
tools/gpu_steps.sh \
  "r06h/mid_plans|300|python -u tools/diag/mid_plans.py" \
  "r06h/pad_ab|300|for k in 1 2 3; do python -u tools/diag/bwd_ab.py pad0 && IRLMX_LIB=build/gran_pad/libirlmx.so python -u tools/diag/bwd_ab.py pad; done"
