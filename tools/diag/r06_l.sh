#!/bin/bash
tools/gpu_steps.sh \
  "r06l/fwd_plans|300|python -u tools/diag/fwd_plans.py && python -u tools/diag/fwd_plans.py 64" \
  "r06l/fwd_dpp|300|for k in 1 2 3; do python -u tools/diag/ab_passes.py lds && IRLMX_LIB=build/fwd_dpp/libirlmx.so python -u tools/diag/ab_passes.py dpp; done"
