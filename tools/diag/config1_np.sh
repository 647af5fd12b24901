#!/bin/bash
# Config 1 drop-in full runs with and without numpy's order (IRLMX_NUMPY_ORDER), plus a
# per-call timing of each numpy-order kernel at 5x5.
tools/gpu_steps.sh "c1np|200|python -u tools/diag/config1_timing.py" "c1fast|200|IRLMX_NUMPY_ORDER=0 python -u tools/diag/config1_timing.py" \
  "npcalls|200|python -u tools/diag/np_calls.py"
