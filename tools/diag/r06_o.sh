#!/bin/bash
# Config-4 / config-3 backward L2 write-back vs the rescale period (32 default, 16 variant)
tools/gpu_steps.sh \
  "r06o/wb_c4|300|VARIANTS='default resc16' bash tools/diag/pmc_writeback.sh 256 32 pmc_wb_c4" \
  "r06o/wb_c3|300|VARIANTS='default resc16' bash tools/diag/pmc_writeback.sh 128 64 pmc_wb_c3" \
  "r06o/resc_ab|400|for k in 1 2 3; do python -u tools/diag/bwd_ab.py resc32 && IRLMX_LIB=build/resc16/libirlmx.so python -u tools/diag/bwd_ab.py resc16; done"
