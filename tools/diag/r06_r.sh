#!/bin/bash
# soft VI cost of numpy's exp / log: LDS tables + tree thresholds (default) vs
# global tables (build/npglob) vs device ocml (build/ocml); then the soft-VI parity tests
tools/gpu_steps.sh \
  "r06r/soft_ab|400|for k in 1 2 3; do python -u tools/diag/soft_ab.py npmath-lds && IRLMX_LIB=build/npglob/libirlmx.so python -u tools/diag/soft_ab.py npmath-global && IRLMX_LIB=build/ocml/libirlmx.so python -u tools/diag/soft_ab.py ocml; done" \
  "r06r/tests|400|python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_npmath.py tests/test_gpu_argmax.py tests/test_gpu_parity.py -k 'npmath or causal or soft or config2 or bellman or vi'"
