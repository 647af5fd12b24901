#!/bin/bash
# Round-6 probe 6: cheap convergence proof (default) -- forward parity, stop-edge tests, plan fuzz,
# bench-plan fixtures; A/B vs full bookkeeping (build/fwdfull) and stamps; default layout now unpadded.
tools/gpu_steps.sh \
  "r06f/fwd_tests|900|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan_fuzz.py tests/test_gpu_bench_plans.py tests/test_gpu_full_size.py tests/test_gpu_errors.py tests/test_gpu_coresidency.py -m gpu -x -v --timeout 600 --timeout-method thread" \
  "r06f/ab|400|for k in 1 2 3; do python -u tools/diag/ab_passes.py proof && IRLMX_LIB=build/fwdfull/libirlmx.so python -u tools/diag/ab_passes.py full; done" \
  "r06f/stamps|300|python -u tools/diag/fwd_stamps.py && IRLMX_LIB=build/fwdfull/libirlmx.so python -u tools/diag/fwd_stamps.py"
