#!/bin/bash
# Round-6 probe 4: forward bookkeeping A/B (ballot default vs build/fwdbranch), forward parity.
tools/gpu_steps.sh \
  "r06d/fwd_tests|600|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan_fuzz.py tests/test_gpu_bench_plans.py -m gpu -x -v --timeout 500 --timeout-method thread -k 'forward or fwd or cluster or fuzz or shapes or config3_bench or config5_bench or config2_bench or stops'" \
  "r06d/ab|400|for k in 1 2 3; do python -u tools/diag/ab_passes.py ballot && IRLMX_LIB=build/fwdbranch/libirlmx.so python -u tools/diag/ab_passes.py branch; done" \
  "r06d/stamps|300|python -u tools/diag/fwd_stamps.py && IRLMX_LIB=build/fwdbranch/libirlmx.so python -u tools/diag/fwd_stamps.py"
