#!/bin/bash
# Round-6 probe 2: config-2 drop-in test (relaxed at sub-ulp soft-VI ties), first-use costs of
# the compaction pieces, the full run with the compaction primed, L2 write-back counters.
tools/gpu_steps.sh \
  "r06b/c2_tests|600|python -u -m pytest tests/test_gpu_argmax.py tests/test_gpu_bench_plans.py -m gpu -x -v --timeout 500 --timeout-method thread -k 'config2 or c2_64'" \
  "r06b/compact_cost|200|python -u tools/diag/compact_cost.py" \
  "r06b/full_run_steps|300|python -u tools/diag/full_run_steps.py" \
  "r06b/pmc_wb|600|bash tools/diag/pmc_writeback.sh"
