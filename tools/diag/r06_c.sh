#!/bin/bash
# Round-6 probe 3: L2 write-back counters of config 3's backward (default vs unpadded granules);
# forward p0-skip A/B (default vs build/p0on); forward parity + plan fuzz on the new build.
tools/gpu_steps.sh \
  "r06c/fwd_tests|600|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan_fuzz.py tests/test_gpu_bench_plans.py -m gpu -x -v --timeout 500 --timeout-method thread -k 'forward or fwd or cluster or fuzz or shapes or config3_bench or config5_bench or config2_bench'" \
  "r06c/ab|400|python -u tools/diag/ab_passes.py p0skip && IRLMX_LIB=build/p0on/libirlmx.so python -u tools/diag/ab_passes.py p0on && python -u tools/diag/ab_passes.py p0skip && IRLMX_LIB=build/p0on/libirlmx.so python -u tools/diag/ab_passes.py p0on" \
  "r06c/stamps|300|python -u tools/diag/fwd_stamps.py && IRLMX_LIB=build/p0on/libirlmx.so python -u tools/diag/fwd_stamps.py" \
  "r06c/pmc_wb|600|bash tools/diag/pmc_writeback.sh"
