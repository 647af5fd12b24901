#!/bin/bash
# Round-6 probe 1 (gpurun, repo root): counter list, config-2 parity tests, new
# table-property / decay-bound tests, full-run step breakdown.
mkdir -p gpurun_out/r06a
(cd /tmp && TMPDIR=/tmp timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r06a/counters.txt 2>&1) ; echo "rocprofv3 -L rc=$?"
tools/gpu_steps.sh \
  "r06a/c2_tests|600|python -u -m pytest tests/test_gpu_argmax.py tests/test_gpu_bench_plans.py -m gpu -x -v --timeout 500 --timeout-method thread -k 'config2 or c2_64'" \
  "r06a/new_tests|300|python -u -m pytest tests/test_gpu_errors.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k 'unsorted or properties or feeding_nobody or rescale_extremes or width256'" \
  "r06a/full_run_steps|300|python -u tools/diag/full_run_steps.py"
