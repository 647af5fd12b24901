#!/bin/bash
# Round-5 evidence run on one MI355X (via gpurun, from the repo root): GPU tests,
# smoke, the bench lines of every config, rocprofv3 kernel-trace + HBM passes
# for configs 3 and 4, SQ counter passes of both backward kernels, phase stamps.
# Each step has its own time limit; a fatal exit stops the script (gpu_steps.sh).
tools/gpu_steps.sh \
  "r05_gputest|900|python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread" \
  "r05_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "r05_bench|400|python -u bench.py" \
  "r05_bench_c2|300|python -u bench.py --config c2 --steps 10 --warmup 3" \
  "r05_bench_c2s|300|python -u bench.py --config c2s --steps 10 --warmup 3" \
  "r05_bench_c4|400|python -u bench.py --config c4 --steps 5 --warmup 2" \
  "r05_bench_c5|400|python -u bench.py --config c5 --steps 5 --warmup 2" \
  "r05_bench_c5b64|400|python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3" \
  "r05_prof_c3|400|bash tools/profile_round.sh r05" \
  "r05_prof_c4|400|bash tools/profile_round.sh r05c4 --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-config1 --first-steps 0 --no-full-run" \
  "r05_pmc_c3|400|bash tools/diag/pmc_bwd.sh pmc_c3 128 64" \
  "r05_pmc_c4|400|bash tools/diag/pmc_bwd.sh pmc_c4 256 32" \
  "r05_stamps|300|python -u tools/diag/c4_variants.py && python -u tools/diag/c4_variants.py 128 64"
