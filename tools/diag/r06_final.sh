#!/bin/bash
# Round-6 evidence run on one MI355X (via gpurun, from the repo root): the bench lines of every
# config, rocprofv3 kernel-trace + HBM passes for configs 3 and 4, SQ counter passes of the
# config-3 backward, L2 write-back counters, phase stamps.  Each step has its own time limit; a
# fatal exit stops the script (tools/gpu_steps.sh).
tools/gpu_steps.sh \
  "r06/gputest|700|python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread" \
  "r06/smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "r06/bench|400|python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06/bench.json" \
  "r06/bench_c2|200|python -u bench.py --config c2 --steps 10 --warmup 3 > gpurun_out/r06/bench_c2.json" \
  "r06/bench_c2s|200|python -u bench.py --config c2s --steps 10 --warmup 3 > gpurun_out/r06/bench_c2s.json" \
  "r06/bench_c4|300|python -u bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/r06/bench_c4.json" \
  "r06/bench_c5|200|python -u bench.py --config c5 --steps 5 --warmup 2 > gpurun_out/r06/bench_c5.json" \
  "r06/bench_c5b64|200|python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 > gpurun_out/r06/bench_c5b64.json" \
  "r06/prof_c3|300|bash tools/profile_round.sh r06" \
  "r06/prof_c4|300|bash tools/profile_round.sh r06c4 --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-config1 --first-steps 0 --no-full-run" \
  "r06/pmc_c3|300|bash tools/diag/pmc_bwd.sh pmc_c3 128 64" \
  "r06/stamps|200|python -u tools/diag/c4_variants.py 128 64 && python -u tools/diag/fwd_stamps.py"
