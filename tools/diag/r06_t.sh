#!/bin/bash
# final numpy exp / log build (bucket count where the tables are in LDS and one
# state per thread, compares elsewhere): soft VI cost vs device ocml, GPU suite, config-5 benches
tools/gpu_steps.sh \
  "r06t/soft_ab|300|for k in 1 2 3; do python -u tools/diag/soft_ab.py npmath && IRLMX_LIB=build/ocml/libirlmx.so python -u tools/diag/soft_ab.py ocml; done" \
  "r06t/gputest|700|python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread" \
  "r06t/bench_c5|200|python -u bench.py --config c5 --steps 5 --warmup 2 > gpurun_out/r06t/bench_c5.json" \
  "r06t/bench_c5b64|200|python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 > gpurun_out/r06t/bench_c5b64.json"
