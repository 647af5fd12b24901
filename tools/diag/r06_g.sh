#!/bin/bash
# Round-6 run 7: the default bench line, granule padding A/B, other configs' lines.
tools/gpu_steps.sh \
  "r06g/bench|400|python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06g/bench.json" \
  "r06g/pad_ab|300|for k in 1 2 3; do python -u tools/diag/bwd_ab.py pad0 && IRLMX_LIB=build/gran_pad/libirlmx.so python -u tools/diag/bwd_ab.py pad; done" \
  "r06g/bench_c5|200|python -u bench.py --config c5 --steps 5 --warmup 2 > gpurun_out/r06g/bench_c5.json" \
  "r06g/bench_c5b64|200|python -u bench.py --config c5 --batch 64 --steps 10 --warmup 3 > gpurun_out/r06g/bench_c5b64.json" \
  "r06g/bench_c2|200|python -u bench.py --config c2 --steps 10 --warmup 3 > gpurun_out/r06g/bench_c2.json"
