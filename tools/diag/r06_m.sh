#!/bin/bash
# Round 6: two ranks on the one GPU (the multi-rank launch path), whole irl runs of configs 4 and 5.
tools/gpu_steps.sh \
  "r06m/bench_2rank|300|python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-full-run > gpurun_out/r06m/bench_2rank.json" \
  "r06m/full_c4|400|python -u bench.py --config c4 --steps 2 --warmup 1 --full-run --no-cpu-baseline --no-config1 --first-steps 0 > gpurun_out/r06m/full_c4.json" \
  "r06m/full_c5|300|python -u bench.py --config c5 --steps 2 --warmup 1 --full-run --no-cpu-baseline --no-config1 --first-steps 0 > gpurun_out/r06m/full_c5.json"
