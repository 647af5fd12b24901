#!/bin/bash
tools/gpu_steps.sh \
  "r06p/npmath|300|python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_npmath.py tests/test_gpu_argmax.py"
