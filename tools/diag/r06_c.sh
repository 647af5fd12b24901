#!/bin/bash
# Round-6 probe 3: L2 write-back counters of config 3's backward (default vs unpadded granules).
tools/gpu_steps.sh "r06c/pmc_wb|600|bash tools/diag/pmc_writeback.sh"
