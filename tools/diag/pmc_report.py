"""Per-wave-sweep table of the SQ counter passes of tools/diag/pmc_bwd.sh.
usage: python tools/diag/pmc_report.py gpurun_out/<tag> SWEEPS_PER_LAUNCH "<header text>"
(the driver runs two launches; the last dispatch of the cluster kernel is used)."""
import csv
import glob
import os
import sys
from collections import defaultdict

src, sweeps, header = sys.argv[1], int(sys.argv[2]), sys.argv[3]
vals = defaultdict(dict)
for path in glob.glob(os.path.join(src, "p*", "*counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        if "cluster_kernel<1" not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]][int(r["Dispatch_Id"])] = float(r["Counter_Value"])
# the last dispatch of the kernel in each pass (the driver's second, measured call)
agg = {k: v[max(v)] for k, v in vals.items()}
waves = agg.get("SQ_WAVES", 1.0)
print(header)
print("SQ_* cycle counters are quad-cycles (MI355X_MICROARCH.md); per wave-sweep = value / SQ_WAVES / sweeps.\n")
for k in sorted(agg):
    print(f"{k:28s} {agg[k]:20.0f}   per wave-sweep {agg[k] / waves / sweeps:10.2f}")
wc = agg.get("SQ_WAVE_CYCLES")
if wc:
    print()
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
              "SQ_WAIT_INST_LDS"):
        if k in agg:
            print(f"{k:28s} {100.0 * agg[k] / wc:6.1f} % of SQ_WAVE_CYCLES")
