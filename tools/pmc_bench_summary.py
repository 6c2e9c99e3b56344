"""Reduce rocprofv3 --pmc CSVs of one bench config to profiles/pmc_r03_<cfg>.json (read by
bench.py): per-launch medians over the dispatches of the timed kernel instance.
HBM bytes per launch (MI355X_MICROARCH.md §HBM): FETCH_SIZE x2 (gfx950 reports half the
bytes of wide coalesced reads) x 1024 + WRITE_SIZE x 1024 (both in KiB).
usage: python tools/pmc_bench_summary.py OUT.json KERNEL FRAMES_PER_LAUNCH file.csv ..."""
import collections
import csv
import json
import os
import statistics
import sys

out, kernel, fpl, files = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4:]
vals = collections.defaultdict(list)
for f in files:
    per = collections.defaultdict(float)
    if not f.endswith(".csv"):
        continue
    for r in csv.DictReader(open(f)):
        if kernel + "(" not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (_, c), v in per.items():
        vals[c].append(v)
med = {c: statistics.median(v) for c, v in vals.items()}
# launches per timed unit (PMC_QUEUES: concurrent parts of one one-frame update, each a launch
# over an equal share of the image's workgroups)
queues = int(os.environ.get("PMC_QUEUES", "1"))
res = {"kernel": kernel, "frames_per_launch": fpl, "queues": queues,
       "dispatches": {c: len(v) for c, v in vals.items()}, "median_per_launch": med}
if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
    res["hbm_read_bytes_per_launch"] = med["FETCH_SIZE"] * 2 * 1024
    res["hbm_write_bytes_per_launch"] = med["WRITE_SIZE"] * 1024
    res["hbm_bytes_per_launch"] = res["hbm_read_bytes_per_launch"] + res["hbm_write_bytes_per_launch"]
    res["correction"] = "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> bytes"
    res["hbm_bytes_per_update"] = res["hbm_bytes_per_launch"] * queues
if "SQ_INSTS_VALU" in med:
    res["valu_insts_per_launch"] = med["SQ_INSTS_VALU"]
    res["valu_insts_per_update"] = med["SQ_INSTS_VALU"] * queues
    res["valu_insts_per_wave"] = med["SQ_INSTS_VALU"] / max(1.0, med.get("SQ_WAVES", 1.0))
if "GRBM_GUI_ACTIVE" in med:
    res["gui_active_cycles_per_xcd"] = med["GRBM_GUI_ACTIVE"] / 8
if "SQ_ACTIVE_INST_VALU" in med:
    # quad-cycles (SQ_WAVE_CYCLES / SQ_WAVES in the same unit matches the measured mean wave
    # life): the VALU pipes' busy cycles summed over all SIMDs
    res["valu_active_cycles_per_launch"] = med["SQ_ACTIVE_INST_VALU"] * 4
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "dispatches"}))
