"""Reduce rocprofv3 --pmc counter_collection CSVs to a per-kernel JSON summary.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB, collected in separate passes; on gfx950 FETCH_SIZE reports half the bytes of a wide
(16 B/lane) coalesced streaming read, so it is doubled before adding WRITE_SIZE.
usage: python tools/pmc_summary.py OUT.json KERNEL_SUBSTR file1.csv [file2.csv ...]
(env FRAMES_PER_LAUNCH=F records the frames each profiled launch ran)
"""
import collections, csv, json, os, statistics, sys

out, ksub, files = sys.argv[1], sys.argv[2], sys.argv[3:]
vals = collections.defaultdict(list)
for f in files:
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if ksub not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
summ = {c: statistics.median(v) for c, v in vals.items()}
res = {"kernel": ksub, "dispatches": {c: len(v) for c, v in vals.items()}, "median_per_launch": summ,
       "frames_per_launch": int(os.environ.get("FRAMES_PER_LAUNCH", "1"))}
if "FETCH_SIZE" in summ and "WRITE_SIZE" in summ:
    res["hbm_read_bytes_per_launch"] = summ["FETCH_SIZE"] * 2 * 1024
    res["hbm_write_bytes_per_launch"] = summ["WRITE_SIZE"] * 1024
    res["hbm_bytes_per_launch"] = res["hbm_read_bytes_per_launch"] + res["hbm_write_bytes_per_launch"]
    res["correction"] = "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> bytes"
if "GRBM_GUI_ACTIVE" in summ:
    res["gui_active_cycles_per_xcd"] = summ["GRBM_GUI_ACTIVE"] / 8
if "SQ_INSTS_VALU" in summ and "SQ_WAVES" in summ:
    res["valu_insts_per_wave"] = summ["SQ_INSTS_VALU"] / summ["SQ_WAVES"]
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
