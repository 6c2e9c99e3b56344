"""VALU attribution of the camera-ray sample by knock-out builds (round-6 verdict item 3).

The knock-out variants come from tools/patches/single_knockouts.patch (applied to a copy of
the tree; `make variant TAG=skoK VFLAGS=-DRT_SKO=K`): bit 1 no accumulator load, 2 no
sphere scan (so no hit shading), 4 no random camera ray (a pinhole ray through the pixel
corner), 8 no hit shading, 16 no image store (one-frame kernel only).  Each variant runs the
driver's K3 command under one rocprofv3 --pmc pass (SQ_INSTS_VALU, SQ_INSTS_SALU,
SQ_WAVES); this script reads the CSVs and prints, per timed kernel, the VALU and SALU
wave-instructions per wave of each build and the differences against the product build: the
dynamic instruction count each phase costs.  Knock-outs overlap a little (a pinhole ray
changes which spheres a pixel tests), so the phases are attributed one at a time against the
product build, and the all-out build (14 = 2|4|8) is what remains: setup, tile
coordinates, masks, list-count loads, the sky and the accumulation.
usage: python tools/valu_attribution.py RAW_DIR > attribution.json"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

raw = sys.argv[1]
KERNELS = {"dispatch": "rt_single_kernel<2>", "chain": "rt_tpair_kernel<2>"}
out = {}
for f in sorted(glob.glob(os.path.join(raw, "**", "*counter_collection.csv"), recursive=True)):
    tag = os.path.basename(f).split("_counter_collection")[0]
    mode, _, build = tag.partition("_")
    kern = KERNELS.get(mode)
    if kern is None:
        continue
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if kern + "(" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    rows = [d for d in per.values() if d.get("SQ_WAVES")]
    if not rows:
        continue
    med = {c: statistics.median(d[c] for d in rows) for c in rows[0]}
    out.setdefault(mode, {})[build] = {
        "dispatches": len(rows),
        "valu_per_wave": round(med["SQ_INSTS_VALU"] / med["SQ_WAVES"], 2),
        "salu_per_wave": round(med["SQ_INSTS_SALU"] / med["SQ_WAVES"], 2),
        "waves": med["SQ_WAVES"]}
NAMES = {"sko1": "accumulator load", "sko2": "sphere scan + hit shading",
         "sko4": "random camera ray (4 hashes, lens, jitter)", "sko8": "hit shading",
         "sko14": "all of 2|4|8 out: what remains (setup, masks, counts, sky, accumulation, load, store)"}
for mode, builds in out.items():
    base = builds.get("base")
    if not base:
        continue
    attr = {}
    for b, v in builds.items():
        if b in NAMES:
            d = base["valu_per_wave"] - v["valu_per_wave"]
            attr[b] = {"phase": NAMES[b],
                       "valu_per_wave": round(d if b != "sko14" else v["valu_per_wave"], 2),
                       "share": round((d if b != "sko14" else v["valu_per_wave"]) /
                                      base["valu_per_wave"], 4)}
    builds["attribution"] = attr
print(json.dumps(out, indent=1))
