#!/bin/bash
# Round 5, session l: where the host time of a frame-chain call goes — rt_update_frames'
# phases stamped (librt_hip_stamps.so, -DRT_CALL_STAMPS: entry, device guard, prepare, kernel
# choice, planning, launch, return; ns, one stderr line per call) on the 8-rank K3 chain
# share and the driver's K3 region.
# Usage: bash tools/sessions/gpu_r05l.sh TAG
set -o pipefail
TAG=${1:-r05l}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
V=gpu-ray-tracing_amd/build/variants
RT_HIP_LIB=$V/librt_hip_stamps.so timeout -k 10 120 python tools/share_region.py 8 0 15 20 > $O/share_n8.json 2> $O/share_n8.err \
  || { tail $O/share_n8.err; exit 1; }
RT_HIP_LIB=$V/librt_hip_stamps.so timeout -k 10 120 python tools/driver_region.py 15 K3 stamps= > $O/region_k3.json 2> $O/region_k3.err \
  || { tail $O/region_k3.err; exit 1; }
for f in share_n8 region_k3; do
  python - $O/$f.err <<'PY'
import sys, statistics as st
rows = [list(map(int, l.split()[1:])) for l in open(sys.argv[1]) if l.startswith("RT_CALL_STAMPS")]
rows = [r for r in rows if r[0] == 20]
print(sys.argv[1], len(rows), "calls of 20 frames; median ns since entry: guard, prepare, choice, planned, launched, return =",
      [round(st.median(r[k] for r in rows)) for k in range(1, 7)])
PY
done
cat $O/share_n8.json
# VALU / SALU instructions of the 8-rank chain share's frame-group kernel (per tile and frame,
# against the one-frame kernel's 332 VALU per tile)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_s8 -o s8 -- python3 tools/share_region.py 8 0 3 20 \
  > $O/pmc_s8.log 2>&1 || { echo "pmc s8 failed"; tail -5 $O/pmc_s8.log; exit 1; }
python - $O/pmc_s8 <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
by = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    by[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in by.items():
    if "trace_kernel" in k:
        # (the 20-frame launches: the calls of 5 frames count a quarter of the work)
        top = max(d["SQ_INSTS_VALU"])
        keep = [i for i, v in enumerate(d["SQ_INSTS_VALU"]) if v > 0.6 * top]
        med = {c: sorted(v[i] for i in keep)[len(keep) // 2] for c, v in d.items()}
        print(k, {c: round(v) for c, v in med.items()}, "VALU per tile-frame", round(med["SQ_INSTS_VALU"] / (4080 * 20), 1),
              "SALU per tile-frame", round(med["SQ_INSTS_SALU"] / (4080 * 20), 1))
PY
