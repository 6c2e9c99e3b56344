"""Timeline of bench.py's timed region (diagnostic): where the wall time of the K steps goes.

Run bench.py with RT_TIMELINE=1 under
    rocprofv3 --kernel-trace --hip-runtime-trace -f csv -d DIR -- python3 bench.py ...
(the line then carries `timeline_host`: CLOCK_MONOTONIC / CLOCK_BOOTTIME ns at the region's
start, when the steps' issue returned, and after the closing synchronize), then
    python tools/timeline.py DIR LINE.json > timeline.json
places the host stamps on the trace (the clock whose t0 falls on the region's first HIP call)
and attributes the region: host time before the first launch reaches the GPU, the kernels'
busy time (the union of every dispatch's interval), idle gaps between them, and the time
from the last kernel's end to the synchronize's return.  Every HIP call and dispatch inside
the region is listed relative to t0 (µs).  The profiler adds its own per-call and
per-dispatch cost, so the absolute figures run longer than an unprofiled run's: the split
between the phases is what the file is for."""
import csv
import glob
import json
import os
import sys


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def find(d, pat):
    hits = sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))
    return hits[-1] if hits else None


def union(iv):
    busy, cs, ce, out = 0, None, None, []
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
                out.append((cs, ce))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        busy += ce - cs
        out.append((cs, ce))
    return busy, out


def main(d, line_path):
    line = json.loads(open(line_path).read().strip().splitlines()[-1])
    host = line["timeline_host"]
    kt = rows(find(d, "*kernel_trace.csv"))
    api_path = find(d, "*hip_api_trace.csv")
    api = rows(api_path) if api_path else []
    calls = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in api]
    # which clock the trace uses: the one whose [t0, issued] window holds HIP calls
    # (no API trace: the one whose [t0, synced] window holds dispatches)
    best = None
    for k, name in enumerate(("monotonic", "boottime")):
        t0, t1 = host["t0"][k], host["issued" if calls else "synced"][k]
        if calls:
            n = sum(1 for s, e, f in calls if t0 <= s <= t1)
        else:
            n = sum(1 for r in kt if t0 <= int(r["Start_Timestamp"]) <= t1)
        if best is None or n > best[0]:
            best = (n, k, name)
    _, k, clock = best
    t0, t_iss, t_sync = host["t0"][k], host["issued"][k], host["synced"][k]
    us = lambda t: round((t - t0) / 1e3, 2)
    disp = []
    for r in kt:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s <= t_sync:
            disp.append((s, e, r["Kernel_Name"].split("(")[0], r.get("Stream_Id", r.get("Queue_Id"))))
    disp.sort()
    region_calls = [(s, e, f) for s, e, f in calls if t0 <= s <= t_sync]
    launches = [c for c in region_calls if "Launch" in c[2]]
    busy, spans = union([(s, e) for s, e, _, _ in disp])
    gaps = [spans[i + 1][0] - spans[i][1] for i in range(len(spans) - 1)]
    first_k, last_k = (disp[0][0], max(e for _, e, _, _ in disp)) if disp else (t0, t0)
    wall = t_sync - t0
    out = {
        "clock": clock,
        "steps": line.get("steps"), "value": line.get("value"),
        "ms_per_step": line.get("ms_per_step"),
        "kernel_avg_us": line.get("roofline", {}).get("kernel_avg_us"),
        "wall_us": us(t_sync),
        "host_issue_us": us(t_iss),
        "first_hip_call_us": us(region_calls[0][0]) if region_calls else None,
        "first_launch_call_us": us(launches[0][0]) if launches else None,
        "first_launch_call_end_us": us(launches[0][1]) if launches else None,
        "first_kernel_start_us": us(first_k),
        "last_kernel_end_us": us(last_k),
        "sync_return_after_last_kernel_us": round((t_sync - last_k) / 1e3, 2),
        "kernel_busy_us": round(busy / 1e3, 2),
        "idle_gaps_us": round(sum(gaps) / 1e3, 2),
        "idle_gaps": len(gaps),
        "largest_gaps_us": sorted((round(g / 1e3, 2) for g in gaps), reverse=True)[:8],
        "dispatches": len(disp),
        "launch_calls": len(launches),
        "attribution_us": {
            "before_first_kernel": us(first_k),
            "kernels_busy": round(busy / 1e3, 2),
            "gaps_between_kernels": round(sum(gaps) / 1e3, 2),
            "after_last_kernel": round((t_sync - last_k) / 1e3, 2),
        },
        "wall_check_us": round(wall / 1e3, 2),
        "hip_calls": [[us(s), round((e - s) / 1e3, 2), f] for s, e, f in region_calls],
        "kernels": [[us(s), us(e), round((e - s) / 1e3, 2), n, q] for s, e, n, q in disp],
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:3])
