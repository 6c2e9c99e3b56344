"""Kernel statistics from a rocprofv3 --kernel-trace database (rocpd SQLite, the default
output): per kernel name the calls, total / average / min / max duration (us), and for
kernels that run as concurrent parts (rt_set_update_queues) the union of their intervals —
the time the GPU had at least one of them running — per `units` (e.g. updates).
With RT_WINDOW=LINE.json (a bench.py line run with RT_TIMELINE=1: its `timeline_host` holds
CLOCK_MONOTONIC / CLOCK_BOOTTIME ns at the timed region's start and after its closing
synchronize) only the dispatches that start inside the timed region are counted — the
profile of the timed steps alone, not the warm-up or the side lines.
usage: [RT_WINDOW=LINE.json] python tools/rocpd_stats.py DB.db [KERNEL_SUBSTRING UNITS] > stats.csv"""
import json
import os
import csv
import sqlite3
import sys


def main(db, sub=None, units=None):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels"))
    win = os.environ.get("RT_WINDOW")
    if win:
        host = json.loads(open(win).read().strip().splitlines()[-1])["timeline_host"]
        # the clock whose [t0, synced] window holds dispatches
        best = max(((k, [r for r in rows if host["t0"][k] <= r[1] <= host["synced"][k]])
                    for k in (0, 1)), key=lambda kr: len(kr[1]))
        rows = best[1]
        print(f"# dispatches starting inside the timed region ({('monotonic', 'boottime')[best[0]]} "
              f"clock): {len(rows)}")
    by = {}
    for name, s, e in rows:
        by.setdefault(name, []).append((s, e))
    w = csv.writer(sys.stdout)
    w.writerow(["name", "calls", "total_us", "average_us", "min_us", "max_us"])
    for name, iv in sorted(by.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
        d = [(e - s) / 1e3 for s, e in iv]
        w.writerow([name, len(d), round(sum(d), 3), round(sum(d) / len(d), 3),
                    round(min(d), 3), round(max(d), 3)])
    if sub:
        iv = sorted((s, e) for name, s, e in rows if sub in name)
        busy, cur_s, cur_e = 0, None, None
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        span = (iv[-1][1] - iv[0][0]) / 1e3 if iv else 0.0
        n = int(units) if units else len(iv)
        w.writerow([])
        w.writerow(["# kernels matching", sub, "launches", len(iv), "units", n])
        w.writerow(["# union of their intervals us", round(busy / 1e3, 3),
                    "per unit", round(busy / 1e3 / max(1, n), 3),
                    "first start to last end us", round(span, 3)])


if __name__ == "__main__":
    main(*sys.argv[1:4])
