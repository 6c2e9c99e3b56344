"""Prints the headline fields of a bench.py JSON line (its last line starting with '{').
usage: python tools/summarize_bench.py LINE.json"""
import json
import sys

d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
r = d["roofline"]
print(d["config"]["workload"][:40], "value", d["value"], "ms/step", d["ms_per_step"],
      "kernel", r["kernel"], r["kernel_avg_us"], "bound", r["bound"], "frac", r["frac"],
      "hbm", r.get("hbm", {}).get("frac", r.get("frac")), "image_ok", d["image_ok"],
      d["image_check"], "share_ok", d.get("share_ok"), "segs/s", d.get("segments_per_s"))
print("timed", d["timed_breakdown_ms"])
if d.get("side_error"):
    print("SIDE ERROR", d["side_error"])
for key in ("dispatch", "k2", "k3"):
    if key in d:
        v = d[key]
        print(key, v["config"], "wall", v["us_per_step"], "ev", v["events_us_per_step"],
              "hbm", v["hbm_frac_events"], v["kernel"], v["image_ok"])
for key in ("k4", "k5"):
    if key in d:
        v = d[key]
        print(key, v["us_per_step"], v["kernel"], v["image_ok"], v.get("segments_per_s"))
rs = d.get("rank_shares")
if rs:
    for s in (20, 200):
        rows = rs[f"K3_chain_{s}_steps"]
        print(f"K3 chain {s} steps", {k: (v["us_per_step"], v["events_us_per_step"],
                                          v["efficiency"], v["image_ok"], v.get("rank_spread"))
                                      for k, v in rows.items()})
    print("call model", rs["K3_call_model"], "runtime floor", rs["runtime_floor_us"])
    for key in ("K5_fused_64", "K5_balanced_64"):
        if key in rs:
            print(key, {k: (v["us_per_step"], v["efficiency"], v["image_ok"],
                            v.get("rank_spread")) for k, v in rs[key].items()
                        if isinstance(v, dict)})
if "cpu_baseline" in d:
    print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
