"""Summarise a rocprofv3 kernel trace of `bench.py --steps K --warmup W
--no-extra ...` (tools/sessions/r5.sh e2etrace): the settle loop's G
evaluations, the kernel leg's one-step sweeps and each run_sharded call of the
end-to-end leg (warm-up run, then the timed run), with their per-step kernel
times and the idle gaps in front of them.

  python tools/e2e_trace_summary.py <trace dir> > summary.json
"""
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    path = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    t0 = ev[0][0]
    # group consecutive launches of one kernel family; a run() shows as
    # eval (Φ(u0)) followed by one multi-step sweep launch
    groups = []
    prev_end = None
    for s, e, name in ev:
        fam = ("sweep" if "sweep_kernel" in name else "eval" if "eval_kernel" in name else
               "ordered_sum" if "ordered_sum" in name else "other")
        gap = 0 if prev_end is None else (s - prev_end) / 1e3
        if groups and groups[-1]["family"] == fam and fam in ("sweep", "eval") and gap < 200:
            g = groups[-1]
            g["launches"] += 1
            g["kernel_us"].append((e - s) / 1e3)
            g["end"] = e
        else:
            groups.append({"family": fam, "name": name[:90], "launches": 1, "kernel_us": [(e - s) / 1e3],
                           "start_ms": (s - t0) / 1e6, "idle_before_us": gap, "end": e})
        prev_end = e
    out = []
    last_end = None
    for g in groups:
        if g["family"] == "other" and g["kernel_us"][0] < 50:
            continue  # the run's small copies and fills
        k = g.pop("kernel_us")
        start = t0 + g["start_ms"] * 1e6
        g["ms_since_previous_group"] = None if last_end is None else (start - last_end) / 1e6
        last_end = g.pop("end")
        g["kernel_ms_total"] = sum(k) / 1e3
        g["kernel_ms_first"], g["kernel_ms_last"] = k[0] / 1e3, k[-1] / 1e3
        g["kernel_ms_mean"] = sum(k) / len(k) / 1e3
        out.append(g)
    print(json.dumps({"trace": os.path.relpath(path), "groups": out}, indent=1))


if __name__ == "__main__":
    main()
