"""The bench line's kernel time from a rocprofv3 kernel trace, restricted to
the launches the line times.

  rocprofv3 --kernel-trace --stats -d DIR -o bench -- python bench.py --steps K --warmup W ...
  python tools/trace_summary.py DIR K W [bench_line.json] > summary.json

bench.py's kernel leg runs first: W untimed and then K timed launches of the
sweep kernel (one pCN step each for a full GPU); every later leg (the
end-to-end runs, f32, REFERENCE arith, the configs) comes after it.  The
dominant sweep kernel is the most-launched l96/burgers sweep kernel name;
its launches sorted by start time, [W, W + K) are the timed ones.  The
rocprofv3 --stats average of the same kernel name (reported beside) also
counts the multi-step launches of the end-to-end legs.
"""
import csv
import glob
import json
import os
import sys


def load(d):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            rows += list(csv.DictReader(f))
    return rows


def summarize(d, steps, warmup, line=None, match="sweep_kernel"):
    rows = [r for r in load(d) if match in r["Kernel_Name"]]
    if not rows:
        raise SystemExit(f"no '{match}' kernels in {d}")
    names = {}
    for r in rows:
        names[r["Kernel_Name"]] = names.get(r["Kernel_Name"], 0) + 1
    # the kernel leg's kernel: the first sweep kernel launched
    first = min(rows, key=lambda r: int(r["Start_Timestamp"]))["Kernel_Name"]
    ks = sorted((r for r in rows if r["Kernel_Name"] == first), key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in ks]
    timed = dur[warmup:warmup + steps]
    if len(timed) != steps:
        raise SystemExit(f"{len(dur)} launches of {first}, expected >= {warmup + steps}")
    out = {"kernel": first, "launches_of_this_kernel": len(dur),
           "timed_launches": f"launches {warmup}..{warmup + steps - 1} in start order (after the {warmup} warm-up "
                             f"launches of the kernel leg)",
           "timed_launch_avg_ms": sum(timed) / steps, "timed_launch_min_ms": min(timed),
           "timed_launch_max_ms": max(timed), "all_launches_of_this_kernel_avg_ms": sum(dur) / len(dur),
           "sweep_kernels_launched": names}
    if line:
        ln = json.load(open(line)) if isinstance(line, str) else line
        out["bench_line_kernel_ms_events"] = ln["roofline"]["kernel_ms"]
        out["ratio_trace_over_events"] = out["timed_launch_avg_ms"] / ln["roofline"]["kernel_ms"]
    return out


if __name__ == "__main__":
    d, k, w = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    print(json.dumps(summarize(d, k, w, sys.argv[4] if len(sys.argv) > 4 else None), indent=1))
