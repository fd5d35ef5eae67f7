"""Summarise rocprofv3 PMC passes of the headline sweep kernel into
profiles/<round>/pmc_l96_<dtype>.json (read by bench.py for roofline.traffic).

  python tools/pmc_summarize.py <dir with fetch/write/sq csv> <dtype> <chains> <out.json> [first]

`first`: only the first N dispatches of the sweep kernel in each pass (start
order) -- bench.py's kernel leg when the run also has later legs.

Inputs: the three separate passes (FETCH_SIZE; WRITE_SIZE; SQ_WAVES,
SQ_INSTS_VALU, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE), each
`rocprofv3 --pmc ... --kernel-trace --output-format csv` of
`bench.py --steps 5 --warmup 1 --no-cpu --no-extra`.  HBM bytes per launch =
2 x FETCH_SIZE + WRITE_SIZE (KB): on gfx950 FETCH_SIZE counts 128-B requests
at 64 B (MI355X_MICROARCH.md, HBM / rocprofv3 section).  The algorithmic bytes
are the compulsory per-chain traffic of one sweep: u read (d·s B), Φ and
the accept counter read and written (2·(s + 8) B); the u write-back of
accepted chains (accept rate x d·s) comes on top and is data dependent.
"""
import csv
import glob
import json
import os
import sys

from collections import defaultdict


def rows(path):
    with open(path) as f:
        yield from csv.DictReader(f)


def per_dispatch(files, match, first=None):
    """{counter: [value per dispatch]} for kernels whose name contains `match`
    (the first `first` dispatches of each file in start order, if given)."""
    acc = defaultdict(lambda: defaultdict(float))
    meta = {}
    for path in files:
        rs = [r for r in rows(path) if match in r["Kernel_Name"]]
        keep = None
        if first:
            starts = sorted({(int(r["Start_Timestamp"]), r["Dispatch_Id"]) for r in rs})
            keep = {d for _, d in starts[:first]}
        for r in rs:
            if keep is not None and r["Dispatch_Id"] not in keep:
                continue
            key = (path, r["Dispatch_Id"])
            acc[r["Counter_Name"]][key] += float(r["Counter_Value"])
            meta[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"])
    return {c: list(v.values()) for c, v in acc.items()}, meta


def main():
    src, dtype, chains, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    first = int(sys.argv[5]) if len(sys.argv) > 5 else None
    files = sorted(glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True))
    vals, meta = per_dispatch(files, "l96_sweep", first)
    mean = lambda xs: sum(xs) / len(xs)
    d, k_bytes = 40, 8 if dtype == "f64" else 4
    fetch, write = mean(vals["FETCH_SIZE"]), mean(vals["WRITE_SIZE"])
    ns = mean([t for t, _ in meta.values()])
    rec = {
        "kernel": sorted({n for _, n in meta.values()}),
        "dtype": dtype,
        "chains": chains,
        "d": d,
        "rk4_steps": 2000,
        "launches_averaged": len(vals["FETCH_SIZE"]),
        "FETCH_SIZE_KB": fetch,
        "WRITE_SIZE_KB": write,
        "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
        "correction": "FETCH_SIZE x2 (gfx950 counts 128-B requests at 64 B, MI355X_MICROARCH.md HBM), "
                      "WRITE_SIZE as read",
        "algorithmic_bytes_per_launch": chains * (d * k_bytes + 2 * (k_bytes + 8)),
        "kernel_ns_profiled": ns,
    }
    for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
        if c in vals:
            rec[c] = mean(vals[c])
    if "GRBM_GUI_ACTIVE" in rec:
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs
        rec["effective_clock_GHz"] = rec["GRBM_GUI_ACTIVE"] / 8 / ns
    if "SQ_INSTS_VALU" in rec and "SQ_WAVES" in rec:
        rec["valu_instr_per_wave"] = rec["SQ_INSTS_VALU"] / rec["SQ_WAVES"]
    if "SQ_INSTS_VALU" in rec and "effective_clock_GHz" in rec:
        # VALU instructions issued per SIMD per cycle over the kernel (1 024
        # SIMDs): a wave64 FP64 (or packed FP32) op holds its 16-lane SIMD for
        # 4 cycles, so 0.25 is the FP64 / packed-FP32 pipe issuing every slot
        cycles = rec["effective_clock_GHz"] * ns
        rec["valu_issue_per_simd_cycle"] = rec["SQ_INSTS_VALU"] / (1024 * cycles)
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
