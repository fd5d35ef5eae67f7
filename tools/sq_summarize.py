"""Per-kernel summary of one rocprofv3 SQ counter pass (stall breakdown).

  python tools/sq_summarize.py <dir with *counter_collection.csv> <kernel substring> [cycles_per_valu]

Counters (one pass): SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE.
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed over
waves (MI355X_MICROARCH.md, rocprofv3 section), so their ratios are fractions
of wave lifetime: active VALU, issue-stalled (dependency / pipe busy) and
parked (s_waitcnt / barrier).  VALU issue utilisation per SIMD =
SQ_INSTS_VALU x cycles per wave64 VALU instruction (4 for FP64 and packed
FP32) / (1024 SIMDs x kernel cycles at the GRBM clock).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    src, match = sys.argv[1], sys.argv[2]
    cpi = float(sys.argv[3]) if len(sys.argv) > 3 else 4.0
    acc = defaultdict(lambda: defaultdict(float))
    dur = {}
    names = set()
    for path in sorted(glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True)):
        with open(path) as f:
            for r in csv.DictReader(f):
                if match not in r["Kernel_Name"]:
                    continue
                key = (path, r["Dispatch_Id"])
                acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
                dur[key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                names.add(r["Kernel_Name"])
    if not acc:
        raise SystemExit(f"no dispatch of a kernel matching {match!r} in {src}")
    keys = list(acc)
    mean = lambda c: sum(acc[k][c] for k in keys) / len(keys)
    ns = sum(dur[k] for k in keys) / len(keys)
    rec = {"kernels": sorted(names), "dispatches": len(keys), "kernel_ns": ns}
    for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
              "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"):
        rec[c] = mean(c)
    wc = rec["SQ_WAVE_CYCLES"]
    rec["frac_active_valu"] = rec["SQ_ACTIVE_INST_VALU"] / wc
    rec["frac_wait_inst"] = rec["SQ_WAIT_INST_ANY"] / wc
    rec["frac_wait_any"] = rec["SQ_WAIT_ANY"] / wc
    clock_ghz = rec["GRBM_GUI_ACTIVE"] / 8 / ns  # GRBM_GUI_ACTIVE summed over the 8 XCDs
    rec["effective_clock_GHz"] = clock_ghz
    rec["valu_instr_per_wave"] = rec["SQ_INSTS_VALU"] / rec["SQ_WAVES"]
    rec["valu_issue_utilisation"] = rec["SQ_INSTS_VALU"] * cpi / (1024 * ns * clock_ghz)
    # the same from the activity counter, no per-instruction cost assumed:
    # VALU-active quad-cycles summed over waves / (SIMDs x kernel cycles)
    rec["valu_busy_from_active_cycles"] = rec["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * ns * clock_ghz)
    rec["cycles_per_valu_assumed"] = cpi
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
