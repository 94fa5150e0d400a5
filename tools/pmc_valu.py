"""VALU issue utilisation of the bench's timed hmc_kernel launch from PMC
passes (tools/pmc_sq.sh + a GRBM pass + a kernel trace on the same command):

  issue_frac = SQ_INSTS_VALU * 2 / (1024 SIMDs * cycles)

A wave64 VALU instruction occupies a SIMD-32 for 2 cycles (MI355X_MICROARCH.md,
wave scheduling); cycles = GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs).
Also against the 2.4 GHz nominal clock over the traced duration.

    python tools/pmc_valu.py gpurun_out/hb [--write]
"""
import argparse
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def timed_dispatch(d, name):
    """counters of the bench's timed launch: its second dispatch of `name`
    (the first is the warm-up)"""
    acc = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if name in r["Kernel_Name"]]
        if not rows:
            continue
        last = sorted({int(r["Dispatch_Id"]) for r in rows})[1]
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--key", default="C4096_D64_L50_K100_f32")
    ap.add_argument("--write", action="store_true")
    a = ap.parse_args()
    c = timed_dispatch(a.prof_dir, "hmc_kernel")
    tr = [r for r in csv.DictReader(open(glob.glob(os.path.join(a.prof_dir, "trace", "*kernel_trace.csv"))[0]))
          if "hmc_kernel" in r["Kernel_Name"]]
    dur = (int(tr[1]["End_Timestamp"]) - int(tr[1]["Start_Timestamp"])) * 1e-9  # the timed launch
    cycles = c["GRBM_GUI_ACTIVE"] / 8.0
    simd_cycles = 2.0 * c["SQ_INSTS_VALU"]
    entry = {
        "valu_insts_per_launch": c["SQ_INSTS_VALU"],
        "valu_insts_per_wave": c["SQ_INSTS_VALU"] / c["SQ_WAVES"],
        "clock_ghz": cycles / dur / 1e9,
        "issue_frac": simd_cycles / (1024 * cycles),
        "issue_frac_at_2p4ghz": simd_cycles / (1024 * 2.4e9 * dur),
        "wave_issue_active_frac": c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"],
        "traced_launch_us": dur * 1e6,
        "source": f"{a.prof_dir}: SQ_INSTS_VALU, SQ_WAVES, SQ_ACTIVE_INST_ANY, SQ_WAVE_CYCLES (pmc_sq.sh), "
                  "GRBM_GUI_ACTIVE (own pass), kernel trace (own pass); second (timed) hmc_kernel dispatch",
    }
    print(json.dumps({a.key: entry}, indent=1))
    if a.write:
        p = os.path.join(ROOT, "profiles", "r01", "pmc_valu.json")
        d = json.load(open(p)) if os.path.exists(p) else {}
        d[a.key] = entry
        json.dump(d, open(p, "w"), indent=1)


if __name__ == "__main__":
    main()
