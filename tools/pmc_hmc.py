"""PMC figures of bench.py's timed hmc_kernel launch, from rocprofv3 passes of
the driver's own command (tools/profile_r02.sh): one run per pass, each pass
in its own directory under PROF_DIR:

  trace/  --kernel-trace --stats      (launch duration)
  fetch/  --pmc FETCH_SIZE            (KiB; gfx950 counts half the bytes of a
                                       wide coalesced read: doubled,
                                       MI355X_MICROARCH.md HBM section)
  write/  --pmc WRITE_SIZE            (KiB)
  sq/     --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY
                SQ_ACTIVE_INST_VALU SQ_WAIT_ANY
  grbm/   --pmc GRBM_GUI_ACTIVE       (GPU busy cycles of the dispatch, summed
                                       over the 8 XCDs)

The timed launch is the bench's FOURTH hmc_kernel dispatch (--index 3: two
device warm-up launches on a scratch sampler and the W-transition warm-up
come first, in either order; --index 1 for profiles taken before the scratch
warm-up existed).
Writes/updates profiles/r02/pmc_hmc.json under the shape key
C{chains}_D{dim}_L{L}_{dtype}, by_steps[K]; with two or more K profiled, also
a linear fit bytes = fixed + K x per-transition, which bench.py uses for a K
that was not profiled (marked scaled).

    python tools/pmc_hmc.py PROF_DIR --steps 20 [--key C4096_D64_L50_f32]
"""
import argparse
import collections
import csv
import glob
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "profiles", "r02", "pmc_hmc.json")


def dispatch_counters(d, kernel="hmc_kernel", index=1):
    acc = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"]]
        if not rows:
            continue
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})
        for r in rows:
            if int(r["Dispatch_Id"]) == ids[index]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    return acc


def launch_seconds(d, kernel="hmc_kernel", index=1):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    r = rows[index]
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--key", default="C4096_D64_L50_f32")
    ap.add_argument("--simds", type=int, default=1024)
    ap.add_argument("--index", type=int, default=3, help="the timed launch's index among hmc_kernel dispatches")
    a = ap.parse_args()
    ix = a.index
    dur = launch_seconds(os.path.join(a.prof_dir, "trace"), index=ix)
    f_kb = dispatch_counters(os.path.join(a.prof_dir, "fetch"), index=ix)["FETCH_SIZE"]
    w_kb = dispatch_counters(os.path.join(a.prof_dir, "write"), index=ix)["WRITE_SIZE"]
    sq = dispatch_counters(os.path.join(a.prof_dir, "sq"), index=ix)
    grbm = dispatch_counters(os.path.join(a.prof_dir, "grbm"), index=ix)
    cycles = grbm["GRBM_GUI_ACTIVE"] / 8.0
    fdir = os.path.join(a.prof_dir, "flops")
    fl = dispatch_counters(fdir, index=ix) if os.path.isdir(fdir) else {}
    entry = {
        "hbm_bytes_per_launch": (2 * f_kb + w_kb) * 1024.0,
        "fetch_size_kb": f_kb, "write_size_kb": w_kb,
        "launch_us_traced": dur * 1e6,
        "valu": {
            "issue_frac": 2.0 * sq["SQ_INSTS_VALU"] / (a.simds * cycles),
            "issue_frac_at_2p4ghz": 2.0 * sq["SQ_INSTS_VALU"] / (a.simds * 2.4e9 * dur),
            "valu_insts_per_wave": sq["SQ_INSTS_VALU"] / max(sq["SQ_WAVES"], 1),
            "wave_valu_active_frac": sq["SQ_ACTIVE_INST_VALU"] / max(sq["SQ_WAVE_CYCLES"], 1),
            "wave_wait_frac": sq["SQ_WAIT_ANY"] / max(sq["SQ_WAVE_CYCLES"], 1),
            "clock_ghz": cycles / dur / 1e9,
            "note": "SQ_INSTS_VALU x 2 cycles (wave64 on a SIMD-32) / (1024 SIMDs x GRBM_GUI_ACTIVE/8)",
        },
        "correction": "HBM bytes = FETCH_SIZE x 2 (gfx950 half count) + WRITE_SIZE, KB = 1024 B",
        "source": f"{a.prof_dir}: trace, fetch, write, sq, grbm passes (rocprofv3, one run each); "
                  f"hmc_kernel dispatch index {ix} (the timed launch)",
    }
    if fl:
        f32 = fl.get("SQ_INSTS_VALU_FLOPS_FP32", 0.0)
        entry["pmc_flops"] = {"fp32_lane_flops": 64 * f32, "fma_f32_insts": fl.get("SQ_INSTS_VALU_FMA_F32"),
                              "fp32_lane_tflops": 64 * f32 / dur / 1e12, "fp32_lane_frac": 64 * f32 / dur / 157.3e12,
                              "note": "SQ_INSTS_VALU_FLOPS_FP32 x 64 (a per-wave-instruction counter) of the launch "
                                      "over its traced duration"}
    d = json.load(open(OUT)) if os.path.exists(OUT) else {}
    e = d.setdefault(a.key, {"by_steps": {}})
    e["by_steps"][str(a.steps)] = entry
    ks = sorted(int(k) for k in e["by_steps"])
    if len(ks) >= 2:
        y = [e["by_steps"][str(k)]["hbm_bytes_per_launch"] for k in ks]
        slope, icpt = np.polyfit(np.array(ks, float), np.array(y), 1)
        e["fit"] = {"fixed_bytes": float(icpt), "bytes_per_transition": float(slope),
                    "source": f"least-squares line through by_steps K = {ks}"}
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    json.dump(d, open(OUT, "w"), indent=1)
    print(json.dumps({a.key: {str(a.steps): entry}}, indent=1))


if __name__ == "__main__":
    main()
