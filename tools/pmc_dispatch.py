"""PMC figures of one kernel dispatch from rocprofv3 passes of the same
command, one run per pass, each pass in its own directory under PROF_DIR:

  trace/  --kernel-trace --stats      (launch duration)
  fetch/  --pmc FETCH_SIZE            (KiB; gfx950 counts half the bytes of a
                                       wide coalesced read: doubled,
                                       MI355X_MICROARCH.md HBM section)
  write/  --pmc WRITE_SIZE            (KiB)
  sq/     --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES
                SQ_ACTIVE_INST_VALU SQ_WAIT_ANY
  grbm/   --pmc GRBM_GUI_ACTIVE       (GPU busy cycles, summed over 8 XCDs)

  flops/  --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 (optional)

The dispatch is selected by kernel name AND grid size (threads), then by its
ordinal among the dispatches that match both. The bench's timed launch is
the 4th from the END of the bench's grid (tools/profile_r03.sh runs bench.py
with --ess-long-discard 0 --no-north-star --cpu-seconds 0): the cfg2 ESS leg
and the two host-output launches follow it, while the time-based scratch
warm-up puts a varying number of launches before it. Other kernels of the
same name (the cfg4 leg, the north-star shape) have other grids, so they
never shift the ordinal.

    python tools/pmc_dispatch.py PROF_DIR --kernel hmc_kernel --grid 262144 \
        --ordinal -4 --key C4096_D64_L50_f32 --steps 20 --out profiles/r03/pmc_hmc.json
"""
import argparse
import collections
import csv
import glob
import json
import os

import numpy as np


def _rows(d, pattern):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True)):
        out += list(csv.DictReader(open(f)))
    return out


def pick_dispatch(rows, kernel, grid, ordinal, grid_key):
    ids = sorted({int(r["Dispatch_Id"]) for r in rows
                  if kernel in r["Kernel_Name"] and int(float(r[grid_key])) == grid})
    if not ids:
        raise SystemExit(f"no {kernel} dispatch with grid {grid}")
    return ids[ordinal]


def counters(d, kernel, grid, ordinal):
    rows = _rows(d, "*counter_collection.csv")
    did = pick_dispatch(rows, kernel, grid, ordinal, "Grid_Size")
    acc = collections.defaultdict(float)
    meta = {}
    for r in rows:
        if int(r["Dispatch_Id"]) == did:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
            meta = {"vgpr_count_column": int(r["VGPR_Count"]), "accum_vgpr_count_column": int(r["Accum_VGPR_Count"]),
                    "sgpr_count_column": int(r["SGPR_Count"]), "lds_block_size": int(r["LDS_Block_Size"]),
                    "scratch_size": int(r["Scratch_Size"]), "kernel_name": r["Kernel_Name"],
                    # rocprofv3's VGPR_Count is the kernel descriptor's granule count x 4; gfx950
                    # allocates (arch + accumulation) registers in granules of 8, so the registers a
                    # lane holds are twice the column (checked against the compiler's NumVgprs +
                    # NumAgprs: 106 -> 56 MH cfg5, 238 -> 120 NUTS cfg3, 256 + 176 -> 216 dense NUTS)
                    "vgpr_total_per_lane": 2 * int(r["VGPR_Count"])}
    return acc, meta


def duration(d, kernel, grid, ordinal):
    rows = _rows(d, "*kernel_trace.csv")
    did = pick_dispatch(rows, kernel, grid, ordinal, "Grid_Size_X")
    r = [r for r in rows if int(r["Dispatch_Id"]) == did][0]
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9


def measure(prof_dir, kernel, grid, ordinal, simds=1024):
    dur = duration(os.path.join(prof_dir, "trace"), kernel, grid, ordinal)
    f, meta = counters(os.path.join(prof_dir, "fetch"), kernel, grid, ordinal)
    w, _ = counters(os.path.join(prof_dir, "write"), kernel, grid, ordinal)
    sq, _ = counters(os.path.join(prof_dir, "sq"), kernel, grid, ordinal)
    grbm, _ = counters(os.path.join(prof_dir, "grbm"), kernel, grid, ordinal)
    cycles = grbm["GRBM_GUI_ACTIVE"] / 8.0
    waves = max(sq["SQ_WAVES"], 1)
    flops = None
    fdir = os.path.join(prof_dir, "flops")
    if os.path.isdir(fdir):
        fl, _ = counters(fdir, kernel, grid, ordinal)
        # SQ_INSTS_VALU_FLOPS_* count per wave instruction (the lanes' flops
        # / 64): x 64 gives lane flops, comparable with F_alg
        flops = {"fp32_lane_flops": 64.0 * fl.get("SQ_INSTS_VALU_FLOPS_FP32", 0.0),
                 "fp64_lane_flops": 64.0 * fl.get("SQ_INSTS_VALU_FLOPS_FP64", 0.0),
                 "note": "SQ_INSTS_VALU_FLOPS_FP32/FP64 x 64 (the counter's unit is per wave instruction, "
                         "1/64 of the lanes' flops)"}
    return {
        "kernel": meta.get("kernel_name"), "grid_threads": grid, "ordinal": ordinal,
        "launch_us_traced": dur * 1e6,
        "hbm_bytes_per_launch": (2 * f["FETCH_SIZE"] + w["WRITE_SIZE"]) * 1024.0,
        "fetch_size_kb": f["FETCH_SIZE"], "write_size_kb": w["WRITE_SIZE"],
        "valu": {
            "issue_frac": 2.0 * sq["SQ_INSTS_VALU"] / (simds * cycles),
            "valu_insts_per_wave": sq["SQ_INSTS_VALU"] / waves,
            "salu_insts_per_wave": sq["SQ_INSTS_SALU"] / waves if "SQ_INSTS_SALU" in sq else None,
            "wave_valu_active_frac": sq["SQ_ACTIVE_INST_VALU"] / max(sq["SQ_WAVE_CYCLES"], 1),
            "wave_wait_frac": sq["SQ_WAIT_ANY"] / max(sq["SQ_WAVE_CYCLES"], 1),
            "wave_issue_stall_frac": (sq["SQ_WAIT_INST_ANY"] / max(sq["SQ_WAVE_CYCLES"], 1)
                                      if "SQ_WAIT_INST_ANY" in sq else None),
            "lds_insts_per_wave": sq["SQ_INSTS_LDS"] / waves if "SQ_INSTS_LDS" in sq else None,
            "salu_per_valu": (sq["SQ_INSTS_SALU"] / max(sq["SQ_INSTS_VALU"], 1)) if "SQ_INSTS_SALU" in sq else None,
            "waves": waves, "clock_ghz": cycles / dur / 1e9,
            "note": "issue_frac = SQ_INSTS_VALU x 2 cycles (wave64 on a SIMD-32) / (1024 SIMDs x "
                    "GRBM_GUI_ACTIVE/8); per-wave counts are SQ_INSTS_* / SQ_WAVES",
        },
        "registers": meta,
        "pmc_flops": flops,
        "correction": "HBM bytes = FETCH_SIZE x 2 (gfx950 half count) + WRITE_SIZE, KB = 1024 B",
        "source": f"{prof_dir}: trace, fetch, write, sq, grbm passes (rocprofv3, one run each); "
                  f"{kernel} dispatch #{ordinal} of grid {grid}",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--kernel", default="hmc_kernel")
    ap.add_argument("--grid", type=int, required=True, help="Grid_Size in threads")
    ap.add_argument("--ordinal", type=int, default=-4)
    ap.add_argument("--key", required=True)
    ap.add_argument("--steps", type=int, default=0, help="transitions of the launch (HMC fit)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    entry = measure(a.prof_dir, a.kernel, a.grid, a.ordinal)
    d = json.load(open(a.out)) if os.path.exists(a.out) else {}
    e = d.setdefault(a.key, {"by_steps": {}})
    e["by_steps"][str(a.steps)] = entry
    ks = sorted(int(k) for k in e["by_steps"])
    if len(ks) >= 2:
        y = [e["by_steps"][str(k)]["hbm_bytes_per_launch"] for k in ks]
        slope, icpt = np.polyfit(np.array(ks, float), np.array(y), 1)
        e["fit"] = {"fixed_bytes": float(icpt), "bytes_per_transition": float(slope),
                    "source": f"least-squares line through by_steps K = {ks}"}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(d, open(a.out, "w"), indent=1)
    print(json.dumps({a.key: {str(a.steps): entry}}, indent=1))


if __name__ == "__main__":
    main()
