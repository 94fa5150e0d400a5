"""Rooflines of the non-headline kernels from rocprofv3 passes
(tools/profile_kernels.sh): for each workload directory PROF/<w>/{trace,
fetch,write,sq,grbm}, the chosen dispatch's duration, HBM bytes (FETCH_SIZE x 2,
the gfx950 correction, + WRITE_SIZE; KB = 1024 B), VALU issue (SQ_INSTS_VALU x
2 cycles over 1024 SIMDs x GRBM_GUI_ACTIVE / 8) and the fraction of the
kernel's own bound, from the algorithmic work per unit:

  cfg3 nuts_kernel<f64,16,2,Gauss>      F = 2D^2 + 8D flop per leapfrog (D = 32),
                                        vs the 78.6 TF FP64 vector peak; the
                                        leapfrog count of the sampling launch
                                        comes from the trace run's own output
  cfg4 hmc_kernel<f32,64,2,Rosenbrock>  F = 15(D-1) + 6D per chain-leapfrog
                                        (D = 128, 8192 chains, L = 50, 100
                                        transitions), vs 157.3 TF FP32
  cfg5 mh_kernel<f64,64,4,IsoGauss>     VALU (Philox + Box-Muller per
                                        coordinate): the PMC issue fraction;
                                        B = (2D+2) x 8 per chain-step reported
                                        as an HBM-equivalent beside it
  hbm  leapfrog_hbm_kernel, 2^20 chains B = (6D+1) x 4 per chain-leapfrog vs
                                        8 TB/s, and the PMC bytes against B

    python tools/pmc_kernels.py gpurun_out/prof_kernels
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "profiles", "r02", "kernels_pmc.json")
FP32, FP64, HBM = 157.3e12, 78.6e12, 8000e9

# workload -> (kernel, dispatch index among that kernel's dispatches)
PICK = {"cfg3": ("nuts_kernel", -1), "cfg4": ("hmc_kernel", 1), "cfg5": ("mh_kernel", 1),
        "hbm": ("leapfrog_hbm_kernel", 4)}


def _match(name, kernel):
    return re.search(r"(^|[^a-z_])" + kernel + r"\b", name) is not None


def counters(d, kernel, index):
    acc = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if _match(r["Kernel_Name"], kernel)]
        if not rows:
            continue
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})
        for r in rows:
            if int(r["Dispatch_Id"]) == ids[index]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    return acc


def trace(d, kernel, index):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted((r for r in csv.DictReader(open(f)) if _match(r["Kernel_Name"], kernel)),
                  key=lambda r: int(r["Start_Timestamp"]))
    r = rows[index]
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9, r["Kernel_Name"][:160], len(rows)


def json_line(log, key):
    try:
        for line in open(log):
            if line.startswith("{") and key in line:
                return json.loads(line)
    except OSError:
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    a = ap.parse_args()
    logs = os.path.join(os.path.dirname(a.prof_dir.rstrip("/")))
    d = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for w, (kernel, idx) in PICK.items():
        base = os.path.join(a.prof_dir, w)
        if not os.path.isdir(os.path.join(base, "trace")):
            continue
        dur, name, ndisp = trace(os.path.join(base, "trace"), kernel, idx)
        fk = counters(os.path.join(base, "fetch"), kernel, idx).get("FETCH_SIZE", 0.0)
        wk = counters(os.path.join(base, "write"), kernel, idx).get("WRITE_SIZE", 0.0)
        sq = counters(os.path.join(base, "sq"), kernel, idx)
        cyc = counters(os.path.join(base, "grbm"), kernel, idx).get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        fl = counters(os.path.join(base, "flops"), kernel, idx) if os.path.isdir(os.path.join(base, "flops")) else {}
        hbm_bytes = (2 * fk + wk) * 1024.0
        e = {"kernel": name, "dispatch": f"{idx} of {ndisp} {kernel} dispatches", "launch_us": dur * 1e6,
             "hbm_bytes": hbm_bytes, "hbm_gbs": hbm_bytes / dur / 1e9,
             "valu_issue_frac": 2.0 * sq["SQ_INSTS_VALU"] / (1024 * cyc) if cyc else None,
             "valu_insts_per_wave": sq["SQ_INSTS_VALU"] / max(sq["SQ_WAVES"], 1),
             "salu_insts_per_wave": sq["SQ_INSTS_SALU"] / max(sq["SQ_WAVES"], 1),
             "lds_insts_per_wave": sq["SQ_INSTS_LDS"] / max(sq["SQ_WAVES"], 1),
             "wave_wait_frac": sq["SQ_WAIT_ANY"] / max(sq["SQ_WAVE_CYCLES"], 1),
             "waves": sq["SQ_WAVES"], "clock_ghz": cyc / dur / 1e9 if dur else None,
             "source": f"{base}: trace, fetch, write, sq, grbm, flops passes (rocprofv3, one run each)"}
        if fl:
            f32, f64 = fl.get("SQ_INSTS_VALU_FLOPS_FP32", 0.0), fl.get("SQ_INSTS_VALU_FLOPS_FP64", 0.0)
            # the counters count per wave instruction: x 64 gives the lanes' flops
            e["pmc_flops"] = {"fp32_lane_flops": 64 * f32, "fp64_lane_flops": 64 * f64,
                              "fma_f32_insts": fl.get("SQ_INSTS_VALU_FMA_F32"),
                              "fma_f64_insts": fl.get("SQ_INSTS_VALU_FMA_F64"),
                              "fp32_lane_frac": 64 * f32 / dur / FP32, "fp64_lane_frac": 64 * f64 / dur / FP64,
                              "note": "SQ_INSTS_VALU_FLOPS_* x 64 (per-wave-instruction counters); VALU only"}
        if w == "cfg3":
            r = json_line(os.path.join(logs, "cfg3_trace.log"), "cfg3")
            D = 32
            if r:
                f = (2 * D * D + 8 * D) * r["leapfrogs"]
                e.update(bound="valu_f64", leapfrogs=r["leapfrogs"], flops_per_leapfrog=2 * D * D + 8 * D,
                         achieved_tflops=f / dur / 1e12, peak_tflops=FP64 / 1e12, frac=f / dur / FP64,
                         leapfrogs_per_s=r["leapfrogs"] / dur)
        elif w == "cfg4":
            D, C, L, K = 128, 8192, 50, 100
            f = (15 * (D - 1) + 6 * D) * C * L * K
            e.update(bound="valu_f32", flops=f, achieved_tflops=f / dur / 1e12, peak_tflops=FP32 / 1e12,
                     frac=f / dur / FP32, chain_leapfrogs_per_s=C * L * K / dur)
        elif w == "cfg5":
            D, C, K = 256, 16384, 100
            b = (2 * D + 2) * 8 * C * K
            e.update(bound="valu_f64", frac=e["valu_issue_frac"], chain_steps_per_s=C * K / dur,
                     hbm_equivalent={"alg_bytes": b, "gbs": b / dur / 1e9, "frac": b / dur / HBM})
        elif w == "hbm":
            D, C = 64, 1 << 20
            b = (6 * D + 1) * 4 * C
            e.update(bound="hbm", alg_bytes=b, achieved_gbs=b / dur / 1e9, peak_gbs=HBM / 1e9,
                     frac=b / dur / HBM, pmc_over_alg=hbm_bytes / b)
        d[w] = e
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    json.dump(d, open(OUT, "w"), indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
