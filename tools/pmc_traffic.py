"""Per-launch HBM traffic of the bench's timed hmc_kernel launch from the
rocprofv3 PMC passes of tools/profile_bench.sh.

FETCH_SIZE and WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced read (MI355X_MICROARCH.md, HBM section), so it is
doubled. The bench's second hmc_kernel dispatch is the timed launch (the first
is the warm-up).

    python tools/pmc_traffic.py gpurun_out/prof_r01 [--key C4096_D64_L50_K100_f32] [--write]
"""
import argparse
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter_rows(d, name):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == name and "hmc_kernel" in r["Kernel_Name"]:
                    rows.append(r)
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--key", default="C4096_D64_L50_K100_f32")
    ap.add_argument("--write", action="store_true", help="update profiles/r01/pmc_traffic.json")
    a = ap.parse_args()
    fetch = counter_rows(os.path.join(a.prof_dir, "fetch"), "FETCH_SIZE")
    write = counter_rows(os.path.join(a.prof_dir, "write"), "WRITE_SIZE")
    if not fetch or not write:
        raise SystemExit("no hmc_kernel PMC rows found")
    # counters of one dispatch may be split over rows (one per XCD / dimension): sum per dispatch
    def per_dispatch(rows):
        acc = {}
        for r in rows:
            acc[int(r["Dispatch_Id"])] = acc.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
        return [acc[k] for k in sorted(acc)]
    # the bench's second hmc_kernel dispatch is its timed launch (the first is
    # the warm-up; later ones, the host-output run, have the same shape)
    f_kb = per_dispatch(fetch)[1]
    w_kb = per_dispatch(write)[1]
    entry = {
        "hbm_bytes_per_launch": (2 * f_kb + w_kb) * 1024.0,
        "fetch_size_kb": f_kb,
        "write_size_kb": w_kb,
        "correction": "FETCH_SIZE x2 (gfx950 counts half of a wide coalesced read), KB = 1024 B",
        "source": f"{a.prof_dir} (rocprofv3 --pmc, timed launch = second hmc_kernel dispatch)",
    }
    print(json.dumps({a.key: entry}, indent=1))
    if a.write:
        p = os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json")
        d = json.load(open(p)) if os.path.exists(p) else {}
        d[a.key] = entry
        json.dump(d, open(p, "w"), indent=1)


if __name__ == "__main__":
    main()
