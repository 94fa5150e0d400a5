"""Per-kernel register / scratch / spill table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks.

    hipcc ... -c csrc/nuts_part0.hip -Rpass-analysis=kernel-resource-usage 2> r0.txt
    python3 tools/kernel_resources.py r0.txt [r1.txt ...] [--filter nuts_kernel] [--json out.json]

ScratchSize includes the call frame of out-of-line device functions (the
NUTS step-size search is noinline), so a kernel can show scratch without a
register spill; "VGPRs Spill" is the spill count.
"""
from __future__ import annotations

import argparse
import json
import re
import subprocess

KEYS = {"TotalSGPRs": "sgprs", "VGPRs": "vgprs", "AGPRs": "agprs", "ScratchSize [bytes/lane]": "scratch",
        "Occupancy [waves/SIMD]": "occupancy", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill",
        "LDS Size [bytes/block]": "lds"}


def parse(paths, filt=""):
    rows, cur = [], None
    for path in paths:
        for line in open(path, errors="replace"):
            m = re.search(r"remark: Function Name: (\S+)", line)
            if m:
                cur = {"mangled": m.group(1)}
                rows.append(cur)
                continue
            m = re.search(r"remark:\s+(.+?): (\S+) \[-Rpass", line)
            if m and cur is not None and m.group(1) in KEYS:
                v = m.group(2)
                cur[KEYS[m.group(1)]] = int(v) if v.isdigit() else v
    names = subprocess.run(["c++filt"], input="\n".join(r["mangled"] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    for r, n in zip(rows, names):
        r["name"] = n.replace("gm::", "").replace("(anonymous namespace)::", "")
    return [r for r in rows if filt in r["name"]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--filter", default="")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    rows = parse(a.files, a.filter)
    for r in rows:
        n = re.sub(r"\(.*\)$", "", r["name"])
        print(f"{n[:78]:78s} v{r.get('vgprs', '?'):>4} a{r.get('agprs', '?'):>4} "
              f"spill{r.get('vgpr_spill', '?'):>4} scr{r.get('scratch', '?'):>5} occ{r.get('occupancy', '?')}")
    if a.json:
        json.dump(rows, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
