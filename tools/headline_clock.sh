#!/bin/bash
# The headline launch's shader clock on this box: a kernel-trace pass and a
# GRBM_GUI_ACTIVE pass of the driver's bench command (legs after the timed
# region off), reduced to cycles / duration for the timed hmc_kernel dispatch.
source tools/gpu_check.sh
O=gpurun_out/hclock
ARGS="--steps 20 --warmup 5 --cpu-seconds 0 --cpu-config-seconds 0 --ess-long-discard 0 --no-north-star"
run hclock_trace 200 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 bench.py $ARGS &&
run hclock_grbm 200 timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $O/grbm -o run --output-format csv -- python3 bench.py $ARGS &&
python3 - <<'PY' > gpurun_out/hclock.json
import csv, glob, json
def rows(p):
    out = []
    for f in glob.glob(p, recursive=True):
        out += list(csv.DictReader(open(f)))
    return out
tr = [r for r in rows("gpurun_out/hclock/trace/**/*kernel_trace.csv") if "hmc_kernel" in r["Kernel_Name"] and int(r["Grid_Size_X"] if "Grid_Size_X" in r else r["Grid_Size"]) == 262144]
tr.sort(key=lambda r: int(r["Dispatch_Id"]))
pm = [r for r in rows("gpurun_out/hclock/grbm/**/*counter_collection.csv") if "hmc_kernel" in r["Kernel_Name"] and int(float(r["Grid_Size"])) == 262144]
ids = sorted({int(r["Dispatch_Id"]) for r in pm})
d = tr[-4]
dur = (int(d["End_Timestamp"]) - int(d["Start_Timestamp"])) * 1e-9
cyc = sum(float(r["Counter_Value"]) for r in pm if int(r["Dispatch_Id"]) == ids[-4]) / 8.0
print(json.dumps({"launch_us": dur * 1e6, "grbm_cycles_per_xcd": cyc, "clock_ghz_est": cyc / dur / 1e9,
                  "note": "timed dispatch = 4th from the end of the hmc_kernel grid-262144 dispatches (tools/pmc_dispatch.py); clock = GRBM_GUI_ACTIVE/8 over the traced duration of the same ordinal in the other run"}))
PY
cat gpurun_out/hclock.json
