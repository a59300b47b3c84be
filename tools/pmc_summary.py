"""Summarise rocprofv3 PMC passes (gpurun_out/<tag>/p*/run_counter_collection.csv)
for one kernel: mean counter value per dispatch, effective clock, MFMA busy."""
import collections
import csv
import glob
import sys

tag, name = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "kernel")
tot, dur = {}, []
for f in sorted(glob.glob(f"gpurun_out/{tag}/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if name not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    for k, v in agg.items():
        tot[k] = sum(v) / len(v)
for k, v in sorted(tot.items()):
    print(f"{k:28s} {v:,.0f}")
if "GRBM_GUI_ACTIVE" in tot and dur:
    t = sorted(dur)[len(dur) // 2]
    clk = tot["GRBM_GUI_ACTIVE"] / 8 / t
    print(f"median dispatch {t*1e3:.3f} ms, effective clock {clk/1e9:.3f} GHz")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in tot:
        print(f"MFMA busy fraction {tot['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (tot['GRBM_GUI_ACTIVE'] / 8):.3f}")
