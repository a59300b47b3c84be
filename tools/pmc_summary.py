"""Summarise rocprofv3 PMC passes (gpurun_out/<tag>/<prefix>p*/run_counter_collection.csv)
for one kernel: mean counter value per dispatch, effective clock, MFMA busy,
HBM traffic per dispatch with the gfx950 FETCH_SIZE correction
(MI355X_MICROARCH.md §HBM: bytes = (2·FETCH_SIZE + WRITE_SIZE) KiB).

usage: python tools/pmc_summary.py <tag> <kernel-substring> [<pass-dir prefix>]
"""
import collections
import csv
import glob
import sys

tag, name = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "kernel")
prefix = sys.argv[3] if len(sys.argv) > 3 else ""
tot, dur = {}, []
for f in sorted(glob.glob(f"gpurun_out/{tag}/{prefix}p*/run_counter_collection.csv")):
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
if dur:
    t = sorted(dur)[len(dur) // 2]
    print(f"median dispatch {t*1e3:.3f} ms")
    if "GRBM_GUI_ACTIVE" in tot:
        clk = tot["GRBM_GUI_ACTIVE"] / 8 / t
        print(f"effective clock {clk/1e9:.3f} GHz")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in tot:
            print(f"MFMA busy fraction {tot['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (tot['GRBM_GUI_ACTIVE'] / 8):.3f}")
    if "SQ_WAVE_CYCLES" in tot:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if k in tot:
                print(f"{k} / SQ_WAVE_CYCLES {tot[k] / tot['SQ_WAVE_CYCLES']:.3f}")
    if "SQ_VALU_MFMA_COEXEC_CYCLES" in tot and "SQ_VALU_MFMA_BUSY_CYCLES" in tot:
        print(f"VALU co-executing with MFMA / MFMA busy cycles "
              f"{tot['SQ_VALU_MFMA_COEXEC_CYCLES'] / tot['SQ_VALU_MFMA_BUSY_CYCLES']:.3f}")
    if "SQ_LDS_BANK_CONFLICT" in tot and tot.get("SQ_INSTS_LDS"):
        print(f"LDS bank-conflict cycles per LDS instruction {tot['SQ_LDS_BANK_CONFLICT'] / tot['SQ_INSTS_LDS']:.3f}")
    if "FETCH_SIZE" in tot and "WRITE_SIZE" in tot:
        b = (2.0 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024.0
        print(f"HBM traffic per dispatch {b/1e6:.2f} MB ((2*FETCH_SIZE + WRITE_SIZE) KiB)")
