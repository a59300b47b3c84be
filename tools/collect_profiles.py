"""Copy one measurement pass of tools/gpu_round4.sh (gpurun_out/<tag>/) into profiles/<name>_*:
bench lines, rocprofv3 kernel-trace summaries and the PMC summaries of the forward and
training kernels (tools/pmc_summary.py), each PMC file headed by the profiled source sha.

usage: python tools/collect_profiles.py <tag> <name> <label>
"""
import os
import shutil
import subprocess
import sys

tag, name, label = sys.argv[1], sys.argv[2], sys.argv[3]
src = os.path.join("gpurun_out", tag)
sha = open(os.path.join(src, "source_sha16.txt")).read().strip()
for f in ("bench_driver", "bench", "cfg1", "cfg1_4096", "cfg4", "nll", "train_cfg2", "train_cfg5"):
    p = os.path.join(src, f + ".json")
    if os.path.exists(p):
        shutil.copy(p, os.path.join("profiles", f"{name}_{f}.json"))
for d, out in (("prof_driver", "driver_cmd_kernel_stats"), ("prof", "kernel_stats"), ("prof_cfg4", "cfg4_kernel_stats"),
               ("prof_t2", "train_cfg2_kernel_stats"), ("prof_t5", "train_cfg5_kernel_stats")):
    p = os.path.join(src, d, "run_kernel_stats.csv")
    if os.path.exists(p):
        shutil.copy(p, os.path.join("profiles", f"{name}_{out}.csv"))
if os.path.exists(os.path.join(src, "pytest_gpu.log")):
    lines = open(os.path.join(src, "pytest_gpu.log")).read().splitlines()
    keep = [l for l in lines if " PASSED" in l or " FAILED" in l or " ERROR" in l or " SKIPPED" in l or "passed" in l]
    with open(os.path.join("profiles", f"{name}_pytest_gpu_summary.txt"), "w") as fo:
        fo.write(f"# pytest -m gpu, {label}, source sha16 {sha}\n" + "\n".join(keep) + "\n")
if os.path.exists(os.path.join(src, "smoke.log")):
    shutil.copy(os.path.join(src, "smoke.log"), os.path.join("profiles", f"{name}_smoke.txt"))

PMC = [
    ("pmc_cfg2", "cfg2 forward, FAST SPLIT kernel", [("uniform_kernel<4, 0", None)]),
    ("pmc_cfg4", "cfg4 forward, wide SPLIT kernel", [("wide_kernel<0", None)]),
    ("pmct_cfg2", "config-2 train step (bench --mode train)",
     [("train_net_kernel<4, 1, 1, true, 3>", "train_net_kernel<4, 1, 1, true, 3> (3-output nets)"),
      ("train_net_kernel<4, 1, 1, true, 2>", "train_net_kernel<4, 1, 1, true, 2> (2-output nets)"),
      ("uniform_kernel<4, 3", "uniform_kernel<4, 3, true, true, true, true>")]),
    ("pmct_cfg4", "config-5 train step (bench --mode train --config cfg4)",
     [("sweep_kernel<16, 1>", "sweep_kernel<16, 1>"), ("wide_kernel<3, true>", "wide_kernel<3, true>"),
      ("ldense_kernel<16, 0, 5, true,", "ldense_kernel<16, 0, 5, true, 8, 2>"),
      ("ldw_split_kernel", "ldw_split_kernel<true>")]),
]
OUT = {"pmc_cfg2": "pmc_cfg2", "pmc_cfg4": "pmc_cfg4", "pmct_cfg2": "pmc_train_cfg2", "pmct_cfg4": "pmc_train_cfg5"}
for d, what, kernels in PMC:
    if not os.path.isdir(os.path.join(src, d)):
        continue
    text = [f"# rocprofv3 PMC passes (tools/pmc_sets.txt, one counter set per run), {what}, {label} "
            f"(tools/gpu_round4.sh)", f"# source sha16 {sha}"]
    for sub, head in kernels:
        r = subprocess.run([sys.executable, "tools/pmc_summary.py", f"{tag}/{d}", sub],
                           capture_output=True, text=True, check=True)
        if head:
            text.append(f"## {head}")
        text.append(r.stdout.rstrip())
    with open(os.path.join("profiles", f"{name}_{OUT[d]}.txt"), "w") as fo:
        fo.write("\n".join(text) + "\n")
print("source", sha)
