"""Condense a gpu_round.sh output directory into profiles/<tag>/ (committed evidence).

Writes: kernel_stats.csv (rocprofv3 --stats of the bench run), pmc_summary.json (per-kernel
mean FETCH_SIZE / WRITE_SIZE per dispatch, with the gfx950 FETCH_SIZE x2 correction), the
bench JSON line, and profiles/pmc_btp_stage.json (read by bench.py for roofline.traffic).
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join("gpurun_out", tag)
dst = os.path.join("profiles", tag)
os.makedirs(dst, exist_ok=True)
stats = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)
shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
for f in ("bench.json", "pytest_gpu.log"):
    if os.path.exists(os.path.join(src, f)):
        shutil.copy(os.path.join(src, f), os.path.join(dst, f))


def pmc(sub, counter):
    per = {}
    for f in glob.glob(os.path.join(src, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0]
            per.setdefault(name, []).append(float(r["Counter_Value"]))
    return {k: statistics.mean(v) for k, v in per.items()}


fetch, write = pmc("pmc_fetch", "FETCH_SIZE"), pmc("pmc_write", "WRITE_SIZE")
summary = {}
for k in sorted(set(fetch) | set(write)):
    f_kb, w_kb = fetch.get(k, 0.0), write.get(k, 0.0)
    summary[k] = {"FETCH_SIZE_kB": f_kb, "WRITE_SIZE_kB": w_kb,
                  "hbm_bytes_per_dispatch": (2.0 * f_kb + w_kb) * 1024.0}
json.dump({"note": "FETCH_SIZE doubled for gfx950 (MI355X_MICROARCH.md, HBM section); kB = 1024 B",
           "kernels": summary}, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
stage = [k for k in summary if "btp_stage_kernel" in k]
if stage:
    b = summary[stage[0]]["hbm_bytes_per_dispatch"]
    json.dump({"config": "dg25L3", "kernel": stage[0], "hbm_bytes_per_launch": round(b), "source": dst},
              open(os.path.join("profiles", "pmc_btp_stage.json"), "w"), indent=1)
    print("stage kernel HBM bytes/launch", b)
print("wrote", dst)
