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
# dominant kernel: the persistent sub-cycle kernel (one launch = N_btp*kstages stages) or the
# per-stage kernel; roofline.traffic is per stage, like roofline.achieved
bj = json.load(open(os.path.join(dst, "bench.json"))) if os.path.exists(os.path.join(dst, "bench.json")) else {}
cfgname = bj.get("config", {}).get("workload", "dg25L3:").split(":")[0] or "dg25L3"
spl = int(sys.argv[2]) if len(sys.argv) > 2 else 100   # stages per sub-cycle launch (dg25L3: 20 x 5)
for short, per in (("btp_subcycle_kernel", spl), ("btp_stage_kernel", 1)):
    ks = [k for k in summary if short in k]
    if ks:
        b = summary[ks[0]]["hbm_bytes_per_dispatch"] / per
        json.dump({"config": cfgname, "kernel": short, "hbm_bytes_per_launch": round(b),
                   "note": f"per barotropic stage ({per} stage(s) per dispatch of {ks[0]})", "source": dst},
                  open(os.path.join("profiles", "pmc_btp_stage.json"), "w"), indent=1)
        print(short, "HBM bytes per stage", b)
        break
print("wrote", dst)
