"""Condense a tools/gpu_profiles.sh output directory into profiles/<tag>/ (committed evidence) and
profiles/roofline_pmc.json (read by bench.py: roofline.traffic and the rocprof kernel duration of
every single-GPU line).

Per config (dg25L3, dg25N7L3, dg316L3, lake200):
  kernel_stats_<cfg>.csv  rocprofv3 --stats of the bench run
  <cfg> entry             dominant stage kernel: mean dispatch duration from the kernel trace
                          (the persistent sub-cycle's stage-less residency trial launch at engine
                          creation excluded: dispatches under 10 % of the median), per-stage
                          duration, HBM bytes per stage from FETCH_SIZE (x2, the gfx950 correction
                          of MI355X_MICROARCH.md) + WRITE_SIZE (kB = 1024 B), and the SQ
                          instruction mix per element-stage (SQ counters are per wave-instruction)

    python tools/profile_summary.py <tag>
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "h-numo_amd"))

from hnumo.roofline import kernel_src_sha16  # noqa: E402

STAGE_KERNELS = ("btp_subcycle_kernel", "btp_stage_kernel")


def _rows(pattern):
    for f in glob.glob(pattern, recursive=True):
        yield from csv.DictReader(open(f))


def _kernel_of(name):
    return next((k for k in STAGE_KERNELS if k in name), None)


def _keep(vals):
    """Drop the stage-less trial launch (and any other dispatch under 10 % of the median)."""
    med = statistics.median(vals)
    return [v for v in vals if v >= 0.1 * med]


def summarize(tag, cfg):
    src = os.path.join(REPO, "gpurun_out", tag)
    dst = os.path.join(REPO, "profiles", tag)
    kt = glob.glob(os.path.join(src, f"kt_{cfg}", "**", "*kernel_stats.csv"), recursive=True)
    if not kt:
        return None
    os.makedirs(dst, exist_ok=True)
    shutil.copy(kt[0], os.path.join(dst, f"kernel_stats_{cfg}.csv"))
    dur = {}
    for r in _rows(os.path.join(src, f"kt_{cfg}", "**", "*kernel_trace.csv")):
        k = _kernel_of(r["Kernel_Name"])
        if k:
            dur.setdefault((k, r["Kernel_Name"].split("(")[0]), []).append(
                int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    (kname, full), d = max(dur.items(), key=lambda kv: sum(kv[1]))
    nall = len(d)
    d = _keep(d)
    from hnumo.case import make_config
    from hnumo.roofline import stage_bytes_cfg
    c = make_config(cfg)
    n_btp = int(round(c["dt"] / c["dt_btp"]))
    per = n_btp * c["kstages"] if kname == "btp_subcycle_kernel" else 1
    out = {"config": cfg, "kernel": kname, "kernel_full": full, "stages_per_dispatch": per,
           "dispatches": len(d), "dispatches_excluded": nall - len(d),
           "dispatch_avg_us": round(statistics.mean(d) / 1e3, 3), "stage_us": round(statistics.mean(d) / 1e3 / per, 4),
           "source": os.path.relpath(dst, REPO), "kernel_src_sha16": kernel_src_sha16()}
    sb = stage_bytes_cfg(c)
    out["algorithmic_bytes_per_stage"] = int(sb)
    out["achieved_GBs"] = round(sb / (out["stage_us"] * 1e-6) / 1e9, 1)
    cnt = {}
    for sub in ("FETCH_SIZE", "WRITE_SIZE", "sq1", "sq2"):
        for r in _rows(os.path.join(src, f"pmc_{sub}_{cfg}", "**", "*counter_collection.csv")):
            if _kernel_of(r["Kernel_Name"]) != kname:
                continue
            cnt.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    if "FETCH_SIZE" in cnt and "WRITE_SIZE" in cnt:
        f, w = statistics.mean(_keep(cnt["FETCH_SIZE"])), statistics.mean(_keep(cnt["WRITE_SIZE"]))
        out["FETCH_SIZE_kB_per_dispatch"] = round(f, 1)
        out["WRITE_SIZE_kB_per_dispatch"] = round(w, 1)
        out["hbm_bytes_per_stage"] = int(round((2.0 * f + w) * 1024.0 / per))
        out["traffic_over_algorithmic"] = round(out["hbm_bytes_per_stage"] / sb, 3)
        out["dram_GBs"] = round(out["hbm_bytes_per_stage"] / (out["stage_us"] * 1e-6) / 1e9, 1)
    E = int(c["nelx"] * c["nely"])
    sq = {k: statistics.mean(_keep(v)) for k, v in cnt.items() if k.startswith("SQ_") and v}
    if sq:
        out["sq_per_element_stage"] = {k: round(v / (E * per), 1) for k, v in sorted(sq.items())
                                       if k.startswith("SQ_INSTS") or k == "SQ_LDS_BANK_CONFLICT"}
        if "SQ_ACTIVE_INST_VALU" in sq and "SQ_WAVE_CYCLES" in sq:
            out["valu_active_over_wave_cycles"] = round(sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_WAVE_CYCLES"], 4)
        if "SQ_WAIT_ANY" in sq and "SQ_WAVE_CYCLES" in sq:
            out["wait_any_over_wave_cycles"] = round(sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"], 4)
    json.dump(out, open(os.path.join(dst, f"roofline_{cfg}.json"), "w"), indent=1)
    return out


def main():
    tag = sys.argv[1]
    path = os.path.join(REPO, "profiles", "roofline_pmc.json")
    allr = json.load(open(path)) if os.path.exists(path) else {}
    for cfg in ("dg25L3", "dg25N7L3", "dg316L3", "lake200"):
        o = summarize(tag, cfg)
        if o:
            allr[cfg] = o
            print(json.dumps(o))
    json.dump(allr, open(path, "w"), indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
