"""Where does the occupancy estimate of the persistent sub-cycle launch disagree with the
dispatcher?  For each LDS pad (dynamic LDS added to every workgroup, HNUMO_PERSIST_LDS_PAD) the
engine is created with the trial launch only (HNUMO_PERSIST_GUARD=trial) and reports the
estimate (workgroups per CU, hipOccupancyMaxActiveBlocksPerMultiprocessor) beside the trial's
outcome (all workgroups of the grid resident at once, or not).
Usage (GPU): python tools/residency_sweep.py cfg pad0 pad1 step"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "h-numo_amd"))
from hnumo.case import build_case, make_config  # noqa: E402
from hnumo.engine import Engine  # noqa: E402
os.environ["HNUMO_EXPERIMENTS"] = "1"   # the engine honours HNUMO_* experiment knobs only with this

cfg, p0, p1, st = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
case = build_case(make_config(cfg), dense=False)
E = case.dims["nelem"] if hasattr(case, "dims") else None
os.environ["HNUMO_PERSIST_GUARD"] = "trial"
print(f"{cfg}: pad bytes | LDS bytes per workgroup | estimate per CU x CUs | trial (1 resident)", flush=True)
for pad in range(p0, p1 + 1, st):
    os.environ["HNUMO_PERSIST_LDS_PAD"] = str(pad)
    e = Engine(case)
    i = e.persistent_info
    nb = i["occupancy_blocks_per_cu"][0]
    print(f"pad {pad:6d} | lds {i['lds_bytes_per_workgroup']:6d} | 3 x lds {3 * i['lds_bytes_per_workgroup']:7d} | "
          f"estimate {nb} x {i['cus']} = {nb * i['cus']:5d} | trial {i['trial_launch'][0]} | "
          f"path {e.stage_path}", flush=True)
    e.close()
