"""bench.py's N>1 branch on the one GPU of the test box (missing 1): `--emulate W:R`
runs rank R of a W-rank processor-face partition under torch.distributed.run with the real run's
code -- the nccl process group, the RCCL id broadcast, face_partition, the engine's own RCCL
communicator, the two-stream schedule, the timed loop with barriers and max over ranks, the halo
check and the strong-scaling base -- the rank's processor faces listed under itself.  The line
must parse, carry a bitwise halo check and the strong-scaling base, and report a finite rate.
(One child process; the parent test process holds the GPU too: two processes on the card.)"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_n_gt_1_branch_runs_on_one_gpu():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--emulate", "2:1", "--config", "bump10", "--steps", "2",
           "--warmup", "1"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, lines  # the JSON line alone (library banners go to stderr)
    d = json.loads(lines[0])
    assert d["halo_bitwise"] is True and d["halo_check"]["max_rel_diff"] == 0.0
    assert d["scaling"] == "emulated" and d["emulated"] is True and d["value"] > 0 and d["ms_per_step"] > 0
    assert "EMULATED" in d["config"]["parallelism"]
    em = d["emulation"]
    assert em["world"] == 2 and em["rank"] == 1 and em["processor_faces"] > 0 and em["projection_eu_per_s"] > 0
    assert d["strong_scaling_base"]["value"] > 0 and d["speedup_vs_base"] > 0
    assert abs(d["efficiency_vs_base"] - d["speedup_vs_base"] / 2) < 1e-3
    for k in ("init_process_group_s", "case_build_s", "engine_create_s", "first_step_s", "halocheck_s"):
        assert k in d["setup_s"], k


def test_bench_emulates_a_morton_lake_rank_with_its_frozen_halo():
    """C5's own shape through bench.py (missing 2): rank 1 of the lake on a 4-rank
    Morton partition keeps its three per-neighbour lists (three RCCL send/recv pairs to itself per
    exchange) and, the lake at rest, the frozen halo; the line carries a bitwise halo check against
    the same self-neighbour partition as a local exchange group, and the state stays finite."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--emulate", "4:1", "--config", "lake10", "--steps", "2",
           "--warmup", "1", "--no-base"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.strip()][0])
    assert d["halo_bitwise"] is True and d["emulated"] is True and d["value"] > 0
    em = d["emulation"]
    assert em["order"] == "morton" and em["halo"] == "frozen" and em["lists"] == "peers"
    assert em["messages_per_exchange"] == 3
