"""RCCL on the MI355X box: a world-size-1 ``nccl`` process group next to the
HIP extension's replay slots and then the shipped config 4 loop -- the
persistent program grid, the family coupler and RCCL migrations at once --
(tools/rccl_check.py, in its own process so the group does not outlive the
test)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_group_beside_replay_slots():
    env = dict(os.environ, FKS_DIST_GROUP="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29700 + os.getpid() % 200), PYTHONPATH=REPO)
    # the shipped config 4 (steady loop, persistent program grid, family coupler)
    # with an RCCL all-gather every 5 generations beside the grid
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "rccl_check.py"), "--steady-s", "20",
                        "--migrate-every", "5", "--config", "configs/config4.json", "--max-stall-s", "1.0"],
                       env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["backend"] == "nccl" and out["torch_backend"] == "nccl" and out["group"]
    assert out["ext_device"] == out["torch_current_device"] and out["rccl_device"].endswith(f":{out['ext_device']}")
    assert any(out["slots_busy_during_collectives"])
    assert out["replays_equal_after_collectives"]
    assert out["steady_migrations"] >= 1 and out["steady_best"] > 0.4
    assert out["service"] and out["service_blocks"] > 0 and out["max_stall_s"] <= 1.0
    # beside the resident grid the migrations go over the gloo group next to RCCL
    assert out["host_collectives"]
