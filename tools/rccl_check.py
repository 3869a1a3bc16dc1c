"""RCCL on one MI355X: a world-size-1 ``nccl`` process group (torch.distributed
over RCCL) used by the island search's collectives while the HIP extension
keeps its four replay slots busy.

The multi-GPU scaling curve is measured by the driver on an 8-GPU node; this
exercises, on the one-GPU box, everything a rank does with RCCL:

* the group's device is the extension's device (one process per GPU);
* `all_gather_bytes`, `all_gather_array_async` (RCCL on its own stream, polled
  with `work.is_completed()`) and `all_reduce_max` complete while four native
  program batches replay on the extension's HIP streams, with results equal
  to the local (``backend="none"``) ones;
* `MigrationChannel.post / poll` round trips with the search's own payloads;
* a short steady-state run of the shipped config 4 (``--config``: steady loop,
  resident program service, family coupler; ``migrate_every`` 5 here, so every
  few seconds a migration all-gather runs beside the persistent grid), ending
  with the service's abort + stop: every gather must complete, none may block
  the dispatcher for more than ``--max-stall-s``, and the run must end
  promptly.  RCCL collectives cannot progress while the grid is resident
  (tools/grid_coexist_probe.py), so those gathers go over the gloo group
  `dist.init_distributed` opens beside RCCL (`host_collectives` in the output).

Prints one JSON line.  Run it under ``rocprofv3 --kernel-trace --stats`` to
see the RCCL all-gather kernels beside ``k_replay_native_duo``.

    FKS_DIST_GROUP=1 python tools/rccl_check.py --steady-s 20
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steady-s", type=float, default=20.0)
    ap.add_argument("--migrate-every", type=int, default=5)
    ap.add_argument("--config", default="configs/config4.json")
    ap.add_argument("--max-stall-s", type=float, default=1.0)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29600 + os.getpid() % 300))
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("RANK", "0")
    import numpy as np
    import torch
    from funsearch_kubernetes_simulator_amd.parallel import dist
    ctx = dist.init_distributed(force_group=True)
    out = {"backend": ctx.backend, "world_size": ctx.world_size, "group": ctx.group}
    assert ctx.backend == "nccl", ctx.backend
    import torch.distributed as tdist
    out["torch_backend"] = str(tdist.get_backend())
    from funsearch_kubernetes_simulator_amd.engine import Evaluator
    from funsearch_kubernetes_simulator_amd.bench.programs import mutation_children
    ev = Evaluator(device="gpu")
    dev = ev.device
    out["rccl_device"] = str(ctx.device)
    out["ext_device"] = int(dev.device)
    out["torch_current_device"] = int(torch.cuda.current_device())
    assert ctx.device.index == dev.device == torch.cuda.current_device()
    # collectives while four replay slots are busy
    progs = mutation_children(256, 3)
    for slot in range(4):
        dev.submit_native(slot, progs[slot * 64:(slot + 1) * 64])
    busy = [not dev.ready(s) for s in range(4)]
    t0 = time.perf_counter()
    payload = os.urandom(5000)
    got = dist.all_gather_bytes(payload)
    assert got == [payload]
    x = np.arange(1 << 16, dtype=np.float64).reshape(-1, 8)
    h = dist.all_gather_array_async(x)
    polls = 0
    while not h.done():
        polls += 1
        time.sleep(0.0005)
    g = h.wait()
    assert g.shape == (1,) + x.shape and np.array_equal(g[0], x)
    assert dist.all_reduce_max(0.625) == 0.625
    out["collectives_s"] = round(time.perf_counter() - t0, 4)
    out["slots_busy_during_collectives"] = busy
    out["async_polls"] = polls
    tabs = [dev.wait(s) for s in range(4)]
    ref = ev.device.evaluate_native(progs[:64])
    out["replays_equal_after_collectives"] = bool(np.array_equal(tabs[0][:, :13], ref[:, :13]))
    if a.steady_s <= 0:
        dist.shutdown()
        print(json.dumps(out), flush=True)
        return
    # a steady config-3 run with RCCL migrations
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    from funsearch_kubernetes_simulator_amd.funsearch.search import load_config
    cfg = load_config(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), a.config))
    tmp = tempfile.mkdtemp(prefix="fks_rccl_")
    cfg["islands"]["migrate_every"] = a.migrate_every
    cfg["islands"].setdefault("steady", {}).update(wall_s=a.steady_s, producers=8, status_every_s=5)
    out["config"] = a.config
    out["service"] = bool(cfg["islands"]["steady"].get("service"))
    cfg["checkpoint"] = {"dir": os.path.join(tmp, "ck"), "every": 1000}
    cfg["log_path"] = os.path.join(tmp, "metrics.jsonl")
    run = IslandFunSearch(cfg, evaluator=ev)
    t0 = time.perf_counter()
    code, score = run.run(None)
    out["steady_s"] = round(time.perf_counter() - t0, 2)
    st = run.steady.stats if getattr(run, "steady", None) is not None else None
    mig = [json.loads(l) for l in open(cfg["log_path"]) if '"steady_migration"' in l]
    out["steady_migrations"] = len(mig)
    out["steady_best"] = round(float(score), 6)
    out["steady_evaluations"] = int(run.evaluations)
    out["collective_wait_s"] = mig[-1]["collective_wait_s"] if mig else None
    out["host_collectives"] = bool(getattr(run.steady, "host_collectives", False))
    out["max_stall_s"] = round(run.steady.channel.max_stall_s, 4)
    out["max_gather_s"] = round(run.steady.channel.max_gather_s, 4)
    out["posted"] = (run.steady.channel.next - run.steady.channel.every) // max(1, run.steady.channel.every) \
        if run.steady.channel.next is not None else 0
    svc = [json.loads(l) for l in open(cfg["log_path"]) if '"steady_service"' in l]
    fin = [json.loads(l) for l in open(cfg["log_path"]) if '"steady_final"' in l]
    out["service_blocks"] = svc[0]["blocks"] if svc else 0
    if fin:
        out["final"] = {k: fin[-1].get(k) for k in ("wall_s", "evals_per_s", "occupancy_mean", "coupled",
                                                      "abandoned", "rollovers")}
    if st is not None:
        out["steady_stats"] = {k: getattr(st, k) for k in ("migrations", "evaluations") if hasattr(st, k)}
    assert len(mig) >= 1, "no migration completed"
    assert not run.steady.channel.pending, "a gather never completed"
    assert out["max_stall_s"] <= a.max_stall_s, f"a collective blocked the dispatcher {out['max_stall_s']} s"
    assert out["steady_s"] <= a.steady_s + 60, "the run did not end promptly after its wall time"
    dist.shutdown()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
