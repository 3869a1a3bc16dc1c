"""Which host/torch/RCCL operations wait for the resident program grid?

A persistent kernel never ends on its own, so any call that waits for the
whole device (or for a stream that synchronises with the grid's) blocks until
the grid is stopped.  Each probe runs in a thread with a deadline while the
service grid is up; a probe still running at its deadline is reported
"blocked" and the grid is stopped (which releases it) and restarted for the
next probe.  Prints one JSON line per probe.

    FKS_DIST_GROUP=1 WORLD_SIZE=1 RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29711 python tools/grid_coexist_probe.py
"""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29650 + os.getpid() % 300))
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("RANK", "0")
    import numpy as np
    import torch
    import torch.distributed as tdist
    from funsearch_kubernetes_simulator_amd.engine import Evaluator
    from funsearch_kubernetes_simulator_amd.parallel import dist
    ctx = dist.init_distributed(force_group=True)
    dev = Evaluator(device="gpu").device
    d = ctx.device
    side = torch.cuda.Stream(device=d)
    x = np.arange(4096, dtype=np.float64)
    pinned = torch.from_numpy(x).pin_memory()
    # warm every path once before the grid is up (allocator blocks, RCCL buffers)
    t = torch.from_numpy(x).to(d)
    out = [torch.empty_like(t) for _ in range(ctx.world_size)]
    tdist.all_gather(out, t)
    torch.cuda.synchronize()

    def gather_default():
        t = torch.from_numpy(x).to(d)
        o = [torch.empty_like(t) for _ in range(ctx.world_size)]
        w = tdist.all_gather(o, t, async_op=True)
        w.wait()
        return torch.stack(o).cpu()

    def gather_side():
        with torch.cuda.stream(side):
            t = pinned.to(d, non_blocking=True)
            o = [torch.empty_like(t) for _ in range(ctx.world_size)]
            w = tdist.all_gather(o, t, async_op=True)
            w.wait()
            r = torch.stack(o).to("cpu", non_blocking=True)
            side.synchronize()
        return r

    def h2d_side():
        with torch.cuda.stream(side):
            t = pinned.to(d, non_blocking=True)
            side.synchronize()

    probes = [
        ("empty_alloc_new", lambda: torch.empty(1 << 28, dtype=torch.uint8, device=d)),
        ("h2d_pageable_default", lambda: torch.from_numpy(x).to(d)),
        ("d2h_default", lambda: t.cpu()),
        ("zeros_default_stream", lambda: torch.zeros(16, device=d)),
        ("h2d_pinned_side_stream", h2d_side),
        ("all_gather_default_stream", gather_default),
        ("all_gather_side_stream", gather_side),
        ("dist_all_gather_array_async", lambda: dist.all_gather_array_async(x).wait()),
        ("host_group_all_gather_async", lambda: (dist.use_host_collectives(True),
                                                 dist.all_gather_array_async(x).wait(),
                                                 dist.use_host_collectives(False))),
        ("host_group_all_reduce_max", lambda: (dist.use_host_collectives(True), dist.all_reduce_max(1.5),
                                               dist.use_host_collectives(False))),
        ("cuda_synchronize", torch.cuda.synchronize),
    ]
    for name, fn in probes:
        dev.start_service(slots=256, share=0.875)
        time.sleep(0.2)
        done = threading.Event()
        err = []

        def run():
            try:
                fn()
            except Exception as exc:   # report, do not hang
                err.append(repr(exc)[:200])
            done.set()

        th = threading.Thread(target=run, daemon=True)
        t0 = time.perf_counter()
        th.start()
        ok = done.wait(3.0)
        dt = time.perf_counter() - t0
        dev.stop_service()          # (releases a blocked probe)
        done.wait(30.0)
        print(json.dumps({"probe": name, "blocked": not ok, "seconds": round(dt, 4),
                          "released_after_stop_s": round(time.perf_counter() - t0, 3), "error": err[:1]}), flush=True)
    dist.shutdown()


if __name__ == "__main__":
    main()
