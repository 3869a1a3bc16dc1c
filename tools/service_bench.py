"""Resident program service vs per-batch launches on the evolved-program set.

The same 2,048 evolved children (bench/programs.py EVOLVED_SET) are replayed
  * batch:   split over the engine's stream slots, one two-wave launch each
             (the shape of bench.py --evolved, cached pass);
  * service: the resident grid (ops/hip_engine.py start_service), the same
             programs queued as batches of --chunk;
  * rolling: both modes driven like the steady loop -- `slots` batches of
             --chunk in flight, a finished batch replaced at once -- for
             --seconds each; programs/s and the mean batch latency.
Rows of the service runs are checked bit-identical to the batch rows.

    python tools/service_bench.py --out gpurun_out/service_bench.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rolling(dev, progs, chunk, slots, seconds, base):
    """Steady-loop pattern: `slots` batches in flight, each replaced on completion."""
    n = len(progs)
    nxt = 0
    inflight = {}
    done = 0
    lat = []
    t0 = time.perf_counter()
    while True:
        now = time.perf_counter()
        for s in range(slots):
            if s not in inflight and now - t0 < seconds:
                part = [progs[(nxt + i) % n] for i in range(chunk)]
                nxt = (nxt + chunk) % n
                dev.submit_native(base + s, part)
                inflight[s] = time.perf_counter()
        if not inflight:
            break
        progressed = False
        for s in list(inflight):
            if dev.ready(base + s):
                dev.wait(base + s)
                lat.append(time.perf_counter() - inflight.pop(s))
                done += chunk
                progressed = True
        if not progressed:
            time.sleep(0.0005)
    wall = time.perf_counter() - t0
    return {"programs": done, "wall_s": round(wall, 3), "evals_per_s": round(done / wall, 1),
            "batch_latency_mean_s": round(float(np.mean(lat)), 4) if lat else None,
            "batch_latency_max_s": round(float(np.max(lat)), 4) if lat else None}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--batch-chunk", type=int, default=512, help="rolling batch mode: programs per slot launch")
    ap.add_argument("--service-slots", type=int, default=16)
    ap.add_argument("--share", type=float, default=1.0)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    from funsearch_kubernetes_simulator_amd.bench.programs import evolved_children
    from funsearch_kubernetes_simulator_amd.core import load_default_workload
    from funsearch_kubernetes_simulator_amd.ops import hip_engine as he

    w = load_default_workload()
    progs = evolved_children(args.n)
    dev = he.DeviceEvaluator(w)
    dev.warm_native()
    out = {"programs": len(progs), "chunk": args.chunk}

    slots = dev.n_slots
    size = -(-len(progs) // slots)
    chunks = [progs[i:i + size] for i in range(0, len(progs), size)]
    dev.set_options(native_inflight=len(progs))
    for s, c in enumerate(chunks):      # JIT pass (every shape compiled and loaded)
        dev.submit_native(s, c)
    for s in range(len(chunks)):
        dev.wait(s)
    t0 = time.perf_counter()
    for s, c in enumerate(chunks):
        dev.submit_native(s, c)
    ref = np.concatenate([dev.wait(s) for s in range(len(chunks))])
    t1 = time.perf_counter()
    for s, c in enumerate(chunks):      # the batch path against itself
        dev.submit_native(s, c)
    ref2 = np.concatenate([dev.wait(s) for s in range(len(chunks))])
    out["batch"] = {"slots": slots, "repeat_differs": int((ref2 != ref).any(axis=1).sum()), "wall_s": round(t1 - t0, 3), "evals_per_s": round(len(progs) / (t1 - t0), 1),
                    "device": {k: v for k, v in dev.info().items() if k.startswith("native_duo")}}
    print(json.dumps({"batch": out["batch"]}), flush=True)
    dev.set_options(native_inflight=args.batch_chunk * slots)
    out["batch_rolling"] = _rolling(dev, progs, args.batch_chunk, slots, args.seconds, 0)
    out["batch_rolling"]["chunk"] = args.batch_chunk
    print(json.dumps({"batch_rolling": out["batch_rolling"]}), flush=True)

    info = dev.start_service(slots=max(16384, 4 * args.chunk * args.service_slots), share=args.share)
    out["service_info"] = info
    try:
        base = dev.SERVICE_SLOT_BASE
        parts = [progs[i:i + args.chunk] for i in range(0, len(progs), args.chunk)]
        t0 = time.perf_counter()
        for k, c in enumerate(parts):
            dev.submit_native(base + k, c)
        tab = np.concatenate([dev.wait(base + k) for k in range(len(parts))])
        t1 = time.perf_counter()
        out["service"] = {"wall_s": round(t1 - t0, 3), "evals_per_s": round(len(progs) / (t1 - t0), 1),
                          "bit_identical_to_batch": bool((tab == ref).all())}
        bad = np.flatnonzero((tab != ref).any(axis=1))
        if bad.size:
            cols = sorted(set(int(c) for c in np.flatnonzero((tab[bad] != ref[bad]).any(axis=0))))
            out["service"]["mismatch"] = {
                "rows": int(bad.size), "columns": cols,
                "examples": [{"i": int(i), "service": tab[i].tolist(), "batch": ref[i].tolist(),
                              "source": progs[i].source[-300:]} for i in bad[:4]]}
            out["service"]["mismatch"]["batch_repeat_differs"] = int((ref2 != ref).any(axis=1).sum())
            # is a wrong service row some other program's batch row?  (a slot mix-up)
            out["service"]["mismatch"]["equals_other_batch_row"] = [
                [int(j) for j in np.flatnonzero((ref == tab[i]).all(axis=1))] for i in bad[:16]]
            out["service"]["mismatch"]["indices"] = [int(i) for i in bad[:64]]
        # the same programs again: all in one submission (one publish), then
        # again as chunks -- which rows differ, and do they repeat?
        for tag, size in (("one_submit", len(progs)), ("chunks_again", args.chunk)):
            parts2 = [progs[i:i + size] for i in range(0, len(progs), size)]
            for k, c in enumerate(parts2):
                dev.submit_native(base + k, c)
            t2 = np.concatenate([dev.wait(base + k) for k in range(len(parts2))])
            out["service"][tag] = [int(i) for i in np.flatnonzero((t2 != ref).any(axis=1))[:64]]
        print(json.dumps({"service": out["service"]}), flush=True)
        out["service_rolling"] = _rolling(dev, progs, args.chunk, args.service_slots, args.seconds, base)
        out["service_rolling"]["slots"] = args.service_slots
        print(json.dumps({"service_rolling": out["service_rolling"]}), flush=True)
        out["service_after"] = dev.info()["service"]
    finally:
        dev.stop_service()
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
