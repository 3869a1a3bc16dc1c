#!/usr/bin/env python3
"""Headline benchmark: policy evaluations / second on the 8,152-pod Alibaba
OpenB trace (16-node / 64-GPU cluster), island-model search on MI355X.

One step = one generation of every island on every GPU: each rank runs
`--islands` islands x `--candidates` random-weight candidate policies (the
reference's `_create_random_policy` family), evaluated exactly (bit-identical
to the reference scorer) in one batched k_replay launch, followed by elite
selection; every `--migrate-every` generations the islands exchange elites
with an RCCL all-gather.  `value` = total evaluations per second over all
ranks (weak scaling: per-GPU work is fixed).

    python bench.py --gpus 1 --steps 10 --warmup 2
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29500 bench.py --gpus 8 --steps 10 --warmup 2
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_EVALS_PER_S = 15.84   # reference eval path, 8 CPU workers


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--islands", type=int, default=4, help="islands per GPU")
    ap.add_argument("--candidates", type=int, default=1024, help="candidates per island per generation")
    ap.add_argument("--elite", type=int, default=32)
    ap.add_argument("--family", default="random_linear", choices=["random_linear", "feature_linear", "composite_linear"])
    ap.add_argument("--migrate-every", type=int, default=5)
    ap.add_argument("--migrants", type=int, default=8)
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--heap-mode", default="auto", choices=["auto", "lds", "hbm"])
    ap.add_argument("--seed", type=int, default=1234)
    args = ap.parse_args()

    from funsearch_kubernetes_simulator_amd.parallel import dist
    ctx = dist.init_distributed(use_gpu=args.device == "gpu")
    if ctx.world_size != args.gpus:
        if ctx.world_size > 1 or args.gpus > 1:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={ctx.world_size}: launch with torch.distributed.run")

    from funsearch_kubernetes_simulator_amd.core import load_default_workload
    from funsearch_kubernetes_simulator_amd.engine import COLS, Evaluator
    from funsearch_kubernetes_simulator_amd.funsearch.param_islands import make_islands, migrate

    workload = load_default_workload()
    device = ctx.local_rank if args.device == "gpu" else "cpu"
    ev = Evaluator(workload, device=device, options={"heap_mode": args.heap_mode})
    if args.device == "gpu" and ev.device is None:
        raise SystemExit("no HIP device visible")
    islands = make_islands(args.islands, args.family, args.candidates, args.elite,
                           seed=args.seed + 104729 * ctx.rank)
    gather = dist.all_gather_array if ctx.distributed else None

    def sync():
        if args.device == "gpu":
            import torch
            torch.cuda.synchronize()
        dist.barrier()

    best_row = [None, -1.0]

    def step(gen: int) -> None:
        props = [isl.propose() for isl in islands]
        W = np.concatenate(props)
        tab = ev.evaluate_family(args.family, W)
        off = 0
        for isl, p in zip(islands, props):
            sc = tab[off:off + len(p), COLS["score"]]
            isl.update(p, sc)
            j = int(np.argmax(sc))
            if sc[j] > best_row[1]:
                best_row[0], best_row[1] = tab[off + j].copy(), float(sc[j])
            off += len(p)
        if args.migrate_every and (gen + 1) % args.migrate_every == 0:
            migrate(islands, args.migrants, gather)

    for g in range(args.warmup):
        step(g)
    sync()
    t0 = time.perf_counter()
    for g in range(args.warmup, args.warmup + args.steps):
        step(g)
    sync()
    elapsed = dist.all_reduce_max(time.perf_counter() - t0)

    per_step = args.islands * args.candidates
    total = per_step * args.steps * ctx.world_size
    value = total / elapsed
    best_score = dist.all_reduce_max(best_row[1])
    if ctx.is_main:
        row = best_row[0]
        out = {
            "metric": "policy evals/sec on 8,152-pod Alibaba trace at 1/2/4/8 GPUs; champion util/frag",
            "value": round(value, 2),
            "unit": "policy_evals/s",
            "n_gpus": ctx.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_EVALS_PER_S, 2),
            "dtype": "fp64",
            "data": "OpenB openb_pod_list_default.csv (8,152 pods) on gpu_models_filtered.csv (16 nodes/64 GPUs); "
                    "random-weight candidate policies (reference _create_random_policy family)",
            "config": {
                "model": f"{args.family} policy family, exact replay (reference-bit-identical scores)",
                "global_batch": per_step * ctx.world_size,
                "seq_len": int(workload.pods.n_pods),
                "parallelism": f"islands: {args.islands}/GPU x {ctx.world_size} GPU(s), RCCL all-gather "
                               f"migration every {args.migrate_every} gens",
                "candidates_per_island": args.candidates,
                "backend": ev.backend,
                "heap_mode": args.heap_mode,
            },
            "best_score": best_score,
        }
        if row is not None and ctx.world_size == 1:
            out["champion"] = {"cpu_util": row[COLS["avg_cpu"]], "mem_util": row[COLS["avg_mem"]],
                               "gpu_count_util": row[COLS["avg_gpu_count"]],
                               "gpu_milli_util": row[COLS["avg_gpu_milli"]], "frag": row[COLS["frag"]]}
        print(json.dumps(out), flush=True)
    dist.shutdown()


if __name__ == "__main__":
    main()
