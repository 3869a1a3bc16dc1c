#!/usr/bin/env python3
"""Headline benchmark: policy evaluations / second on the 8,152-pod Alibaba
OpenB trace (16-node / 64-GPU cluster), island-model search on MI355X.

One step = one generation of every island on every GPU: each rank runs
`--islands` islands x `--candidates` random-weight candidate policies,
evaluated exactly (bit-identical to the reference scorer) in one batched
k_replay launch, followed by elite selection; every `--migrate-every`
generations the islands exchange elites with an RCCL all-gather.  `value` =
total evaluations per second over all ranks (weak scaling: per-GPU work is
fixed).  The second half of the headline metric -- the champion's
utilisation / fragmentation -- is the best policy found during the run
(all-gathered over ranks after the timed region); `--save-best` writes it as
a policy program in the reference's results-JSON schema.

Candidate families (models/families.py): `composite_linear` (default; the
reference's `_create_random_policy` idea generalised to a 16-term linear
basis that contains the README champion), `feature_linear`, and
`random_linear` (exactly `_create_random_policy`,
`funsearch/funsearch_integration.py:403-431`).

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
BASELINE_SYNTHETIC_EVALS_PER_S = 0.1   # config 5: ~10 s per reference eval on 1 CPU core


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--islands", type=int, default=4, help="islands per GPU")
    # 12,288 per island: each row of the persistent row kernel drains ~3 policies
    # per launch, so short replays backfill behind long ones (4,096: one policy
    # per row, every wave waits for its longest replay; profiles/README.md)
    ap.add_argument("--candidates", type=int, default=12288, help="candidates per island per generation")
    ap.add_argument("--elite", type=int, default=32)
    ap.add_argument("--family", default="composite_linear", choices=["random_linear", "feature_linear", "composite_linear"])
    ap.add_argument("--migrate-every", type=int, default=5)
    ap.add_argument("--migrants", type=int, default=8)
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--heap-mode", default="auto", choices=["auto", "lds", "hbm"])
    ap.add_argument("--heap-top", type=int, default=-1,
                    help="wave kernel (> 16 nodes): heap slots kept in LDS per policy (2^k - 1; -1: auto)")
    ap.add_argument("--row-composite-waves", type=int, default=5, choices=[4, 5],
                    help="waves per SIMD of the composite row kernel (register budget 128 / 96 VGPRs; "
                         "5: heap top 63 slots in LDS instead of 127)")
    ap.add_argument("--row-min-lds", type=int, default=0,
                    help="occupancy experiments: at least this many LDS bytes per row-kernel wave")
    ap.add_argument("--row-split-heap", action="store_true",
                    help="composite row kernel with exec-masked LDS/HBM heap accesses instead of flat ones")
    ap.add_argument("--row-wave-share", type=float, default=1.0,
                    help="fraction of the chip's resident waves one island launch takes (row kernel)")
    ap.add_argument("--wave-duo", type=int, default=-1, choices=[-1, 0, 1],
                    help="256-node clusters: two-wave (heap wave + scoring wave) kernel on/off (-1: engine default)")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--trace", default="default", choices=["default", "synthetic"],
                    help="default: 8,152-pod OpenB trace on 16 nodes; synthetic: BASELINE config 5 shape")
    ap.add_argument("--nodes", type=int, default=256, help="synthetic trace: nodes")
    ap.add_argument("--pods", type=int, default=65536, help="synthetic trace: pods")
    ap.add_argument("--sync-islands", action="store_true",
                    help="one launch per generation for all islands (default: one HIP stream per island)")
    ap.add_argument("--save-best", default="", help="write the champion program (reference results-JSON schema)")
    ap.add_argument("--programs", type=int, default=64,
                    help="after the timed region: evaluate this many FunSearch candidate programs (offline-mutation "
                         "children) through the native program backend and report them as `program_path` (0: skip)")
    ap.add_argument("--novel", type=int, default=256,
                    help="after the timed region: this many programs, every one a NEW shape (JIT included), "
                         "against the CPU VM on the same batch; reported as `program_path.novel` (0: skip)")
    ap.add_argument("--novel-large", type=int, default=2048,
                    help="after the timed region: an LLM-scale batch of this many new-shape programs (JIT included, "
                         "chunks over the slots, all in flight at once); reported as `program_path.novel_large` (0: skip)")
    ap.add_argument("--evolved-service-s", type=float, default=8.0,
                    help="seconds of sustained evolved-program replay through the resident program service "
                         "(`program_path.evolved.service`; 0: skip)")
    ap.add_argument("--evolved", type=int, default=2048,
                    help="children of an evolved population (data/populations, frozen sources) through the "
                         "native backend, all in flight; reported as `program_path.evolved` (0: skip)")
    ap.add_argument("--time-budget", type=float, default=0.0,
                    help="run generations until this many seconds have passed (instead of --steps); "
                         "steps = generations completed")
    args = ap.parse_args()

    from funsearch_kubernetes_simulator_amd.parallel import dist
    ctx = dist.init_distributed(use_gpu=args.device == "gpu")
    if ctx.world_size != args.gpus:
        if ctx.world_size > 1 or args.gpus > 1:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={ctx.world_size}: launch with torch.distributed.run")

    from funsearch_kubernetes_simulator_amd.core import load_default_workload
    from funsearch_kubernetes_simulator_amd.engine import COLS, Evaluator
    from funsearch_kubernetes_simulator_amd.funsearch.param_islands import inject, inject_one, make_islands, migration_records
    from funsearch_kubernetes_simulator_amd.utils.trace import roctx_range

    if args.trace == "synthetic":
        from funsearch_kubernetes_simulator_amd.core import synthetic_workload
        workload = synthetic_workload(n_nodes=args.nodes, n_pods=args.pods, seed=0)
    else:
        workload = load_default_workload()
    if args.device == "gpu":
        import torch
        device = ctx.local_rank % max(1, torch.cuda.device_count())   # one rank per GPU (wraps on smaller boxes)
    else:
        device = "cpu"
    # the per-event trace hash only serves cross-engine equality tests: off here
    opts = {"heap_mode": args.heap_mode, "trace_hash": False, "row_wave_share": args.row_wave_share,
            "row_composite_waves": args.row_composite_waves, "row_flat": not args.row_split_heap,
            "row_min_lds": args.row_min_lds}
    if args.heap_top >= 0:
        opts["heap_top"] = args.heap_top
    if args.wave_duo >= 0:
        opts["wave_duo"] = bool(args.wave_duo)
    ev = Evaluator(workload, device=device, options=opts,
                   n_slots=max(1, args.islands))
    if args.device == "gpu" and ev.device is None:
        raise SystemExit("no HIP device visible")
    if args.device == "gpu" and ctx.backend == "nccl":
        # the RCCL collective buffers and the replay engine must live on the same card
        import torch
        assert ctx.device.index == device == ev.device.device == torch.cuda.current_device(), \
            (ctx.device, device, ev.device.device, torch.cuda.current_device())
    islands = make_islands(args.islands, args.family, args.candidates, args.elite,
                           seed=args.seed + 104729 * ctx.rank)
    def propose(isl) -> np.ndarray:
        return isl.propose()

    def sync():
        if args.device == "gpu":
            import torch
            torch.cuda.synchronize(device)
        dist.barrier()

    best_row = [None, -1.0, None, -1]   # table row, score, weights, generation
    events = [0.0]

    def absorb(isl, props, tab, gen: int) -> None:
        sc = tab[:, COLS["score"]]
        isl.update(props, sc, tab[:, COLS["n_events"]])
        events[0] += float(tab[:, COLS["n_events"]].sum())
        j = int(np.argmax(sc))
        if sc[j] > best_row[1]:
            best_row[:] = [tab[j].copy(), float(sc[j]), props[j].copy(), gen]

    def epoch_sync(gen0: int, n: int) -> None:
        """All islands in one launch per generation (--sync-islands)."""
        for gen in range(gen0, gen0 + n):
            props = [propose(isl) for isl in islands]
            tab = ev.evaluate_family(args.family, np.concatenate(props))
            off = 0
            for isl, p in zip(islands, props):
                absorb(isl, p, tab[off:off + len(p)], gen)
                off += len(p)

    def run_async(g0: int, count: int) -> None:
        """`count` generations of every island, back to back on each island's
        own slot: no island waits for another, at migration points included
        (an epoch barrier idled the chip while the last island finished its
        epoch).  When the slowest local island has passed a boundary (a
        multiple of --migrate-every) the rank's current elites go into a
        non-blocking all-gather -- issued in boundary order, so every rank
        issues the same sequence -- and each island takes its ring
        predecessor's migrants from the newest completed gather when it next
        reaches a boundary (islands that finish first take it at the end)."""
        M = args.migrate_every
        k = len(islands)
        props, gens, left = [None] * k, [g0] * k, [count] * k
        bounds = [b for b in range(g0 + 1, g0 + count + 1) if M and b % M == 0]
        issued, gathers, newest, taken = 0, [], None, [-1] * k

        def launch(i: int) -> None:
            props[i] = propose(islands[i])
            ev.submit_family(i, args.family, props[i])

        for i in range(k):
            launch(i)
        pending = set(range(k))
        while pending or gathers:
            progressed = False
            while issued < len(bounds) and min(gens) >= bounds[issued]:
                gathers.append((issued, dist.all_gather_array_async(migration_records(islands, args.migrants))))
                issued += 1
            while gathers and gathers[0][1].done():
                newest = (gathers[0][0], gathers[0][1].wait())
                gathers.pop(0)
                progressed = True
            for i in sorted(pending):
                if not ev.ready(i):
                    continue
                absorb(islands[i], props[i], ev.wait(i), gens[i])
                gens[i] += 1
                left[i] -= 1
                progressed = True
                if M and gens[i] % M == 0 and newest is not None and taken[i] < newest[0]:
                    inject_one(islands, i, newest[1], ctx.rank)
                    taken[i] = newest[0]
                if left[i]:
                    launch(i)
                else:
                    pending.discard(i)
            if not progressed:
                time.sleep(0.0002)
        if newest is not None:
            for i in range(k):
                if taken[i] < newest[0]:
                    inject_one(islands, i, newest[1], ctx.rank)

    def run(g0: int, count: int) -> None:
        """`count` generations of every island; migration at every multiple of
        --migrate-every.  Asynchronous islands: run_async.  --sync-islands: one
        launch per generation, the elite all-gather (RCCL) started without
        blocking at each migration point and injected one epoch later."""
        if not args.sync_islands:
            return run_async(g0, count)
        M = args.migrate_every or (g0 + count + 1)
        g = g0
        pending = None
        while g < g0 + count:
            n = min(M - g % M, g0 + count - g)
            with roctx_range(f"bench.generations {g}-{g + n - 1}"):
                epoch_sync(g, n)
            g += n
            if args.migrate_every and g % M == 0:
                with roctx_range("bench.migrate"):
                    if pending is not None:
                        inject(islands, pending.wait(), ctx.rank)
                    pending = dist.all_gather_array_async(migration_records(islands, args.migrants))
        if pending is not None:
            inject(islands, pending.wait(), ctx.rank)

    run(0, args.warmup)
    sync()
    events[0] = 0.0
    t0 = time.perf_counter()
    if args.time_budget > 0:
        # whole migration epochs until the budget is spent (ranks agree on when to stop)
        g, chunk = args.warmup, max(1, args.migrate_every or 5)
        while True:
            run(g, chunk)
            g += chunk
            if dist.all_reduce_max(time.perf_counter() - t0) >= args.time_budget:
                break
        args.steps = g - args.warmup
    else:
        run(args.warmup, args.steps)
    sync()
    elapsed = dist.all_reduce_max(time.perf_counter() - t0)
    events_total = dist.all_reduce_sum(events[0])

    program_path = None
    jit_init_s = None
    if ev.device is not None and (args.programs > 0 or args.novel > 0 or args.novel_large > 0 or args.evolved > 0):
        # first-use JIT initialisation, reported on its own (not in the first batch's jit_s)
        jit_init_s = round(ev.device.warm_native(), 3)
    if args.programs > 0 and ev.device is not None:
        # the program-for-program comparison with the reference's eval path (outside the timed region)
        from funsearch_kubernetes_simulator_amd.bench.programs import measure_native, mutation_children
        program_path = measure_native(ev.device, mutation_children(args.programs, seed=args.seed + ctx.rank))
        program_path["vs_baseline"] = round(program_path["evals_per_s_incl_jit"] / BASELINE_EVALS_PER_S, 2)
        program_path["engine"] = "hip-native (JIT-compiled programs called from a precompiled replay kernel)"
        program_path["note"] = ("top level: offline-mutation children, shapes may repeat within the batch; "
                                "`novel`: every program a fresh shape (the real-LLM case)")
        if args.novel > 0:
            from funsearch_kubernetes_simulator_amd.bench.programs import measure_novel
            nov = measure_novel(ev.device, workload, args.novel, seed=args.seed + 17 + 1000 * ctx.rank)
            nov["vs_baseline"] = round(nov["evals_per_s_incl_jit"] / BASELINE_EVALS_PER_S, 2)
            program_path["novel"] = nov
        if args.novel_large > 0:
            from funsearch_kubernetes_simulator_amd.bench.programs import measure_novel_large
            big = measure_novel_large(ev.device, workload, args.novel_large, seed=args.seed + 31 + 1000 * ctx.rank)
            big["vs_baseline"] = round(big["evals_per_s_incl_jit"] / BASELINE_EVALS_PER_S, 2)
            program_path["novel_large"] = big
        if args.evolved > 0 and args.trace == "default":
            # the search's late-run workload: children of an evolved population
            from funsearch_kubernetes_simulator_amd.bench.programs import measure_evolved
            evo = measure_evolved(ev.device, workload, args.evolved, service_s=args.evolved_service_s)
            evo["vs_baseline"] = round(evo["evals_per_s_incl_jit"] / BASELINE_EVALS_PER_S, 2)
            program_path["evolved"] = evo

    per_step = args.islands * args.candidates
    total = per_step * args.steps * ctx.world_size
    value = total / elapsed
    # champion over all ranks (outside the timed region): [score, generation, table row, weights]
    from funsearch_kubernetes_simulator_amd.models import families as fam
    rec = np.concatenate([[best_row[1], best_row[3]], best_row[0], fam.pad_weights(best_row[2])[0]])
    allrec = dist.all_gather_array(rec[None]).reshape(-1, rec.size) if ctx.distributed else rec[None]
    champ = allrec[int(np.argmax(allrec[:, 0]))]
    ncol = len(COLS)
    row, wbest = champ[2:2 + ncol], champ[2 + ncol:]
    if ctx.is_main:
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
            "vs_baseline": round(value / (BASELINE_EVALS_PER_S if args.trace == "default"
                                          else BASELINE_SYNTHETIC_EVALS_PER_S), 2),
            "dtype": "fp64",
            "data": ("OpenB openb_pod_list_default.csv (8,152 pods) on gpu_models_filtered.csv (16 nodes/64 GPUs)"
                     if args.trace == "default" else
                     f"synthetic scaled trace {workload.pods.n_pods} pods / {workload.cluster.n_nodes} nodes "
                     "(BASELINE config 5 shape, tiled OpenB rows)")
                    + f"; random-weight candidate policies ({args.family} family, random init)",
            "config": {
                "model": f"{args.family} policy family, exact replay (reference-bit-identical scores)",
                "global_batch": per_step * ctx.world_size,
                "seq_len": int(workload.pods.n_pods),
                "parallelism": f"islands: {args.islands}/GPU x {ctx.world_size} rank(s), "
                               + (f"{'RCCL' if ctx.backend == 'nccl' else ctx.backend} all-gather migration every "
                                  f"{args.migrate_every} gens" if ctx.distributed else "single rank (no collectives)"),
                "dist_backend": ctx.backend,
                "world_size": ctx.world_size,
                "candidates_per_island": args.candidates,
                "backend": ev.backend,
                "heap_mode": args.heap_mode,
                "islands_async": not args.sync_islands,
            },
            "events_per_s": round(events_total / elapsed, 1),
            "best_score": float(champ[0]),
            "champion": {"cpu_util": row[COLS["avg_cpu"]], "mem_util": row[COLS["avg_mem"]],
                         "gpu_count_util": row[COLS["avg_gpu_count"]],
                         "gpu_milli_util": row[COLS["avg_gpu_milli"]], "frag": row[COLS["frag"]]},
            "reference_champion": {"score": 0.49013357497851473, "cpu_util": 0.459, "mem_util": 0.261,
                                   "gpu_count_util": 0.734, "frag": 0.033},
            "vs_baseline_note": "value = parametric-family evals/s (BASELINE config 2: random-weight candidates) "
                                "divided by the reference's PROGRAM evals/s (15.84, 8 CPU workers); program_path "
                                "is the program-for-program comparison",
            "program_path": program_path,
            "program_path_jit_init_s": jit_init_s,
        }
        if ev.device is not None:
            from funsearch_kubernetes_simulator_amd.ops.hip_engine import math_selfcheck_info
            out["device_math"] = math_selfcheck_info()
        if args.time_budget > 0:
            out["time_budget_s"] = args.time_budget
        if args.save_best:
            k = {"random_linear": 4, "feature_linear": fam.N_FEATURES}.get(args.family, fam.N_COMPOSITE)
            code = fam.to_program(args.family, wbest[:k])
            with open(args.save_best, "w") as f:
                json.dump({"score": float(champ[0]), "generation": int(champ[1]), "code": code,
                           "timestamp": time.strftime("%Y%m%d_%H%M%S"), "family": args.family,
                           "weights": [float(x) for x in wbest[:k]],
                           "results": {c: float(row[i]) for c, i in COLS.items()}}, f, indent=2)
            out["saved"] = args.save_best
        print(json.dumps(out), flush=True)
    dist.shutdown()


if __name__ == "__main__":
    main()
