"""Device throughput on an evolved population's children (native JIT path).

Children of the best programs in a steady-state checkpoint (or a top-k
results file) are made with the offline mutator, compiled, JIT-compiled
once, then replayed in `--batch`-program launches on one slot; prints one
JSON line per variant with the cached device evals/s.  Variants run in
child processes with different environment knobs, so JIT code-generation
choices can be A/B'd on the same programs in one GPU session:

    python tools/population_bench.py --ck gpurun_out/r4g/ck/islands_rank0.json \
        --children 2048 --variant base= --variant narrow=FKS_JIT_NARROW_SAVES=1

--save-sources FILE writes the children's sources (CPU only); --sources FILE
replays exactly those programs, so code-generation changes can be compared
across commits on identical programs.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _programs_from(sources: str, n: int):
    """Programs from a JSON list of source strings (--save-sources output):
    the same programs whatever the compiler or mutator version (A/B of code
    generation changes across commits)."""
    from funsearch_kubernetes_simulator_amd.policy.compiler import try_compile
    out = []
    if sources.endswith(".gz"):
        from funsearch_kubernetes_simulator_amd.bench.programs import load_program_set
        srcs = load_program_set(sources)
    else:
        srcs = json.load(open(sources))
    for src in srcs:
        p, _ = try_compile(src)
        if p is not None and p.device_ok:
            out.append(p)
    return out[:n]


def _programs(path: str, n: int, seed: int):
    import random
    from funsearch_kubernetes_simulator_amd.funsearch import steady
    from funsearch_kubernetes_simulator_amd.policy.compiler import try_compile
    d = json.load(open(path))
    pop = []

    def walk(o):
        if isinstance(o, dict):
            if isinstance(o.get("code"), str) and isinstance(o.get("score"), (int, float)):
                pop.append((o["code"], float(o["score"])))
            for v in o.values():
                walk(v)
        elif isinstance(o, list):
            if len(o) == 2 and isinstance(o[0], str) and isinstance(o[1], (int, float)):
                pop.append((o[0], float(o[1])))
            else:
                for v in o:
                    walk(v)
    walk(d)
    pop.sort(key=lambda x: -x[1])
    elites = pop[:8]
    steady._producer_init({"backend": "mutation", "seed": seed}, 3, 1)
    # deterministic children (the producer seeds from its pid): the same programs
    # in every variant's process
    steady._W["rng"] = random.Random(seed)
    steady._W["gen"].llm_client.rng = random.Random(seed + 1)
    random.seed(seed)
    out = []
    while len(out) < n:
        items, _ = steady._produce((0, elites, 64))
        out += [p for _, _, p in items if p is not None and p.device_ok]
    return out[:n]


def child(args) -> None:
    import numpy as np
    from funsearch_kubernetes_simulator_amd.core import load_default_workload
    from funsearch_kubernetes_simulator_amd.ops.hip_engine import DeviceEvaluator
    progs = _programs_from(args.sources, args.children) if args.sources else _programs(args.ck, args.children, args.seed)
    dev = DeviceEvaluator(load_default_workload())
    dev.set_options(native_inflight=args.batch)
    if args.rows:
        dev.set_options(native_rows=args.rows)   # programs per wave (four: k_replay_rows_native)
    if args.polish:
        # constant variants of one shape (a steady-mode polish batch)
        from funsearch_kubernetes_simulator_amd.funsearch.polish import _perturb, tunable_literals, with_values
        import random
        rng = random.Random(args.seed)
        base_p = progs[0]
        tune = tunable_literals(base_p)
        vals = {base_p.literals[j][0]: (base_p.fconst[base_p.literals[j][0]] if base_p.ctag[base_p.literals[j][0]] == 1
                                        else base_p.iconst[base_p.literals[j][0]]) for j in range(len(base_p.literals))}
        progs = [with_values(base_p, _perturb(base_p, vals, tune, 0.35, rng)) for _ in range(len(progs))]
    dev.native_compiler.tier = "baseline"
    t0 = time.perf_counter()
    for i in range(0, len(progs), args.batch):
        dev.evaluate_native(progs[i:i + args.batch])
    first = time.perf_counter() - t0
    best = None
    for _ in range(args.reps):
        t0 = time.perf_counter()
        rows = [dev.evaluate_native(progs[i:i + args.batch]) for i in range(0, len(progs), args.batch)]
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    tab = np.concatenate(rows)
    print(json.dumps({"variant": args.name, "rows": args.rows, "polish": args.polish, "programs": len(progs),
                      "batch": args.batch,
                      "first_pass_s": round(first, 3), "cached_s": round(best, 3),
                      "cached_evals_per_s": round(len(progs) / best, 1),
                      "exc_rows": int((tab[:, 10] != 0).sum()), "mean_events": float(tab[:, 8].mean()),
                      # every replayed program-event (first pass + reps): the PMC summary's denominator
                      "events": float(tab[:, 8].sum()) * (1 + args.reps),
                      "jit": {k: v for k, v in dev.native_compiler.stats.items()
                              if k in ("baseline_shapes", "rejected", "compile_s", "load_s")}}), flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ck", default="data/populations/config3_steady_r4f_islands.json")
    ap.add_argument("--children", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--variant", action="append", default=[], help="NAME=ENV1=V1,ENV2=V2 (empty: no change)")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--name", default="base")
    ap.add_argument("--rows", type=int, default=0, help="native programs per wave (0: the two-wave kernel)")
    ap.add_argument("--polish", action="store_true", help="constant variants of one program instead of children")
    ap.add_argument("--sources", default="", help="JSON list of program sources to run instead of fresh children")
    ap.add_argument("--save-sources", default="", help="write the children's sources (JSON) and exit (no GPU)")
    args = ap.parse_args()
    if args.save_sources:
        progs = _programs(args.ck, args.children, args.seed)
        json.dump([p.source for p in progs], open(args.save_sources, "w"))
        print(json.dumps({"saved": len(progs), "file": args.save_sources}))
        return
    if args.child:
        child(args)
        return
    for spec in args.variant or ["base="]:
        name, _, envs = spec.partition("=")
        env = dict(os.environ)
        for kv in filter(None, envs.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        cmd = [sys.executable, "-u", os.path.abspath(__file__), "--child", "--name", name, "--ck", args.ck,
               "--sources", args.sources,
               "--children", str(args.children), "--batch", str(args.batch), "--reps", str(args.reps),
               "--seed", str(args.seed), "--rows", str(args.rows)] + (["--polish"] if args.polish else [])
        r = subprocess.run(cmd, env=env, timeout=600)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
