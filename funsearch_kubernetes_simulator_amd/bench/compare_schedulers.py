"""Scheduler comparison harness (the reference README table).

Twin of the reference's `SchedulerTester.compare_all_schedulers`
(`tests/test_scheduler.py:223-361`): replays first-fit, best-fit and the three
published FunSearch champions -- plus every policy under
``data/policies/discovered`` -- on the default trace and prints utilisation,
fragmentation and score per policy.  Scores come from the exact engines
(`engine.Evaluator`: MI355X when visible, else the native CPU VM); `--object`
additionally times the CPython object engine (the reference's own algorithm)
for each policy, the number the reference reports as "simulation time".

    python -m funsearch_kubernetes_simulator_amd.bench.compare_schedulers [--device cpu] [--object]
"""

from __future__ import annotations

import argparse
import json
import time
from typing import Dict, List

from ..core import load_default_workload
from ..engine import Evaluator, object_engine_eval
from ..models.library import discovered_policies, reference_policies, reference_scores


def collect(include_discovered: bool = True) -> Dict[str, str]:
    progs = dict(reference_policies())
    if include_discovered:
        for name, rec in discovered_policies().items():
            progs[name] = rec["code"]
    return progs


def compare(device="auto", object_engine: bool = False, include_discovered: bool = True) -> List[dict]:
    w = load_default_workload()
    progs = collect(include_discovered)
    ev = Evaluator(w, device=device)
    t0 = time.perf_counter()
    res = ev.evaluate_programs(list(progs.values()))
    batch_s = time.perf_counter() - t0
    ref = reference_scores()
    rows = []
    for (name, code), r in zip(progs.items(), res):
        row = {"policy": name, "score": r.score, "engine": r.engine, "exc": r.exc, "events": r.n_events}
        if r.results is not None:
            e = r.results
            row.update(cpu=e.avg_cpu_utilization, mem=e.avg_memory_utilization,
                       gpu=e.avg_gpu_count_utilization, gpu_milli=e.avg_gpu_memory_utilization,
                       frag=e.gpu_fragmentation_score, snapshots=e.num_snapshots,
                       frag_events=e.num_fragmentation_events)
        if name in ref:
            row["reference_score"] = ref[name]
            row["matches_reference"] = r.score == ref[name]
        if object_engine:
            t = time.perf_counter()
            o = object_engine_eval(code, w)
            row["object_engine_s"] = time.perf_counter() - t
            row["object_engine_score"] = o.score
        rows.append(row)
    for row in rows:
        row["batch_eval_s"] = batch_s
    return rows


def format_table(rows: List[dict]) -> str:
    hdr = f"{'Policy':<40} {'Score':>8} {'CPU%':>6} {'Mem%':>6} {'GPU%':>6} {'GPUm%':>6} {'Frag':>6} {'Snap':>5} {'FragEv':>7}  engine"
    lines = [hdr, "-" * len(hdr)]
    for r in rows:
        if "cpu" in r:
            lines.append(f"{r['policy'][:40]:<40} {r['score']:>8.4f} {100 * r['cpu']:>6.1f} {100 * r['mem']:>6.1f} "
                         f"{100 * r['gpu']:>6.1f} {100 * r['gpu_milli']:>6.1f} {r['frag']:>6.3f} {r['snapshots']:>5d} "
                         f"{r['frag_events']:>7d}  {r['engine']}")
        else:
            lines.append(f"{r['policy'][:40]:<40} {r['score']:>8.4f}  (exception {r['exc']})  {r['engine']}")
    return "\n".join(lines)


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--device", default="auto")
    ap.add_argument("--object", action="store_true", help="also time the CPython object engine per policy")
    ap.add_argument("--no-discovered", action="store_true")
    ap.add_argument("--json", default="", help="write the rows as JSON")
    a = ap.parse_args(argv)
    device = int(a.device) if a.device.isdigit() else a.device
    rows = compare(device, a.object, not a.no_discovered)
    print(format_table(rows))
    bad = [r["policy"] for r in rows if r.get("matches_reference") is False]
    print(f"\nreference scores reproduced bit-exactly: {'NO ' + str(bad) if bad else 'yes'}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=2)


if __name__ == "__main__":
    main()
