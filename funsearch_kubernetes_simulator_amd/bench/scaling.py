"""Scaling curve of the headline benchmark (BASELINE config 4: evals/s at
1/2/4/8 GPUs of one node).

Runs ``bench.py`` once per GPU count -- one rank per GPU through
``torch.distributed.run`` (RCCL over xGMI; gloo with ``--device cpu``) -- and
prints each run's JSON line plus a summary with the weak-scaling efficiency
``value_N / (N * value_1)``.  Each run is a separate child process, so a
failing size does not take the others down; sizes above the visible GPU count
are skipped.

    python -m funsearch_kubernetes_simulator_amd.bench.scaling --gpus 1,2,4,8 -- --steps 10 --warmup 2

Arguments after ``--`` go to every ``bench.py`` run unchanged.
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
from typing import List, Optional

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench_cmd(n: int, port: int, extra: List[str]) -> List[str]:
    bench = os.path.join(REPO, "bench.py")
    if n == 1:
        return [sys.executable, bench, "--gpus", "1"] + extra
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), bench, "--gpus", str(n)] + extra


def run_size(n: int, port: int, extra: List[str], timeout: float) -> Optional[dict]:
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    r = subprocess.run(bench_cmd(n, port, extra), env=env, capture_output=True, text=True, timeout=timeout)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not lines:
        sys.stderr.write(f"[scaling] N={n} failed (rc={r.returncode}):\n{r.stderr[-2000:]}\n")
        return None
    return json.loads(lines[-1])


def summarize(results: dict) -> List[dict]:
    """Rows {n_gpus, value, ms_per_step, efficiency} (efficiency vs N=1, weak scaling)."""
    base = results.get(1)
    rows = []
    for n in sorted(results):
        rec = results[n]
        if rec is None:
            rows.append({"n_gpus": n, "value": None, "ms_per_step": None, "efficiency": None})
            continue
        eff = rec["value"] / (n * base["value"]) if base else None
        cfg = rec.get("config", {})
        rows.append({"n_gpus": n, "value": rec["value"], "ms_per_step": rec["ms_per_step"],
                     "efficiency": None if eff is None else round(eff, 4),
                     "dist_backend": cfg.get("dist_backend"), "world_size": cfg.get("world_size")})
    return rows


def visible_gpus() -> int:
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    extra: List[str] = []
    if "--" in argv:
        k = argv.index("--")
        argv, extra = argv[:k], argv[k + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1,2,4,8", help="comma-separated rank counts")
    ap.add_argument("--port", type=int, default=29600)
    ap.add_argument("--timeout", type=float, default=1800.0, help="seconds per size")
    a = ap.parse_args(argv)
    sizes = [int(s) for s in a.gpus.split(",") if s.strip()]
    cpu = "--device" in extra and extra[extra.index("--device") + 1] == "cpu"
    if not cpu:
        have = visible_gpus()
        skipped = [n for n in sizes if n > have]
        if skipped:
            sys.stderr.write(f"[scaling] {have} GPU(s) visible: skipping N={skipped}\n")
        sizes = [n for n in sizes if n <= have]
    results = {}
    for i, n in enumerate(sizes):
        results[n] = run_size(n, a.port + i, extra, a.timeout)
        if results[n] is not None:
            print(json.dumps(results[n]), flush=True)
    rows = summarize(results)
    print(json.dumps({"scaling": rows}), flush=True)
    return 0 if all(r["value"] is not None for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
