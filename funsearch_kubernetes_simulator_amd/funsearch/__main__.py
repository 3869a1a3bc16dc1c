"""CLI: multi-island FunSearch.

    python -m funsearch_kubernetes_simulator_amd.funsearch --config configs/offline_islands.json \
        --generations 200 [--islands 4] [--migrate-every 50] [--resume] [--save top5.json]
    torchrun --nproc-per-node 8 -m funsearch_kubernetes_simulator_amd.funsearch ...   # 1 rank per GPU
"""
import argparse
import json

from ..parallel import dist
from .islands import IslandFunSearch
from .search import load_config


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="configs/offline_islands.json")
    ap.add_argument("--generations", type=int)
    ap.add_argument("--islands", type=int)
    ap.add_argument("--migrate-every", type=int)
    ap.add_argument("--policies-per-generation", type=int)
    ap.add_argument("--device", choices=["auto", "cpu", "gpu"])
    ap.add_argument("--resume", action="store_true")
    ap.add_argument("--checkpoint-dir")
    ap.add_argument("--log", "--metrics-log", dest="log",
                    help="JSONL metrics path (--metrics-log under torchrun, whose parser claims --log)")
    ap.add_argument("--save", help="write the top-5 JSON (reference schema) here")
    ap.add_argument("--device-min-batch", type=int,
                    help="smallest program batch sent to the device VM (smaller ones run on the CPU VM)")
    ap.add_argument("--wall-s", type=float, help="steady mode: stop after this many seconds (ranks agree)")
    ap.add_argument("--mode", choices=["sync", "pipeline", "steady"], help="island loop (overrides islands.mode)")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    cfg = load_config(a.config)
    isl = cfg.setdefault("islands", {})
    if a.islands:
        isl["per_rank"] = a.islands
    if a.migrate_every:
        isl["migrate_every"] = a.migrate_every
    if a.policies_per_generation:
        cfg["funsearch"]["policies_per_generation"] = a.policies_per_generation
    if a.device:
        cfg.setdefault("device", {})["kind"] = a.device
    if a.mode:
        isl["mode"] = a.mode
        isl["pipeline"] = a.mode == "pipeline"
    if a.wall_s is not None:
        isl.setdefault("steady", {})["wall_s"] = a.wall_s
    if a.device_min_batch is not None:
        cfg.setdefault("device", {})["min_batch"] = a.device_min_batch
    if a.checkpoint_dir:
        cfg.setdefault("checkpoint", {})["dir"] = a.checkpoint_dir
    if a.log:
        cfg["log_path"] = a.log
    run = IslandFunSearch(cfg, verbose=a.verbose)
    code, score = run.run(a.generations, resume=a.resume)
    if run.ctx.is_main:
        best_isl = max(run.islands, key=lambda s: s.best_score)
        if a.save:
            best_isl.save_top_policies(5, a.save)
        print(json.dumps({"best_score": score, "generations": run.generation, "evaluations": run.evaluations,
                          "ranks": run.ctx.world_size, "islands_per_rank": run.n_islands,
                          "engine_stats": run.evaluator.stats}))
    dist.shutdown()


if __name__ == "__main__":
    main()
