"""`SimpleFunSearch`: the reference's evolution loop on the batched engines.

Semantics follow `funsearch/funsearch_integration.py:124-679`:
seed population = first-fit + best-fit; each generation keeps the top
``elite_size`` programs, asks the LLM for ``min(8, population_size - elites)``
children (two random elite parents each, threads for LLM I/O), evaluates them,
drops children that are >= 85 % similar (difflib) to an equal-or-better member
of the *current* population, and keeps the top ``population_size`` of
elites + children (non-elites are discarded); early stop at
``early_stop_threshold``; results saved with the reference's JSON schema.

What changes underneath: children are evaluated in ONE batched call
(`engine.Evaluator`: MI355X k_replay waves, native CPU VM, exact fallbacks)
instead of a ProcessPoolExecutor that re-parses the trace per program, and
results are merged in candidate order (deterministic) rather than completion
order.  Extensions (all optional config keys): ``funsearch.policies_per_generation``
(overrides the hard-coded 8), an ``llm`` section selecting the backend
(``mutation`` for offline runs), ``checkpoint`` (periodic JSON checkpoints +
`resume`), and a JSONL metrics log.
"""

from __future__ import annotations

import concurrent.futures
import difflib
import json
import os
import random
import threading
import time
from datetime import datetime
from typing import List, Optional, Tuple

from .._paths import REPO_DIR
from ..engine import EvalResult, Evaluator
from ..models.library import seed_policies
from ..policy.sandbox import SafeExecutor
from ..utils.metrics import MetricsLog
from .generator import LLMCodeGenerator
from .llm import make_client
from .scheduler import FunSearchScheduler


def _difflib_at_least(a: str, b: str, threshold: float) -> bool:
    return difflib.SequenceMatcher(None, a, b).ratio() >= threshold


try:
    from ..ops._fks_cpu import similar_at_least as _similar_at_least
    from ..ops._fks_cpu import similar_to_any as _similar_to_any
except ImportError:  # native CPU module not built: the reference's own difflib path
    _similar_at_least = _difflib_at_least

    def _similar_to_any(a: str, bs, threshold: float, threads: int = 1) -> int:
        for i, b in enumerate(bs):
            if _difflib_at_least(a, b, threshold):
                return i
        return -1

FEEDBACK = ("Elite policies achieve good performance by balancing resource utilization "
            "and considering GPU/CPU workload separation. "
            "Focus on: CPU/mem/GPU util, efficiency, GPU placement strategies, fragmentation reduction.")


def load_config(config_path) -> dict:
    if isinstance(config_path, dict):
        return json.loads(json.dumps(config_path))
    p = str(config_path)
    if not os.path.exists(p) and os.path.exists(os.path.join(REPO_DIR, p)):
        p = os.path.join(REPO_DIR, p)
    with open(p) as fh:
        return json.load(fh)


class SimpleFunSearch:
    def __init__(self, config_path="configs/llm_config.json", evaluator: Optional[Evaluator] = None,
                 llm_client=None, seed: Optional[int] = None, verbose: bool = True):
        self.config = load_config(config_path)
        self.verbose = verbose
        self.safe_executor = SafeExecutor(timeout_seconds=self.config.get("safe_execution", {}).get("timeout_seconds", 3))
        llm_cfg = dict(self.config.get("llm") or {})
        if not llm_cfg:
            llm_cfg = dict(self.config.get("openrouter", {}))
            llm_cfg.setdefault("backend", "openai")
        self.llm_client = llm_client or make_client(llm_cfg)
        self.model = llm_cfg.get("model")
        self.code_generator = LLMCodeGenerator(self.llm_client, self.safe_executor, self.model,
                                               llm_cfg.get("max_tokens", 400), llm_cfg.get("temperature", 0.7))
        fs = self.config["funsearch"]
        self.population_size = fs["population_size"]
        self.max_generations = fs["generations"]
        self.early_stop_threshold = fs["early_stop_threshold"]
        self.elite_size = fs["elite_size"]
        self.similarity_threshold = fs.get("similarity_threshold", 0.85)
        #: host threads for one child's similarity scan against the population
        self.similarity_threads = int(fs.get("similarity_threads", 4))
        self.max_workers = fs.get("max_workers", 8)
        self.policies_per_generation = fs.get("policies_per_generation", 8)
        self.print_lock = threading.Lock()
        self.rng = random.Random(seed)
        dev = (self.config.get("device") or {}).get("kind", "auto")
        self.evaluator = evaluator or Evaluator(device=dev)
        self.population: List[Tuple[str, float]] = []
        self.generation = 0
        self.best_policy: Optional[str] = None
        self.best_score = float("-inf")
        self.evaluations = 0
        ck = self.config.get("checkpoint") or {}
        self.checkpoint_dir = ck.get("dir")
        self.checkpoint_every = int(ck.get("every", 0))
        self.log = MetricsLog(self.config.get("log_path"))

    def _print(self, *a, **k) -> None:
        if self.verbose:
            with self.print_lock:
                print(*a, **k)

    # -- evaluation ------------------------------------------------------------------
    def _evaluate_policy_full(self, policy_code: str) -> Optional[float]:
        """In-process evaluation; None on any failure (reference `:433-459`)."""
        r = self.evaluator.evaluate_programs([policy_code])[0]
        self.evaluations += 1
        return None if r.exc else r.score

    def evaluate_batch(self, codes: List[str]) -> List[EvalResult]:
        self.evaluations += len(codes)
        return self.evaluator.evaluate_programs(codes)

    # -- population ----------------------------------------------------------------------
    def initialize_population(self) -> None:
        seeds = seed_policies()
        baseline = [seeds["first_fit"], seeds["best_fit"]]
        # optional extra seeds (not in the reference): "discovered" = the policies
        # under data/policies/discovered, "reference" = the published champions,
        # or any seed/library policy name
        for extra in self.config.get("funsearch", {}).get("extra_seeds", []) or []:
            if extra == "discovered":
                from ..models.library import discovered_policies
                baseline += [r["code"] for r in discovered_policies().values()]
            elif extra == "reference":
                from ..models.library import reference_policies
                baseline += [c for n, c in reference_policies().items() if n.startswith("funsearch")]
            else:
                from ..models.library import policy
                baseline.append(policy(extra))
        self._print("Evaluating baseline policies on OpenB dataset...")
        for i, code in enumerate(baseline):
            score = self._evaluate_policy_full(code)
            if score is not None:
                self.population.append((code, score))
                if score > self.best_score:
                    self.best_score, self.best_policy = score, code
            self._print(f"Evaluating baseline policy {i + 1}/{len(baseline)}... " +
                        (f"Score: {score:.4f}" if score else "Failed"))
        self.population.sort(key=lambda x: x[1], reverse=True)
        self.population = self.population[:self.population_size]
        self._print(f"Initialized population with {len(self.population)} policies")
        self._print(f"Best baseline score: {self.best_score:.4f}")

    def _is_too_similar(self, new_code: str, new_score: float) -> bool:
        """Reference `_is_too_similar` (difflib ratio against every member that
        scores at least as well).  The ratio comes from the native exact
        SequenceMatcher (`csrc/cpu/seqmatch.hpp`, ~40x faster) when built."""
        a = new_code.strip()
        others = [code.strip() for code, score in self.population if score >= new_score]
        return bool(others) and _similar_to_any(a, others, self.similarity_threshold,
                                                self.similarity_threads if len(others) > 2 else 1) >= 0

    def _generate_single_policy(self, idx: int, elites, feedback: str) -> Tuple[int, Optional[str]]:
        with self.print_lock:
            parents = self.rng.sample(elites, min(2, len(elites)))
        code = self.code_generator.generate_policy(parent_policies=parents, performance_feedback=feedback)
        self._print(f"Policy {idx + 1}: " + ("Generated successfully" if code else "Generation failed"))
        return idx, code

    def evolve_generation(self) -> None:
        t0 = time.time()
        self.generation += 1
        self._print(f"\n--- Generation {self.generation} ---")
        self.population.sort(key=lambda x: x[1], reverse=True)
        elites = self.population[:self.elite_size]
        n_new = min(self.policies_per_generation, self.population_size - len(elites))
        if n_new <= 0 or not elites:
            self._print("No new policies to generate")
            return
        self._print(f"Generating {n_new} policies in parallel...")
        with concurrent.futures.ThreadPoolExecutor(max_workers=self.max_workers) as ex:
            gen = list(ex.map(lambda i: self._generate_single_policy(i, elites, FEEDBACK), range(n_new)))
        generated = [(i, c) for i, c in sorted(gen) if c]
        if not generated:
            self._print("No policies generated successfully")
            return
        t_gen = time.time()
        self._print(f"Generated {len(generated)} policies successfully")
        results = self.evaluate_batch([c for _, c in generated])
        t_eval = time.time()
        new: List[Tuple[str, float]] = []
        for (idx, code), res in zip(generated, results):
            score = res.score
            if self._is_too_similar(code, score):
                self._print(f"Policy {idx + 1}: Score {score:.4f} - Too similar, skipped")
                continue
            new.append((code, score))
            if score > self.best_score:
                self.best_score, self.best_policy = score, code
                self._print(f"NEW BEST! Policy {idx + 1} Score: {score:.4f}")
            else:
                self._print(f"Policy {idx + 1}: Score {score:.4f}")
        merged = sorted(elites + new, key=lambda x: x[1], reverse=True)
        self.population = merged[:self.population_size]
        self._print(f"Generation complete: {len(new)} new policies evaluated")
        self._print(f"Population: {len(self.population)} policies, best score: {self.best_score:.4f}")
        self.log.write(kind="generation", generation=self.generation, best=self.best_score,
                       population=len(self.population), generated=len(generated), accepted=len(new),
                       llm_s=round(t_gen - t0, 4), eval_s=round(t_eval - t_gen, 4),
                       evals_per_s=round(len(generated) / max(1e-9, t_eval - t_gen), 2))
        if self.checkpoint_dir and self.checkpoint_every and self.generation % self.checkpoint_every == 0:
            self.save_checkpoint()

    def run_evolution(self, generations: Optional[int] = None) -> Tuple[str, float]:
        generations = generations or self.max_generations
        self._print("Starting FunSearch evolution...")
        if not self.population:
            self.initialize_population()
        for _ in range(generations):
            t0 = time.time()
            self.evolve_generation()
            self._print(f"Generation {self.generation} completed in {time.time() - t0:.1f}s")
            if self.best_score >= self.early_stop_threshold:
                self._print(f"Reached target score ({self.best_score:.4f}), stopping early")
                break
        self._print(f"Evolution complete! Best score: {self.best_score:.4f}")
        return self.best_policy, self.best_score

    def get_best_scheduler(self) -> FunSearchScheduler:
        if not self.best_policy:
            raise ValueError("No evolved policy available. Run evolution first.")
        return FunSearchScheduler(self.best_policy, self.safe_executor)

    # -- persistence (reference JSON schema) ---------------------------------------------
    def save_best_policy(self, filepath: Optional[str] = None) -> str:
        if not self.best_policy:
            raise ValueError("No best policy to save")
        ts = datetime.now().strftime("%Y%m%d_%H%M%S")
        if filepath is None:
            os.makedirs("policies/discovered", exist_ok=True)
            filepath = f"policies/discovered/funsearch_{ts}_score{self.best_score:.4f}.json"
        else:
            base, ext = os.path.splitext(filepath)
            filepath = f"{base}_{ts}{ext}"
        with open(filepath, "w") as fh:
            json.dump({"score": self.best_score, "generation": self.generation, "code": self.best_policy,
                       "timestamp": datetime.now().isoformat()}, fh, indent=2)
        self._print(f"Best policy saved to {filepath}")
        return filepath

    def save_top_policies(self, top_k: int = 5, filepath: Optional[str] = None) -> str:
        if not self.population:
            raise ValueError("No policies to save")
        self.population.sort(key=lambda x: x[1], reverse=True)
        top = self.population[:min(top_k, len(self.population))]
        best = top[0][1] if top else 0
        if filepath is None:
            os.makedirs("policies/discovered", exist_ok=True)
            ts = datetime.now().strftime("%Y%m%d_%H%M%S")
            filepath = f"policies/discovered/funsearch_top{top_k}_{ts}_best{best:.4f}.json"
        now = datetime.now().isoformat()
        data = {"top_k": top_k, "generation": self.generation, "best_score": best, "timestamp": now,
                "policies": [{"rank": i, "score": s, "generation": self.generation, "code": c, "timestamp": now}
                             for i, (c, s) in enumerate(top, 1)]}
        with open(filepath, "w") as fh:
            json.dump(data, fh, indent=2)
        self._print(f"Top {len(top)} policies saved to {filepath}")
        for i, (_, s) in enumerate(top, 1):
            self._print(f"  Rank {i}: {s:.4f}")
        return filepath

    # -- checkpoint / resume (new) ----------------------------------------------------------
    def state_dict(self) -> dict:
        return {"format": "fks-funsearch-checkpoint-v1", "generation": self.generation,
                "population": [{"code": c, "score": s} for c, s in self.population],
                "best_policy": self.best_policy, "best_score": self.best_score,
                "evaluations": self.evaluations, "rng_state": repr(self.rng.getstate()),
                "timestamp": datetime.now().isoformat()}

    def save_checkpoint(self, path: Optional[str] = None) -> str:
        path = path or os.path.join(self.checkpoint_dir or ".", f"checkpoint_gen{self.generation:06d}.json")
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        tmp = path + ".tmp"
        with open(tmp, "w") as fh:
            json.dump(self.state_dict(), fh)
        os.replace(tmp, path)   # atomic: a crash never leaves a torn checkpoint
        return path

    def load_checkpoint(self, path: str) -> None:
        with open(path) as fh:
            st = json.load(fh)
        if st.get("format") != "fks-funsearch-checkpoint-v1":
            raise ValueError(f"not a checkpoint: {path}")
        self.generation = int(st["generation"])
        self.population = [(p["code"], float(p["score"])) for p in st["population"]]
        self.best_policy, self.best_score = st["best_policy"], float(st["best_score"])
        self.evaluations = int(st.get("evaluations", 0))
        import ast as _ast
        try:
            self.rng.setstate(_ast.literal_eval(st["rng_state"]))
        except Exception:
            pass

    @staticmethod
    def latest_checkpoint(directory: str) -> Optional[str]:
        if not directory or not os.path.isdir(directory):
            return None
        cks = sorted(f for f in os.listdir(directory) if f.startswith("checkpoint_gen") and f.endswith(".json"))
        return os.path.join(directory, cks[-1]) if cks else None
