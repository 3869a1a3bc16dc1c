"""Sandbox, template/prompt, LLM backends, SimpleFunSearch semantics, islands, checkpoints."""
import json
import os

import pytest

from funsearch_kubernetes_simulator_amd.core.model import GPU, Node, Pod
from funsearch_kubernetes_simulator_amd.funsearch import (FunSearchScheduler, LLMCodeGenerator, MutationClient,
                                                          ScriptedClient, SimpleFunSearch, evaluate_policy_standalone,
                                                          run_funsearch)
from funsearch_kubernetes_simulator_amd.models.library import reference_scores, seed_policies
from funsearch_kubernetes_simulator_amd.policy.sandbox import SafeExecutor
from funsearch_kubernetes_simulator_amd.policy.template import PolicyTemplate

REF = "/root/reference/funsearch/safe_execution.py"


class _Obj:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def test_safe_execution_basics():
    ex = SafeExecutor(timeout_seconds=1)
    ok = "def priority_function(pod, node):\n    score = 0.0\n    if node.cpu_milli_left >= pod.cpu_milli:\n        score = 100.0\n    return score\n"
    assert ex.execute_policy_function(ok, _Obj(cpu_milli=100), _Obj(cpu_milli_left=200)) == 100.0
    with pytest.raises(ValueError):
        ex.execute_policy_function("import os\ndef priority_function(pod, node):\n    return 1.0\n", _Obj(), _Obj())
    with pytest.raises(ValueError):   # substring blacklist quirk: 'dir' in 'direction'
        ex.validate_code_content("direction = 1")
    with pytest.raises(ValueError):
        ex.validate_code_structure("def priority_function(pod, node):\n    return eval('1')\n")
    env = ex.create_safe_environment()
    assert set(env["__builtins__"]) <= SafeExecutor.ALLOWED_BUILTINS
    assert env["math"].sqrt(4) == 2.0


@pytest.mark.skipif(not os.path.exists(REF), reason="reference checkout not mounted")
def test_template_and_prompt_verbatim_vs_reference():
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_safe", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert PolicyTemplate.TEMPLATE == mod.PolicyTemplate.TEMPLATE
    parents = [("def priority_function(pod, node):\n    return 1\n", 0.4321), ("code2", 0.1)]
    assert (PolicyTemplate.create_prompt_for_llm(parents, "fb") ==
            mod.PolicyTemplate.create_prompt_for_llm(parents, "fb"))
    assert PolicyTemplate.create_prompt_for_llm([], "") == mod.PolicyTemplate.create_prompt_for_llm([], "")


def test_generator_fills_template_and_validates():
    gen = LLMCodeGenerator(ScriptedClient(["```python\n    score = node.cpu_milli_left * 0.01\n```",
                                           "    import os"]))
    code = gen.generate_policy([], "")
    assert code is not None and "score = node.cpu_milli_left * 0.01" in code
    assert PolicyTemplate.extract_logic(code).strip() == "score = node.cpu_milli_left * 0.01"
    assert gen.generate_policy([], "") is None      # forbidden pattern rejected


def test_mutation_client_produces_valid_programs():
    gen = LLMCodeGenerator(MutationClient(seed=1))
    parents = [(seed_policies()["best_fit"], 0.44), (seed_policies()["first_fit"], 0.43)]
    ok = 0
    for _ in range(30):
        code = gen.generate_policy(parents, "fb")
        if code:
            compile(code, "<p>", "exec")
            ok += 1
    assert ok >= 20


def test_scheduler_reraises():
    sched = FunSearchScheduler("def priority_function(pod, node):\n    return 1 / 0\n")
    pod = Pod("p", 1, 1, 0, 0, "", 0, 1)
    node = Node("n", 10, 10, 10, 10, 0, [])
    with pytest.raises(ZeroDivisionError):
        sched(pod, node)
    assert FunSearchScheduler("def priority_function(pod, node):\n    return -5.5\n")(pod, node) == 0


def test_evaluate_policy_standalone():
    idx, code, score = evaluate_policy_standalone((3, seed_policies()["first_fit"]))
    assert (idx, score) == (3, reference_scores()["first_fit"])
    assert evaluate_policy_standalone((4, "not python"))[2] == 0


def _cfg(tmp_path, **fs):
    base = {"population_size": 6, "generations": 3, "early_stop_threshold": 1.0, "elite_size": 3,
            "max_workers": 2, "policies_per_generation": 4}
    base.update(fs)
    return {"llm": {"backend": "mutation", "seed": 5}, "safe_execution": {"timeout_seconds": 3},
            "funsearch": base, "device": {"kind": "cpu"},
            "checkpoint": {"dir": str(tmp_path / "ck"), "every": 1}, "log_path": str(tmp_path / "log.jsonl")}


def test_simple_funsearch_semantics(tmp_path):
    fs = SimpleFunSearch(_cfg(tmp_path), verbose=False, seed=0)
    fs.initialize_population()
    assert [round(s, 6) for _, s in fs.population] == [0.446548, 0.429206]
    fs.run_evolution(2)
    assert fs.generation == 2
    assert len(fs.population) <= 6
    assert fs.best_score >= reference_scores()["best_fit"]
    # reference JSON schema
    top = json.load(open(fs.save_top_policies(3, str(tmp_path / "top.json"))))
    assert set(top) == {"top_k", "generation", "best_score", "timestamp", "policies"}
    assert set(top["policies"][0]) == {"rank", "score", "generation", "code", "timestamp"}
    best = json.load(open(fs.save_best_policy(str(tmp_path / "best.json"))))
    assert set(best) == {"score", "generation", "code", "timestamp"}
    # checkpoints + resume
    ck = SimpleFunSearch.latest_checkpoint(str(tmp_path / "ck"))
    fs2 = SimpleFunSearch(_cfg(tmp_path), verbose=False)
    fs2.load_checkpoint(ck)
    assert fs2.generation == fs.generation and fs2.population == fs.population
    logs = [json.loads(l) for l in open(tmp_path / "log.jsonl")]
    assert logs and logs[-1]["kind"] == "generation"


def test_dedup_rule(tmp_path):
    fs = SimpleFunSearch(_cfg(tmp_path), verbose=False)
    code = seed_policies()["best_fit"]
    fs.population = [(code, 0.5)]
    assert fs._is_too_similar(code + "\n", 0.4)        # worse and near-identical -> skip
    assert not fs._is_too_similar(code + "\n", 0.6)    # better -> kept


def test_run_funsearch_islands_cpu(tmp_path):
    cfg = _cfg(tmp_path)
    cfg["islands"] = {"per_rank": 2, "migrate_every": 1, "migrants": 1}
    code, score = run_funsearch(cfg, generations=2)
    assert score >= reference_scores()["best_fit"]
    assert "def priority_function" in code
    assert os.path.exists(tmp_path / "ck" / "islands_rank0.json")


def test_runaway_program_is_bounded():
    """`while True` stops on the VM call budget, then on the object engine's wall clock."""
    import numpy as np
    from funsearch_kubernetes_simulator_amd.core import load_default_workload
    from funsearch_kubernetes_simulator_amd.core.arrays import Workload
    from funsearch_kubernetes_simulator_amd.engine import Evaluator
    from funsearch_kubernetes_simulator_amd.policy.bytecode import Exc
    w = load_default_workload()
    sub = Workload(w.cluster, w.pods.subset(np.arange(0, 50)))
    ev = Evaluator(sub, device="cpu", options={"object_timeout_s": 1.0})
    code = "def priority_function(pod, node):\n    x = 0\n    while True:\n        x += 1\n    return 1\n"
    r = ev.evaluate_programs([code])[0]
    assert (r.score, r.exc, r.engine) == (0.0, int(Exc.BUDGET), "object")


def test_openai_compatible_client_retries_and_parses():
    """OpenAI-compatible HTTP backend against a local stub server: 503 is retried, 401 is not."""
    import http.server
    import threading
    from funsearch_kubernetes_simulator_amd.funsearch.llm import OpenAICompatibleClient
    seen = []

    class H(http.server.BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_POST(self):
            body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
            seen.append((self.path, self.headers.get("Authorization"), body["model"]))
            if body["model"] == "deny":
                self.send_response(401); self.end_headers(); self.wfile.write(b"no"); return
            if len(seen) == 1:
                self.send_response(503); self.end_headers(); return
            out = json.dumps({"choices": [{"message": {"content": "    score = 1.0"}}]}).encode()
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(out)))
            self.end_headers()
            self.wfile.write(out)

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        c = OpenAICompatibleClient("k123", f"http://127.0.0.1:{srv.server_address[1]}/v1", timeout_s=5,
                                   max_retries=2, backoff_s=0.01)
        r = c.chat.completions.create(model="m", messages=[{"role": "user", "content": "hi"}])
        assert r.choices[0].message.content == "    score = 1.0"
        assert seen[0] == ("/v1/chat/completions", "Bearer k123", "m") and len(seen) == 2
        n = len(seen)
        with pytest.raises(RuntimeError):
            c.chat.completions.create(model="deny", messages=[])
        assert len(seen) == n + 1      # not retried
    finally:
        srv.shutdown()


def test_search_survives_injected_faults(tmp_path):
    """Fault-injection hooks (LLM failures, failing evaluations) do not stop the search."""
    cfg = _cfg(tmp_path)
    cfg["islands"] = {"per_rank": 2, "migrate_every": 1, "migrants": 1}
    cfg["fault_injection"] = {"llm_failure_rate": 0.3, "eval_failure_rate": 0.3, "seed": 1}
    code, score = run_funsearch(cfg, generations=3)
    assert score >= reference_scores()["best_fit"]
    logs = [json.loads(l) for l in open(tmp_path / "log.jsonl")]
    assert logs[-1]["generation"] == 3


def _fake_island(codes_scores, gen):
    return {"format": "fks-funsearch-checkpoint-v1", "generation": gen,
            "population": [{"code": c, "score": s} for c, s in codes_scores],
            "best_policy": codes_scores[0][0], "best_score": codes_scores[0][1], "evaluations": 0}


def test_elastic_resume_reshards_islands(tmp_path):
    """A checkpoint written by 2 ranks x 2 islands resumes on 1 rank with 1
    island (populations merged) and with 8 islands (populations cloned)."""
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    seeds = seed_policies()
    ck = tmp_path / "ck"
    ck.mkdir()
    base = seeds["best_fit"]
    for r in range(2):
        isl = [_fake_island([(base + f"\n# r{r} i{i} a", 0.5 + 0.01 * (2 * r + i)),
                             (base + f"\n# r{r} i{i} b", 0.1)], 40) for i in range(2)]
        st = {"format": "fks-islands-checkpoint-v1", "generation": 40, "rank": r, "world_size": 2,
              "evaluations": 100, "islands": isl}
        (ck / f"islands_rank{r}.json").write_text(json.dumps(st))
    # stale file from an older, larger run must be ignored
    (ck / "islands_rank2.json").write_text(json.dumps(
        {"format": "fks-islands-checkpoint-v1", "generation": 10, "rank": 2, "world_size": 4, "islands": []}))
    cfg = _cfg(tmp_path)
    cfg["funsearch"]["population_size"] = 20
    cfg["islands"] = {"per_rank": 1, "migrate_every": 0}
    one = IslandFunSearch(cfg)
    assert one.load_elastic(str(ck))
    assert one.generation == 40 and one.evaluations == 200
    pop = one.islands[0].population
    assert len(pop) == 8 and pop[0][1] == 0.53 and one.islands[0].best_score == 0.53
    cfg["islands"]["per_rank"] = 8
    many = IslandFunSearch(cfg)
    assert many.load_elastic(str(ck))
    assert [round(s.best_score, 2) for s in many.islands] == [0.5, 0.51, 0.52, 0.53] * 2
    # a resumed run keeps evolving from there
    code, score = many.run(generations=1, resume=False)
    assert many.generation == 41 and score >= 0.53


def test_cli_elastic_resume_changes_island_count(tmp_path):
    """CLI: a 2-island run, then `--resume --islands 3` on the same checkpoint
    directory continues from its generation (islands re-sharded)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfgp = tmp_path / "cfg.json"
    cfgp.write_text(json.dumps(_cfg(tmp_path)))
    base = [sys.executable, "-m", "funsearch_kubernetes_simulator_amd.funsearch", "--config", str(cfgp),
            "--device", "cpu", "--checkpoint-dir", str(tmp_path / "ck"), "--metrics-log", str(tmp_path / "m.jsonl")]
    env = dict(os.environ, PYTHONPATH=repo, OMP_NUM_THREADS="2")
    r1 = subprocess.run(base + ["--islands", "2", "--generations", "2"], env=env, capture_output=True, text=True,
                        timeout=600)
    assert r1.returncode == 0, r1.stderr[-2000:]
    r2 = subprocess.run(base + ["--islands", "3", "--generations", "1", "--resume"], env=env, capture_output=True,
                        text=True, timeout=600)
    assert r2.returncode == 0, r2.stderr[-2000:]
    out = json.loads([l for l in r2.stdout.splitlines() if l.startswith("{")][-1])
    assert out["generations"] == 3 and out["islands_per_rank"] == 3
    assert out["best_score"] >= reference_scores()["best_fit"]
    assert len(json.loads((tmp_path / "ck" / "islands_rank0.json").read_text())["islands"]) == 3


def test_pipelined_islands_match_lockstep_with_one_worker(tmp_path):
    """Pipelined islands (each island steps on its own; LLM / JIT / device
    stages overlap across islands) keep every island's per-generation
    semantics: with one LLM worker (deterministic request order) and one
    island the populations equal the lock-step `evolve` loop's."""
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    pops = []
    for pipe in (False, True):
        cfg = _cfg(tmp_path, max_workers=1)
        cfg["islands"] = {"per_rank": 1, "migrate_every": 0, "migrants": 1, "pipeline": pipe}
        cfg["log_path"] = str(tmp_path / f"log{int(pipe)}.jsonl")
        cfg["checkpoint"] = {}
        fs = IslandFunSearch(cfg)
        fs.run(3)
        assert fs.generation == 3
        pops.append([(c, s) for c, s in fs.islands[0].population])
    assert pops[0] == pops[1]
    recs = [json.loads(l) for l in open(tmp_path / "log1.jsonl")]
    kinds = {r["kind"] for r in recs}
    assert {"island_generation", "generation"} <= kinds
    g = [r for r in recs if r["kind"] == "generation"]
    assert [r["generation"] for r in g] == [1, 2, 3] and all("device_busy" in r for r in g)


def test_pipelined_islands_migrate_at_barrier(tmp_path):
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    cfg = _cfg(tmp_path)
    cfg["islands"] = {"per_rank": 3, "migrate_every": 2, "migrants": 1, "pipeline": True}
    cfg["checkpoint"] = {"dir": str(tmp_path / "ck"), "every": 2}
    fs = IslandFunSearch(cfg)
    code, score = fs.run(4)
    assert fs.generation == 4 and score >= reference_scores()["best_fit"]
    recs = [json.loads(l) for l in open(tmp_path / "log.jsonl")]
    assert len([r for r in recs if r["kind"] == "island_generation"]) == 12
    assert (tmp_path / "ck" / "islands_rank0.json").exists()


def test_pipelined_islands_checkpoint_mid_run(tmp_path):
    """A due checkpoint holds idle islands back until all are between
    generations, so the file is written mid-run (not only by run()'s final
    save) and holds a consistent generation."""
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    cfg = _cfg(tmp_path)
    cfg["islands"] = {"per_rank": 3, "migrate_every": 0, "migrants": 1, "pipeline": True}
    cfg["checkpoint"] = {"dir": str(tmp_path / "ck"), "every": 2}
    fs = IslandFunSearch(cfg)
    saved = []
    orig = fs.save_checkpoint

    def spy():
        saved.append((fs.generation, [s.generation for s in fs.islands]))
        return orig()
    fs.save_checkpoint = spy
    fs.run(6)
    assert fs.generation == 6
    mid = [s for s in saved if s[0] < 6]
    assert mid, saved                                   # written before the last generation
    for g, per_island in mid:
        # every island between generations, none behind the completed global generation
        assert g % 2 == 0 and all(x >= g for x in per_island), saved
    st = json.load(open(tmp_path / "ck" / "islands_rank0.json"))
    assert st["generation"] == 6


def test_islands_with_constant_polish(tmp_path):
    """polish.every: island champions get a batched constant search; the
    rewritten program enters the population only with its exact re-score."""
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    cfg = _cfg(tmp_path)
    cfg["islands"] = {"per_rank": 2, "migrate_every": 0, "migrants": 1, "pipeline": True}
    cfg["polish"] = {"every": 1, "variants": 6, "rounds": 1}
    cfg["checkpoint"] = {}
    fs = IslandFunSearch(cfg)
    fs.run(2)
    recs = [json.loads(l) for l in open(tmp_path / "log.jsonl")]
    pol = [r for r in recs if r["kind"] == "polish"]
    assert pol and all(r["evaluated"] >= 6 for r in pol)
    for r in pol:
        if "rescored" in r:
            assert r["rescored"] == r["polished"]


def test_pipelined_polish_repeats_and_runs_in_the_island_pipeline(tmp_path):
    """polish.repeat: the champion is polished again at every due generation
    (fresh random variants), asynchronously inside the island's own pipeline
    step: every island still completes every generation, the polish records
    land in the log, and the evaluation count includes the variants."""
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    cfg = _cfg(tmp_path)
    cfg["islands"] = {"per_rank": 2, "migrate_every": 2, "migrants": 1, "pipeline": True}
    cfg["polish"] = {"every": 1, "variants": 4, "rounds": 1, "repeat": True}
    cfg["checkpoint"] = {}
    fs = IslandFunSearch(cfg)
    fs.run(3)
    assert fs.generation == 3
    recs = [json.loads(l) for l in open(tmp_path / "log.jsonl")]
    pol = [r for r in recs if r["kind"] == "polish"]
    assert len(pol) == 6                        # 2 islands x 3 generations, champions repeated
    assert len([r for r in recs if r["kind"] == "island_generation"]) == 6
    assert fs.evaluations >= sum(r["evaluated"] for r in pol)


@pytest.mark.parametrize("pipe", [False, True])
def test_family_coupling_feeds_program_islands(tmp_path, pipe):
    """coupling.every: a parametric family search (the reference's
    `_create_random_policy` family) runs beside the program islands; its
    champion is rendered as program text, re-scored through the normal program
    path (bit-identical to the family score) and injected into the island with
    the lowest best score; the coupler's state survives a checkpoint."""
    from funsearch_kubernetes_simulator_amd.engine import Evaluator
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    cfg = _cfg(tmp_path)
    cfg["islands"] = {"per_rank": 2, "migrate_every": 0, "migrants": 1, "pipeline": pipe}
    cfg["coupling"] = {"every": 1, "generations": 1, "candidates": 24, "elite": 4,
                       "families": ["random_linear"]}
    cfg["checkpoint"] = {"dir": str(tmp_path / "ck"), "every": 1}
    fs = IslandFunSearch(cfg)
    fs.run(2)
    recs = [json.loads(l) for l in open(tmp_path / "log.jsonl")]
    cp = [r for r in recs if r["kind"] == "coupling"]
    assert cp and all(r["family"] == "random_linear" for r in cp)
    assert all(r["score"] == r["family_score"] for r in cp)    # program text == family member, exactly
    assert fs.coupler.rounds >= 1 and fs.coupler.evaluated >= 24
    acc = [r for r in cp if r["accepted"]]
    if acc:
        pops = {c for s in fs.islands for c, _ in s.population}
        assert any("node.cpu_milli_left *" in c for c in pops)
    # checkpoint round trip of the coupler state
    fs.save_checkpoint()
    fs2 = IslandFunSearch(cfg, evaluator=Evaluator(device="cpu"))
    assert fs2.load_elastic(str(tmp_path / "ck"))
    isl1, isl2 = fs.coupler.islands["random_linear"], fs2.coupler.islands["random_linear"]
    assert fs2.coupler.rounds == fs.coupler.rounds
    assert (isl1.elite_scores == isl2.elite_scores).all() and (isl1.elites == isl2.elites).all()


def test_compile_workers_give_identical_results(default_workload):
    """device.compile_workers: bytecode compiles of a batch run in spawned
    worker processes (off the GIL of pipelined islands); same programs, same
    scores, rejected programs still counted."""
    from funsearch_kubernetes_simulator_amd.bench.programs import mutation_children
    from funsearch_kubernetes_simulator_amd.core.arrays import Workload
    from funsearch_kubernetes_simulator_amd.engine import Evaluator
    import numpy as np
    sub = Workload(default_workload.cluster, default_workload.pods.subset(np.arange(0, 400)))
    codes = [p.source for p in mutation_children(6, seed=11)] + ["def priority_function(pod, node):\n    import os\n"]
    a = Evaluator(sub, device="cpu")
    b = Evaluator(sub, device="cpu", options={"compile_workers": 2})
    ca, cb = a.compile_batch(codes), b.compile_batch(codes)
    assert [p is None for p in ca] == [p is None for p in cb] and cb[-1] is None
    assert all(x.code == y.code and x.source == y.source for x, y in zip(ca, cb) if x is not None)
    assert [r.score for r in a.evaluate_programs(codes)] == [r.score for r in b.evaluate_programs(codes)]
    assert b.stats["compile_errors"] == 2


class _DecliningDevice:
    """Stand-in for `DeviceEvaluator` whose native backend declines every
    program: its device VM answers with the CPU VM's rows, and every slot
    refuses a second batch while one is in flight (the real engine's rule)."""

    def __init__(self, workload, n_slots=5):
        import threading
        self.workload = workload
        self.n_slots = n_slots
        self.busy = {}
        self.lock = threading.Lock()
        self.vm_slots = []

    def _take(self, slot, payload):
        with self.lock:
            if slot in self.busy:
                raise RuntimeError(f"slot busy: wait() for its batch first (slot {slot})")
            self.busy[slot] = payload

    def prepare_native(self, progs):
        import numpy as np
        from funsearch_kubernetes_simulator_amd.ops.jit import NativeBatch
        n = len(progs)
        return NativeBatch(np.zeros(n, np.uint64), np.zeros(1, np.int64), np.zeros(n, np.int32),
                           np.zeros(n, bool), {i: "declined" for i in range(n)}, 0.0, 0)

    def release_native(self, batch):
        pass

    def submit_native(self, slot, progs, batch=None):
        import numpy as np
        n = len(progs)
        tab = np.zeros((n, 13))
        tab[:, 10] = 100.0                                   # EXC_UNSUPPORTED: not native
        self._take(slot, tab)
        return batch if batch is not None else self.prepare_native(progs)

    def ready(self, slot):
        return True

    def wait(self, slot):
        with self.lock:
            return self.busy.pop(slot)

    def evaluate_programs(self, progs, slot=None):
        from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
        assert slot is not None, "device VM fallback must run on the caller's slot"
        self.vm_slots.append(slot)
        self._take(slot, None)
        try:
            return ce.simulate_program_batch(self.workload, list(progs), threads=2)
        finally:
            self.wait(slot)


def test_pipelined_islands_native_declines_everything(tmp_path):
    """when the native backend declines a whole batch, the device
    VM fallback runs on the island's own slot (no 'slot busy' between
    pipelined islands), and every child still gets its exact score."""
    import numpy as np
    from funsearch_kubernetes_simulator_amd.core.arrays import Workload
    from funsearch_kubernetes_simulator_amd.core import load_default_workload
    from funsearch_kubernetes_simulator_amd.engine import Evaluator
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    w = load_default_workload()
    sub = Workload(w.cluster, w.pods.subset(np.arange(0, 600)))
    ev = Evaluator(sub, device="cpu", options={"device_min_batch": 1})
    ev.device = _DecliningDevice(sub)
    cfg = _cfg(tmp_path)
    cfg["islands"] = {"per_rank": 2, "migrate_every": 0, "migrants": 1, "pipeline": True}
    cfg["checkpoint"] = {}
    fs = IslandFunSearch(cfg, evaluator=ev)
    fs.run(2)
    assert fs.generation == 2
    assert ev.stats["device"] > 0 and ev.stats["device_native"] == 0
    assert set(ev.device.vm_slots) <= {0, 1} and len(set(ev.device.vm_slots)) == 2


def test_structural_mutations_compile_and_diversify():
    """The offline mutator's structural operators (feature-grammar terms,
    ast operator / aggregation swaps, subexpression crossover, wrapping)
    produce programs that compile and, unlike constant edits, new shapes."""
    import random
    from funsearch_kubernetes_simulator_amd.models.library import reference_policies
    from funsearch_kubernetes_simulator_amd.policy.compiler import try_compile
    from funsearch_kubernetes_simulator_amd.policy.native_codegen import shape_key
    c = MutationClient(9)
    parents = list(reference_policies().values()) + list(seed_policies().values())
    rng = random.Random(2)
    by_op, ok_by_op, shapes = {}, {}, set()
    for _ in range(600):
        pa = rng.sample(parents, 2)
        prompt = PolicyTemplate.create_prompt_for_llm([(pa[0], 0.45), (pa[1], 0.44)], "fb")
        body = c.chat.completions.create(model="m", messages=[{"role": "user", "content": prompt}]).choices[0].message.content
        op = c.last_op
        by_op[op] = by_op.get(op, 0) + 1
        prog, _ = try_compile(PolicyTemplate.fill_template(body))
        if prog is not None:
            ok_by_op[op] = ok_by_op.get(op, 0) + 1
            shapes.add(shape_key(prog))
    structural = ("random_term", "swap_binop", "swap_aggregate", "subexpr_crossover", "wrap")
    assert all(by_op.get(o, 0) > 0 for o in structural), by_op
    assert sum(ok_by_op.values()) >= 0.9 * 600, (by_op, ok_by_op)
    assert len(shapes) > 250       # constant-only edits would keep ~a dozen parent shapes


def test_island_reset_and_migrant_dedup(tmp_path):
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    cfg = _cfg(tmp_path)
    cfg["islands"] = {"per_rank": 4, "migrate_every": 0, "migrants": 1, "reset_every": 1, "migrant_dedup": True}
    fs = IslandFunSearch(cfg)
    fs.initialize()
    progs = [f"def priority_function(pod, node):\n    return {k} * node.cpu_milli_left + {k}\n" for k in range(4)]
    for i, s in enumerate(fs.islands):
        s.population = [(progs[i], 0.40 + 0.01 * i)]
        s.best_policy, s.best_score = progs[i], 0.40 + 0.01 * i
    weak = fs.reset_weak_islands()
    assert sorted(weak) == [0, 1]
    for i in weak:       # re-seeded with a surviving island's best
        assert fs.islands[i].best_policy in progs[2:] and len(fs.islands[i].population) == 1
    assert [s.best_policy for s in fs.islands[2:]] == progs[2:]
    # dedup: a near-copy of a better member is refused, a worse-than-worst one too
    s = fs.islands[3]
    s.population = [(progs[3], 0.5)] + [(f"def priority_function(pod, node):\n    return {j}\n", 0.3)
                                         for j in range(s.population_size - 1)]
    fs.apply_migrants(3, [(progs[3].replace("3 *", "3.0 *"), 0.45), ("def priority_function(pod, node):\n"
                                                                    "    return node.gpu_left\n", 0.1)])
    assert len(s.population) == s.population_size and max(sc for _, sc in s.population) == 0.5
    assert all(sc != 0.45 and sc != 0.1 for _, sc in s.population)
    fs.apply_migrants(3, [("def priority_function(pod, node):\n    return node.memory_mib_left // 7 - 1\n", 0.44)])
    assert 0.44 in [sc for _, sc in s.population]


def test_diverse_island_reset_keeps_lineages_apart(tmp_path):
    """islands.reset_diverse: a reset island restarts from the best surviving
    program that is not similar to any program another island leads with."""
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    cfg = _cfg(tmp_path)
    cfg["islands"] = {"per_rank": 4, "migrate_every": 0, "migrants": 1, "reset_every": 1, "reset_diverse": True}
    fs = IslandFunSearch(cfg)
    fs.initialize()
    lead = "def priority_function(pod, node):\n    return 3 * node.cpu_milli_left + 3\n"
    near = lead.replace("3 *", "4 *")                                   # similar to the lead
    other = "def priority_function(pod, node):\n    return node.memory_mib_left // 7 - pod.cpu_milli\n"
    weakp = [f"def priority_function(pod, node):\n    return {k}\n" for k in range(2)]
    for i, s in enumerate(fs.islands):
        s.population = [(weakp[i], 0.30)] if i < 2 else [(lead, 0.50), (near, 0.49), (other, 0.45)]
        s.best_policy, s.best_score = s.population[0]
    weak = fs.reset_weak_islands()
    assert sorted(weak) == [0, 1]
    # the lead (0.50) and its near copy (0.49) are taken by / similar to island 2-3's lead:
    # the first reset island gets `other`; nothing dissimilar is left for the second one,
    # which falls back to a survivor's best
    assert fs.islands[weak[0]].best_policy == other
    assert fs.islands[weak[1]].best_policy == lead


def test_mutator_library_terms_compile_for_the_device():
    """Every term and feature the offline mutator can insert passes the
    sandbox and compiles to device bytecode (a term that does not would only
    ever produce rejected children)."""
    from funsearch_kubernetes_simulator_amd.funsearch.llm import FEATURES, TERM_LIBRARY
    from funsearch_kubernetes_simulator_amd.policy.compiler import try_compile
    from funsearch_kubernetes_simulator_amd.policy.sandbox import SafeExecutor
    from funsearch_kubernetes_simulator_amd.policy.template import PolicyTemplate
    ex = SafeExecutor()
    bodies = ["score = 0.0\n" + t.format(c=1.5) for t in TERM_LIBRARY]
    bodies += [f"score = 0.0\nscore += 2.0 * ({f})" for f in FEATURES]
    for body in bodies:
        code = PolicyTemplate.fill_template("    " + body.replace("\n", "\n    "))
        assert ex.validate(code)
        prog, err = try_compile(code)
        assert prog is not None and prog.device_ok, (body, err)


def test_mutator_prunes_bloated_parents_by_lines():
    """Bloat control: a parent body past the cap loses random score-only
    top-level statements (their source lines, the rest verbatim) until it fits;
    the first statement, statements sharing a line and non-score statements
    stay."""
    import ast
    import random
    from funsearch_kubernetes_simulator_amd.funsearch.llm import MutationClient
    head = "x = node.cpu_milli_left / max(1, node.cpu_milli_total)\nscore = 0.0\n"
    terms = "".join(f"score += {i}.5 * x * (node.memory_mib_left / max(1, node.memory_mib_total))\n" for i in range(60))
    body = head + "a = 1; score += a\n" + terms + "if x > 0.5:\n    score -= 3.0\n"
    mc = MutationClient(0)
    out = mc._prune(body, random.Random(4), 1500)
    assert len(out) <= 1500 and len(out) < len(body)
    tree = ast.parse(out)
    assert out.split("\n")[0] == head.split("\n")[0]          # first statement kept verbatim
    assert "a = 1; score += a" in out                          # shared line kept
    kept = [ln for ln in out.split("\n") if ln.startswith("score += ")]
    assert all(ln in body.split("\n") for ln in kept)          # surviving lines verbatim
    assert isinstance(tree.body[0], ast.Assign)


def test_numeric_subexprs_match_naive_definition():
    """The one-pass candidate search equals the definition: numeric nodes not
    inside a comprehension iterable, an assignment target or a called name;
    `portable` ones read no parent-local name."""
    import ast
    from funsearch_kubernetes_simulator_amd.funsearch import llm
    from funsearch_kubernetes_simulator_amd.models.library import reference_policies, seed_policies

    def naive(tree, portable):
        skip = set()
        for n in ast.walk(tree):
            if isinstance(n, ast.comprehension):
                skip.update(id(x) for x in ast.walk(n.iter))
            elif isinstance(n, (ast.Assign, ast.AugAssign)):
                for t in (n.targets if isinstance(n, ast.Assign) else [n.target]):
                    skip.update(id(x) for x in ast.walk(t))
            elif isinstance(n, ast.Call):
                skip.update(id(x) for x in ast.walk(n.func))
        out = []
        for n in ast.walk(tree):
            if id(n) in skip:
                continue
            ok = (isinstance(n, (ast.BinOp, ast.UnaryOp))
                  or (isinstance(n, ast.Constant) and isinstance(n.value, (int, float)) and not isinstance(n.value, bool))
                  or (isinstance(n, ast.Attribute) and isinstance(n.value, ast.Name) and n.value.id in ("pod", "node")
                      and n.attr in llm._NUMERIC_FIELDS)
                  or (isinstance(n, ast.Call) and isinstance(n.func, ast.Name)
                      and n.func.id in ("abs", "min", "max", "sum")))
            if ok and (not portable or llm._free_names(n) <= llm._FREE_OK):
                out.append(id(n))
        return sorted(out)

    for code in list(reference_policies().values()) + list(seed_policies().values()):
        tree = ast.parse(code)
        for portable in (False, True):
            assert sorted(id(n) for n in llm._numeric_subexprs(tree, portable)) == naive(tree, portable)
