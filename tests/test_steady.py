"""Steady-state island mode (funsearch/steady.py) on the CPU: children from
producer processes, batches on evaluator slots, one-by-one merges, async
migration with a consistent distributed stop."""
import collections
import json
import os
import subprocess
import sys

import numpy as np

from funsearch_kubernetes_simulator_amd.models.library import reference_scores
from funsearch_kubernetes_simulator_amd.parallel import dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(tmp_path, gens=3, threshold=1.0, migrate_every=0, per_rank=2):
    return {"llm": {"backend": "mutation", "seed": 5}, "safe_execution": {"timeout_seconds": 3},
            "funsearch": {"population_size": 6, "generations": gens, "early_stop_threshold": threshold,
                          "elite_size": 3, "max_workers": 2, "policies_per_generation": 4},
            "islands": {"per_rank": per_rank, "migrate_every": migrate_every, "migrants": 1, "mode": "steady",
                        "steady": {"batch": 8, "producers": 2, "task_size": 2, "status_every_s": 0.5}},
            "device": {"kind": "cpu"}, "checkpoint": {"dir": str(tmp_path / "ck"), "every": 1},
            "log_path": str(tmp_path / "log.jsonl")}


def test_migrant_blob_round_trip_and_drops():
    from funsearch_kubernetes_simulator_amd.models.library import seed_policies
    from funsearch_kubernetes_simulator_amd.policy.template import PolicyTemplate
    body = "    return node.cpu_milli_left - pod.cpu_milli * 0.5"
    templ = PolicyTemplate.fill_template(body)
    b, is_templ = dist.program_body(templ)
    assert is_templ and b.strip() == body.strip() and PolicyTemplate.fill_template(b) == templ
    recs = [(0, templ, 0.5), (1, seed_policies()["best_fit"], 0.44)]
    out = dist.unpack_migrants(dist.pack_migrants(recs))
    assert out == recs
    # a blob too small for everything drops the lowest scores, and says so
    big = [(i, "def priority_function(pod, node):\n    return %d\n# %s" % (i, os.urandom(600).hex()), 1.0 - i * 0.01)
           for i in range(8)]
    logged = []
    blob = dist.pack_migrants(big, capacity=4096, log=logged.append)
    got = dist.unpack_migrants(blob)
    assert got == big[:len(got)] and 0 < len(got) < 8
    assert len(logged) == 8 - len(got) and all(r["kind"] == "migrant_dropped" for r in logged)
    assert blob.size == 4096 and int(np.frombuffer(blob[:8].tobytes(), np.int64)[0]) <= 4088


def test_steady_single_rank(tmp_path):
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    fs = IslandFunSearch(_cfg(tmp_path, migrate_every=2))
    code, score = fs.run(3)
    assert score >= reference_scores()["best_fit"] and "def priority_function" in code
    st = fs.steady.stats
    # every island produced its 3 generations x 4 children (bytecode rejects excluded)
    assert st.produced == 2 * 3 * 4 and st.evaluations == st.produced - st.rejected
    assert fs.generation == 3 and all(s.generation == 3 for s in fs.islands)
    assert all(len(s.population) <= 6 for s in fs.islands)
    recs = [json.loads(l) for l in open(tmp_path / "log.jsonl")]
    kinds = {r["kind"] for r in recs}
    assert {"steady_batch", "steady_final"} <= kinds
    fin = [r for r in recs if r["kind"] == "steady_final"][-1]
    for key in ("evals_per_s", "device_busy", "new_shape_fraction", "inflight", "migrations"):
        assert key in fin
    assert fin["evaluations"] == st.evaluations
    assert (tmp_path / "ck" / "islands_rank0.json").exists()


def test_steady_stager_depths(tmp_path):
    """Batches compiled ahead on the stager threads (``ahead`` 1 and 3, one or
    two ``stagers``, small batches so several are staged at once): every child
    is still evaluated exactly once and merged."""
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    for ahead, stagers in ((1, 1), (3, 1), (3, 2)):
        cfg = _cfg(tmp_path / f"a{ahead}s{stagers}", gens=2)
        cfg["islands"]["steady"].update(batch=3, ahead=ahead, stagers=stagers)
        fs = IslandFunSearch(cfg)
        fs.run(2)
        st = fs.steady.stats
        assert fs.steady.ahead == ahead and fs.steady.stagers == stagers
        assert st.produced == 2 * 2 * 4 and st.evaluations == st.produced - st.rejected
        assert st.batches >= st.evaluations // 3
        assert fs.generation == 2


def test_steady_early_stop_single_rank(tmp_path):
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    fs = IslandFunSearch(_cfg(tmp_path, gens=50, threshold=0.0))
    fs.run(50)
    assert fs.steady.stats.evaluations < 50 * 8


def _two_ranks(tmp_path, cfg, port_base):
    script = tmp_path / "w.py"
    script.write_text(
        "import json, os\n"
        "from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch\n"
        "if __name__ == '__main__':   # producers are spawned: they re-import this file\n"
        f"    fs = IslandFunSearch({str(tmp_path)!r} + '/cfg' + os.environ['RANK'] + '.json')\n"
        "    code, score = fs.run()\n"
        "    print(json.dumps({'rank': fs.ctx.rank, 'world': fs.ctx.world_size, 'score': score,\n"
        "                      'generation': fs.generation, 'migrations': fs.steady.stats.migrations,\n"
        "                      'evaluations': fs.steady.stats.evaluations, 'failures': len(fs.failures)}))\n")
    port = str(port_base + os.getpid() % 1000)
    procs = []
    for rank in (0, 1):
        env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="2", FKS_DIST_TIMEOUT_S="120", RANK=str(rank),
                   LOCAL_RANK=str(rank), WORLD_SIZE="2", LOCAL_WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, GLOO_SOCKET_IFNAME="lo")
        cfg_r = dict(cfg, log_path=str(tmp_path / f"log{rank}.jsonl"))
        (tmp_path / f"cfg{rank}.json").write_text(json.dumps(cfg_r))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=600)
        assert p.returncode == 0, e[-3000:]
        outs.append(json.loads([l for l in o.splitlines() if l.startswith("{")][-1]))
    return outs


def test_steady_two_gloo_ranks_migrate_without_lockstep(tmp_path):
    cfg = _cfg(tmp_path, gens=4, migrate_every=1, per_rank=1)
    outs = _two_ranks(tmp_path, cfg, 35000)
    assert [o["world"] for o in outs] == [2, 2] and not any(o["failures"] for o in outs)
    # both ranks posted the same gathers (one per generation) and agree on the global best
    assert outs[0]["migrations"] == outs[1]["migrations"] == 4
    assert outs[0]["score"] == outs[1]["score"] >= reference_scores()["best_fit"]


def test_steady_two_gloo_ranks_agree_on_stop(tmp_path):
    """Threshold reached at once: the ranks stop at the same migration (one
    gather carries the votes) and post the same number of gathers."""
    # (enough generations that the children cannot all be done before the
    # first asynchronous gather completes)
    cfg = _cfg(tmp_path, gens=2000, threshold=0.0, migrate_every=1, per_rank=1)
    outs = _two_ranks(tmp_path, cfg, 36000)
    assert outs[0]["migrations"] == outs[1]["migrations"] <= 4
    assert all(o["evaluations"] < 2000 * 4 for o in outs)


def test_host_fallback_sheds_object_engine_programs():
    """A program only CPython can score (an int64 overflow -> bigint in the
    replay) is shed, not replayed, when the caller turns the object engine
    off (steady `host_object: false`); with it on, CPython scores it."""
    from funsearch_kubernetes_simulator_amd.engine import Evaluator
    from funsearch_kubernetes_simulator_amd.policy.template import PolicyTemplate
    code = PolicyTemplate.fill_template(
        "    score = node.cpu_milli_left * node.memory_mib_left * node.cpu_milli_total * node.memory_mib_total\n"
        "    score = score * 1000000 / 10 ** 30")
    ev = Evaluator(device="cpu")
    prog = ev.compile_batch([code])
    shed = ev._evaluate_compiled([code], prog, native=False, host_only=True, object_ok=False)[0]
    assert shed.engine == "shed" and ev.stats["shed"] == 1
    full = ev._evaluate_compiled([code], prog, native=False, host_only=True, object_ok=True)[0]
    assert full.engine == "object" and full.exc == 0 and full.score > 0


def test_steady_constant_polish_batches(tmp_path):
    """Constant polish in steady mode: due island champions get a batch of
    literal variants (one shape), and a better setting re-enters the island as
    an ordinary child; children accounting is unaffected by the variants."""
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    cfg = _cfg(tmp_path, gens=4)
    cfg["polish"] = {"every": 1, "variants": 8, "repeat": True}
    fs = IslandFunSearch(cfg)
    fs.run(4)
    st = fs.steady.stats
    assert st.polish_batches > 0 and st.polish_evals == 8 * st.polish_batches
    assert st.evaluations == st.produced - st.rejected + st.polish_improved
    recs = [json.loads(l) for l in open(tmp_path / "log.jsonl")]
    pol = [r for r in recs if r["kind"] == "steady_polish"]
    # (records for the improving batches only)
    assert len(pol) == st.polish_improved and all(r["variants"] == 8 and r["improved"] for r in pol)
    fin = [r for r in recs if r["kind"] == "steady_final"][-1]
    assert fin["polish_batches"] == st.polish_batches


def test_steady_idle_slot_polish(tmp_path):
    """polish.idle: while the producers refill the child queue, a free slot
    runs a champion's constant polish instead of idling; children accounting
    (evals_per_s) stays children-only, all_evals_per_s adds the variants."""
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    cfg = _cfg(tmp_path, gens=6)
    cfg["polish"] = {"every": 1000, "variants": 8, "repeat": True, "idle": True}
    fs = IslandFunSearch(cfg)
    fs.run(6)
    st = fs.steady.stats
    assert st.polish_idle > 0 and st.polish_batches >= st.polish_idle
    assert st.polish_evals == 8 * st.polish_batches
    assert st.evaluations == st.produced - st.rejected + st.polish_improved
    fin = [json.loads(l) for l in open(tmp_path / "log.jsonl") if '"steady_final"' in l][-1]
    assert fin["polish_idle"] == st.polish_idle and fin["all_evals_per_s"] >= fin["evals_per_s"]


def test_steady_with_family_coupler(tmp_path):
    """`coupling.every` in steady mode: family-search rounds run on a worker
    thread and the evaluator's last slot (the program batches use the others);
    their champions enter the islands as exactly re-scored program text."""
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    cfg = _cfg(tmp_path, gens=4)
    cfg["coupling"] = {"every": 1, "generations": 1, "candidates": 64, "elite": 8,
                       "families": ["random_linear"], "seed": 1}
    fs = IslandFunSearch(cfg)
    code, score = fs.run(4)
    assert fs.coupler is not None and fs.coupler.rounds >= 1
    recs = [json.loads(l) for l in open(tmp_path / "log.jsonl")]
    coupled = [r for r in recs if r["kind"] == "coupling"]
    assert coupled and all(r["family"] == "random_linear" for r in coupled)
    final = [r for r in recs if r["kind"] == "steady_final"][-1]
    assert final["coupled"] == len(coupled) and final["coupler_evals"] >= 64
    # the exported program re-scores to the family score it was exported with
    best = max(coupled, key=lambda r: r["score"])
    assert best["score"] == best["family_score"]


def test_llm_fanout_overlaps_request_latency():
    """llm.concurrency: a producer task's requests wait concurrently (threads),
    so a task of 8 requests to a 0.4 s model takes ~0.4 s, not 3.2 s; the
    children are the scripted replies, validated and compiled as usual."""
    import time
    from funsearch_kubernetes_simulator_amd.funsearch import steady
    from funsearch_kubernetes_simulator_amd.funsearch.llm import LatencyClient, make_client, remote_like
    from funsearch_kubernetes_simulator_amd.models.library import seed_policies
    cfg = {"backend": "scripted", "responses": ["return node.cpu_milli_left - pod.cpu_milli * 0.5",
                                                "return -node.memory_mib_left"], "latency_s": [0.4, 0.4]}
    assert remote_like(cfg) and not remote_like({"backend": "mutation"})
    assert isinstance(make_client(cfg), LatencyClient)
    saved = dict(steady._W)
    try:
        steady._producer_init(cfg, 3, 0, fanout=8)
        elites = [(seed_policies()["first_fit"], 0.43), (seed_policies()["best_fit"], 0.45)]
        t0 = time.time()
        out, _, _, _ = steady._produce((1, elites, 8, [1.0, 3.0]))   # starts 8 requests, returns what is ready
        assert out == [] and time.time() - t0 < 0.3
        out2, _, _, _ = steady._produce((0, [], 0, None))             # flush: waits for the 8 in flight
        dt = time.time() - t0
        assert len(out2) == 8 and all(isl == 1 and prog is not None for isl, code, prog in out2)
        assert dt < 1.6, dt        # sequential: 8 x 0.4 s
        assert steady._W["gen"].llm_client.calls == 8
        # a task never leaves more than `fanout` requests in flight: the 9th..16th
        # wait for earlier ones and return their children
        steady._produce((1, elites, 8, None))
        out3, _, _, _ = steady._produce((1, elites, 8, None))
        assert len(out3) == 8 and len(steady._W["pending"]) == 8
        steady._produce((0, [], 0, None))
    finally:
        pool = steady._W.get("fanout")
        if pool is not None:
            pool.shutdown(wait=True)
        steady._W.clear()
        steady._W.update(saved)


def test_weighted_parent_sampling_prefers_cheap_parents():
    import random
    from funsearch_kubernetes_simulator_amd.funsearch.steady import _sample_parents
    rng = random.Random(3)
    elites = [("a", 1.0), ("b", 0.9), ("c", 0.8)]
    counts = {"a": 0, "b": 0, "c": 0}
    for _ in range(3000):
        ps = _sample_parents(rng, elites, [0.25, 0.25, 4.0])
        assert len(ps) == 2 and ps[0] != ps[1]
        for c, _ in ps:
            counts[c] += 1
    assert counts["c"] > 2900 and counts["a"] > 1000 and counts["b"] > 1000
    assert sorted(_sample_parents(rng, elites[:2], [1.0, 9.0])) == sorted(elites[:2])


def test_steady_with_llm_concurrency(tmp_path):
    """A steady run with a latency-modelled client and `llm.concurrency`:
    requests spread over producers x task_size threads (the steady_llm record)."""
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    cfg = _cfg(tmp_path, gens=2)
    cfg["llm"] = {"backend": "mutation", "seed": 5, "latency_s": [0.05, 0.15], "concurrency": 8}
    fs = IslandFunSearch(cfg)
    fs.run(2)
    recs = [json.loads(l) for l in open(tmp_path / "log.jsonl")]
    llm = [r for r in recs if r["kind"] == "steady_llm"]
    # 2 producers x 4 requests in flight each, topped up one at a time
    assert llm and llm[0]["concurrency"] == 8 and llm[0]["task_size"] == 1
    assert fs.steady.stats.produced == 2 * 2 * 4
    fin = [r for r in recs if r["kind"] == "steady_final"][-1]
    assert fin["children_per_s"] > 0


def test_deferred_merge_rechecks_members_added_since():
    """The program service's merges: the similarity scan runs on a worker
    thread against a snapshot; at completion the child is also scanned against
    members appended after the snapshot, and truncation is re-checked."""
    from funsearch_kubernetes_simulator_amd.funsearch.steady import SteadyStateSearch

    class Island:
        population_size, similarity_threshold, similarity_threads = 3, 0.85, 2
        best_score, best_policy = float("-inf"), None

        def __init__(self):
            self.population = []

        def _is_too_similar(self, code, score):
            raise AssertionError("deferred path must not scan synchronously")

    st = object.__new__(SteadyStateSearch)
    st._pending_merges, st._sim_pool, st._cost = collections.deque(), None, {}
    st.cost_bloat, st.service_cfg = 3.0, {}
    st.stats = type("S", (), {"cost_rejected": 0})()
    s = Island()
    a = "def f(pod, node):\n    return 1 + node.cpu_milli_left * 0.5\n"
    b = "def f(pod, node):\n    return 1 + node.cpu_milli_left * 0.6\n"          # similar to a
    c = "def g(pod, node):\n    x = [q for q in node.gpus]\n    return len(x) * 77 - pod.num_gpu\n"
    assert st._merge_one(s, a, 0.5, defer=True)        # empty population: appended at once
    assert not st._merge_one(s, c, 0.4, defer=True)    # scan against a deferred
    st._append(s, b, 0.45, 0.0, None)                   # a member added after c's snapshot
    assert not st._merge_one(s, b + "#", 0.44, defer=True)
    st._finish_merges(block=True)
    codes = [x for x, _ in s.population]
    assert a in codes and c in codes and b in codes and (b + "#") not in codes
    st._sim_pool.shutdown()


def test_device_cost_steers_selection_never_scores():
    """Per-program device cycles (service row column 13) decide only whether a
    non-best child is merged (bloat vs the island median and the run's anchor)
    and how parents are weighted: a merged child keeps its exact score, a new
    island best is merged whatever it costs, host-scored children (cost < 0)
    enter only as a new best."""
    from funsearch_kubernetes_simulator_amd.funsearch.steady import HOST_COST, SteadyStateSearch

    class Island:
        population_size, similarity_threshold, similarity_threads = 8, 0.85, 1
        best_score, best_policy = 0.6, None

        def __init__(self):
            self.population = []

        def _is_too_similar(self, code, score):
            return False

    st = object.__new__(SteadyStateSearch)
    st._pending_merges, st._sim_pool, st._cost = collections.deque(), None, {}
    st.cost_bloat, st.service_cfg = 3.0, {}
    st.cost_anchor, st.cost_anchor_cap = 100.0, 3.0
    st.stats = type("S", (), {"cost_rejected": 0})()
    s = Island()
    progs = [f"def f(pod, node):\n    return {k} + node.cpu_milli_left\n" for k in range(8)]
    for k in range(3):
        assert st._merge_one(s, progs[k], 0.5 + 0.01 * k, cost=100.0, island=0)
    assert not st._merge_one(s, progs[3], 0.55, cost=1000.0, island=0)     # 10x the median, not a best
    assert not st._merge_one(s, progs[4], 0.55, cost=HOST_COST, island=0)  # host-scored, not a best
    assert st._merge_one(s, progs[5], 0.7, cost=1e6, island=0)             # new best: merged regardless
    assert st._merge_one(s, progs[6], 0.55, cost=250.0, island=0)          # within 3x median and anchor
    assert st.stats.cost_rejected == 2
    assert dict(s.population) == {progs[0]: 0.5, progs[1]: 0.51, progs[2]: 0.52, progs[5]: 0.7, progs[6]: 0.55}
