"""Trace ingestion quirks, synthetic generator, and multi-process (gloo) collectives."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.core import TraceParser, synthetic_workload
from funsearch_kubernetes_simulator_amd.core.arrays import Workload, dense_rank

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parser_defaults_and_files():
    p = TraceParser()
    cluster, pods = p.parse_workload()
    assert len(cluster.nodes_dict) == 16 and len(pods) == 8152
    assert cluster.num_gpus == 64
    assert "openb_pod_list_default.csv" in p.get_available_pod_files()
    assert p.get_available_node_files() == ["openb_node_list_all_node.csv", "openb_node_list_gpu_node.csv"]
    assert pods[1].duration_time == 12902960 - 427061


def test_multigpu_traces_raise_like_reference():
    with pytest.raises(KeyError):
        TraceParser().parse_pods("openb_pod_list_multigpu20.csv")


def test_all_node_csv_has_cpu_only_nodes():
    nodes = TraceParser().parse_nodes("openb_node_list_all_node.csv")
    assert len(nodes) == 1523
    assert sum(1 for n in nodes.values() if not n.gpus) == 310


def test_k8s_yaml_matches_csv():
    p = TraceParser()
    y = p.parse_node_yaml()
    c = p.parse_cluster("openb_node_list_gpu_node.csv")
    assert len(y) == len(c) == 1213
    for nid, n in list(c.nodes_dict.items())[:50]:
        m = y.nodes_dict[nid]
        assert (m.cpu_milli_total, m.memory_mib_total, m.gpu_left, len(m.gpus)) == \
               (n.cpu_milli_total, n.memory_mib_total, n.gpu_left, len(n.gpus))


def test_dense_rank_ties():
    assert list(dense_rank(["b", "a", "b", "c"])) == [1, 0, 1, 2]


def test_synthetic_workload_shape():
    w = synthetic_workload(n_nodes=64, n_pods=4000, seed=1)
    assert w.cluster.n_nodes == 64 and w.pods.n_pods == 4000
    assert np.all(np.diff(w.pods.pod_ctime) >= 0)
    c, p = w.to_objects()
    w2 = Workload.from_objects(c, p)
    assert w2.fingerprint() == w.fingerprint()


def _run_torchrun(script: str, nproc: int = 2, timeout: int = 600):
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(29000 + os.getpid() % 1000), script]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)


def test_gloo_collectives_and_migration(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(
        "import json, numpy as np\n"
        "from funsearch_kubernetes_simulator_amd.parallel import dist\n"
        "from funsearch_kubernetes_simulator_amd.funsearch.param_islands import make_islands, migrate\n"
        "ctx = dist.init_distributed(use_gpu=False)\n"
        "x = np.full((2, 3), ctx.rank, dtype=np.float64)\n"
        "g = dist.all_gather_array(x)\n"
        "assert g.shape == (2, 2, 3) and g[1].max() == 1\n"
        "pg = dist.all_gather_array_async(x + 5)\n"
        "assert np.array_equal(pg.wait(), g + 5)\n"
        "assert dist.all_reduce_max(ctx.rank * 10.0) == 10.0\n"
        "isl = make_islands(2, 'random_linear', 4, 3, seed=ctx.rank)\n"
        "for i in isl:\n"
        "    w = i.propose(); i.update(w, np.arange(len(w)) + 100.0 * ctx.rank)\n"
        "migrate(isl, 2, dist.all_gather_array)\n"
        "rec = dist.pack_programs(['abc' * ctx.rank, 'x'], [1.0, 2.0])\n"
        "allr = dist.all_gather_array(rec)\n"
        "progs = dist.unpack_programs(allr)\n"
        "assert ('x', 2.0) in progs\n"
        "if ctx.rank == 0: print(json.dumps({'ok': True, 'best_island0': float(isl[0].elite_scores.max())}))\n"
        "dist.shutdown()\n")
    r = _run_torchrun(str(script))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    # island 0 of rank 0 received rank 1's migrants (scores >= 100)
    assert out["ok"] and out["best_island0"] >= 100


def test_host_group_collectives_two_ranks(tmp_path):
    """The gloo group opened beside the default one (RCCL on a GPU node; a
    second gloo group here, FKS_HOST_GROUP=force): with use_host_collectives
    every host-array collective goes through it and returns what the default
    group returns."""
    script = tmp_path / "h.py"
    script.write_text(
        "import json, os, numpy as np\n"
        "os.environ['FKS_HOST_GROUP'] = 'force'\n"
        "from funsearch_kubernetes_simulator_amd.parallel import dist\n"
        "ctx = dist.init_distributed(use_gpu=False)\n"
        "x = np.full((2, 3), ctx.rank, dtype=np.float64)\n"
        "ref = dist.all_gather_array(x)\n"
        "assert dist.use_host_collectives(True)\n"
        "assert dist._host_group()[0] is not None\n"
        "g = dist.all_gather_array(x)\n"
        "assert np.array_equal(g, ref)\n"
        "assert np.array_equal(dist.all_gather_array_async(x + 1).wait(), ref + 1)\n"
        "assert dist.all_reduce_max(ctx.rank * 10.0) == 10.0 and dist.all_reduce_sum(1.0) == 2.0\n"
        "assert dist.all_gather_bytes(b'r%d' % ctx.rank) == [b'r0', b'r1']\n"
        "dist.barrier()\n"
        "assert not dist.use_host_collectives(False)\n"
        "if ctx.rank == 0: print(json.dumps({'ok': True}))\n"
        "dist.shutdown()\n")
    r = _run_torchrun(str(script))
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])["ok"]


def test_global_best_carries_long_program_across_ranks(tmp_path):
    """The cross-rank champion travels whatever its length: rank 1 holds a
    >8 KB best program, both ranks return it (no fixed-width record)."""
    _rank_loss_config(tmp_path)
    script = tmp_path / "w.py"
    script.write_text(
        "import json\n"
        "from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch\n"
        "from funsearch_kubernetes_simulator_amd.parallel import dist\n"
        f"fs = IslandFunSearch({str(tmp_path / 'cfg.json')!r})\n"
        "s = fs.islands[0]\n"
        "if fs.ctx.rank == 1:\n"
        "    s.best_policy = 'def priority_function(pod, node):\\n' + '    x = 1\\n' * 1200 + '    return 7\\n'\n"
        "    s.best_score = 0.9\n"
        "else:\n"
        "    s.best_policy, s.best_score = 'def priority_function(pod, node):\\n    return 1\\n', 0.5\n"
        "code, score = fs.global_best()\n"
        "try:\n"
        "    dist.pack_programs([code], [score])\n"
        "    raised = False\n"
        "except dist.RecordTooLong:\n"
        "    raised = True\n"
        "print(json.dumps({'rank': fs.ctx.rank, 'len': len(code), 'score': score, 'raised': raised,\n"
        "                  'same': code == s.best_policy}))\n"
        "dist.shutdown()\n")
    r = _run_torchrun(str(script))
    assert r.returncode == 0, r.stderr[-2000:]
    import re
    outs = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", r.stdout)]
    assert sorted(o["rank"] for o in outs) == [0, 1]
    for o in outs:
        assert o["len"] > 8192 and o["score"] == 0.9 and o["raised"]
        assert o["same"] == (o["rank"] == 1)


def test_no_migration_ranks_agree_on_stop(tmp_path):
    """migrate_every = 0 with two ranks: a stop-only channel makes both ranks
    stop at the same generation (threshold 0 is reached at once), so neither
    waits in the champion gather for a peer that runs on."""
    cfg = {"llm": {"backend": "mutation", "seed": 3}, "safe_execution": {"timeout_seconds": 3},
           "funsearch": {"population_size": 6, "generations": 6, "early_stop_threshold": 0.0, "elite_size": 3,
                         "max_workers": 2, "policies_per_generation": 2},
           "islands": {"per_rank": 2, "migrate_every": 0, "migrants": 1},
           "device": {"kind": "cpu"}}
    outs = []
    for mode in ("sync", "pipeline"):
        c = json.loads(json.dumps(cfg))
        c["islands"]["pipeline"] = mode == "pipeline"
        (tmp_path / f"{mode}.json").write_text(json.dumps(c))
    script = tmp_path / "w.py"
    script.write_text(
        "import json, sys\n"
        "from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch\n"
        "from funsearch_kubernetes_simulator_amd.parallel import dist\n"
        "res = {}\n"
        "for mode in ('sync', 'pipeline'):\n"
        f"    fs = IslandFunSearch({str(tmp_path)!r} + '/' + mode + '.json')\n"
        "    code, score = fs.run()\n"
        "    res[mode] = [fs.generation, [s.generation for s in fs.islands], score]\n"
        f"open({str(tmp_path)!r} + '/out%d.json' % fs.ctx.rank, 'w').write(json.dumps({{'rank': fs.ctx.rank, 'res': res}}))\n"
        "dist.shutdown()\n")
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1", FKS_DIST_TIMEOUT_S="120")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(35000 + os.getpid() % 1000), str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    # (each rank writes its own file: the ranks' stdout lines can interleave)
    outs = [json.loads((tmp_path / f"out{k}.json").read_text()) for k in range(2)]
    a, b = outs
    assert a["res"]["sync"][0] == b["res"]["sync"][0] == 1          # lock-step: stop agreed in generation 1
    assert a["res"]["sync"][2] == b["res"]["sync"][2]                 # same champion score on both ranks
    # pipelined: both ranks stop well before the configured 6 generations, each within the
    # channel's documented delay (lookahead * every generations after the first vote)
    for o in (a, b):
        assert o["res"]["pipeline"][0] <= 4, outs
    assert a["res"]["pipeline"][2] == b["res"]["pipeline"][2]


def test_inject_one_per_island_equals_ring_inject():
    """bench.py's asynchronous migration injects island by island (inject_one);
    applied to every island it is the ring migration of inject()."""
    import numpy as np
    from funsearch_kubernetes_simulator_amd.funsearch.param_islands import (
        inject, inject_one, make_islands, migration_records)

    def fresh():
        isl = make_islands(3, "random_linear", 8, 4, seed=5)
        for k, i in enumerate(isl):
            w = i.propose()
            i.update(w, np.arange(len(w)) + 100.0 * k)
        return isl
    a, b = fresh(), fresh()
    glob = np.stack([migration_records(a, 2), migration_records(a, 2) + 0.5])   # two ranks
    inject(a, glob, rank=1)
    for li in range(len(b)):
        inject_one(b, li, glob, rank=1)
    for x, y in zip(a, b):
        assert np.array_equal(x.elite_scores, y.elite_scores)
        assert np.array_equal(x.elites, y.elites)


def test_bench_two_ranks_cpu():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(30000 + os.getpid() % 1000),
                        os.path.join(REPO, "bench.py"), "--gpus", "2", "--device", "cpu", "--steps", "2",
                        "--warmup", "1", "--islands", "1", "--candidates", "4", "--migrate-every", "1"],
                       env=dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1"), capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["scaling"] == "weak"
    assert line["config"]["global_batch"] == 8


def test_native_csv_loader_matches_python_parser():
    """C++ trace loader (csrc/cpu/trace_io.hpp) == the object-graph parser, field by field."""
    p = TraceParser()
    for nf in ("gpu_models_filtered.csv", "openb_node_list_all_node.csv"):
        for pf in ("openb_pod_list_default.csv", "openb_pod_list_gpuspec33.csv", "openb_pod_list_cpu050.csv"):
            a = p.load_workload(nf, pf, native=False)
            b = p.load_workload(nf, pf, native=True)
            assert a.cluster.node_ids == b.cluster.node_ids and a.pods.pod_ids == b.pods.pod_ids
            assert a.pods.gpu_spec == b.pods.gpu_spec
            for name in ("node_cpu_total", "node_cpu_left", "node_mem_total", "node_mem_left", "node_gpu_left",
                         "node_ngpus", "gpu_start", "gpu_milli_total", "gpu_milli_left", "gpu_mem_total",
                         "gpu_mem_left"):
                assert np.array_equal(getattr(a.cluster, name), getattr(b.cluster, name)), name
            for name in ("pod_cpu", "pod_mem", "pod_ngpu", "pod_gmilli", "pod_ctime", "pod_dur", "pod_rank"):
                assert np.array_equal(getattr(a.pods, name), getattr(b.pods, name)), name
    with pytest.raises(KeyError):
        p.load_workload("gpu_models_filtered.csv", "openb_pod_list_multigpu20.csv", native=True)


def _rank_loss_config(tmp_path):
    ck = tmp_path / "ck"
    cfg = {"llm": {"backend": "mutation", "seed": 3}, "safe_execution": {"timeout_seconds": 3},
           "funsearch": {"population_size": 6, "generations": 4, "early_stop_threshold": 1.0, "elite_size": 3,
                         "max_workers": 2, "policies_per_generation": 2},
           "islands": {"per_rank": 1, "migrate_every": 1, "migrants": 1},
           "device": {"kind": "cpu"}, "checkpoint": {"dir": str(ck), "every": 1}}
    (tmp_path / "cfg.json").write_text(json.dumps(cfg))
    return ck


def test_island_search_survives_rank_crash(tmp_path):
    """Rank 1 is SIGKILLed mid-run (gloo, 2 ranks started directly with the
    env:// rendezvous -- no torchrun agent, which would tear the whole group
    down on a crash): rank 0's next collective fails, it logs a rank_failure
    record, checkpoints and finishes alone; a later --resume on one process
    picks the run up from rank 0's file."""
    ck = _rank_loss_config(tmp_path)
    script = tmp_path / "w.py"
    script.write_text(
        "import json, os, signal, sys\n"
        "from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch\n"
        f"fs = IslandFunSearch({str(tmp_path / 'cfg.json')!r})\n"
        "fs.initialize()\n"
        "for g in range(4):\n"
        "    if fs.ctx.rank == 1 and g == 2:\n"
        "        sys.stdout.flush(); os.kill(os.getpid(), signal.SIGKILL)   # a real crash\n"
        "    fs.evolve()\n"
        "code, score = fs.global_best()\n"
        "print(json.dumps({'gen': fs.generation, 'world': fs.ctx.world_size, 'score': score,\n"
        "                  'failures': [f['collective'] for f in fs.failures]}))\n")
    port = str(31000 + os.getpid() % 1000)
    procs = []
    for rank in (0, 1):
        env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1", FKS_DIST_TIMEOUT_S="60", RANK=str(rank),
                   LOCAL_RANK=str(rank), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    out0, err0 = procs[0].communicate(timeout=600)
    procs[1].communicate(timeout=60)
    assert procs[1].returncode == -9                       # killed by the signal, not a clean exit
    assert procs[0].returncode == 0, err0[-3000:]
    out = json.loads([l for l in out0.splitlines() if l.startswith("{")][-1])
    assert out["gen"] == 4 and out["world"] == 1 and len(out["failures"]) == 1
    assert out["score"] > 0.44
    st = json.loads((ck / "islands_rank0.json").read_text())
    assert st["generation"] == 4 and st["world_size"] == 1
    from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch
    fs = IslandFunSearch(str(tmp_path / "cfg.json"))
    assert fs.load_elastic(str(ck)) and fs.generation == 4


def test_torchrun_restart_resumes_after_rank_crash(tmp_path):
    """Under torchrun a crashing rank (non-zero exit) makes the agent stop the
    whole group, so in-process survival cannot happen there; the reachable
    recovery is ``--max-restarts`` + elastic resume: the restarted group
    reloads the per-rank checkpoints and finishes the run."""
    ck = _rank_loss_config(tmp_path)
    script = tmp_path / "w.py"
    script.write_text(
        "import json, os, sys\n"
        "from funsearch_kubernetes_simulator_amd.funsearch.islands import IslandFunSearch\n"
        f"fs = IslandFunSearch({str(tmp_path / 'cfg.json')!r})\n"
        f"if not fs.load_elastic({str(ck)!r}):\n"
        "    fs.initialize()\n"
        "first = os.environ.get('TORCHELASTIC_RESTART_COUNT', '0') == '0'\n"
        "while fs.generation < 4:\n"
        "    if first and fs.ctx.rank == 1 and fs.generation == 2:\n"
        "        sys.stdout.flush(); os._exit(3)   # crash on the first attempt only\n"
        "    fs.evolve()\n"
        "code, score = fs.global_best()\n"
        "print(json.dumps({'gen': fs.generation, 'world': fs.ctx.world_size, 'score': score,\n"
        "                  'restart': os.environ.get('TORCHELASTIC_RESTART_COUNT')}))\n")
    env = dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1", FKS_DIST_TIMEOUT_S="60", GLOO_SOCKET_IFNAME="lo")
    # dynamic (c10d) rendezvous; the agent's store outlives a round, so dist.init_distributed keys
    # every round's group formation by TORCHELASTIC_RESTART_COUNT (a restarted group once read the
    # killed round's peer addresses: "connectFullMesh ... Connection refused").  One restart is enough.
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--max-restarts=1",
           "--rdzv-backend=c10d", "--local-addr=127.0.0.1", f"--rdzv-endpoint=127.0.0.1:{33000 + os.getpid() % 1000}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    import re
    outs = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", r.stdout)]   # the two ranks' lines may interleave
    assert outs and all(o["gen"] == 4 and o["world"] == 2 and o["restart"] == "1" for o in outs)
    assert max(o["score"] for o in outs) > 0.44


def test_scaling_harness_cpu():
    """bench.scaling drives bench.py at 1 and 2 ranks (gloo) and reports the
    weak-scaling efficiency relative to N=1."""
    from funsearch_kubernetes_simulator_amd.bench import scaling
    rows = scaling.summarize({1: {"value": 10.0, "ms_per_step": 5.0}, 2: {"value": 18.0, "ms_per_step": 5.5},
                              4: None})
    assert rows[1]["efficiency"] == 0.9 and rows[2]["value"] is None
    r = subprocess.run([sys.executable, "-m", "funsearch_kubernetes_simulator_amd.bench.scaling", "--gpus", "1,2",
                        "--port", str(32000 + os.getpid() % 1000), "--", "--device", "cpu", "--steps", "1",
                        "--warmup", "1", "--islands", "1", "--candidates", "4"],
                       env=dict(os.environ, PYTHONPATH=REPO, OMP_NUM_THREADS="1"), capture_output=True, text=True,
                       timeout=900, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    summary = json.loads(r.stdout.strip().splitlines()[-1])["scaling"]
    assert [s["n_gpus"] for s in summary] == [1, 2]
    assert all(s["value"] > 0 for s in summary) and summary[0]["efficiency"] == 1.0


def test_config4_launcher_two_gloo_ranks(tmp_path):
    """tools/run_config4.sh (BASELINE config 4: one island per rank, RCCL elite
    migration, torchrun --max-restarts + --resume) rehearsed with 2 gloo ranks."""
    # (the CPU rehearsal config: config 4's structure -- steady loop, polish,
    # family coupler -- with per-generation work a CPU evaluator finishes)
    env = dict(os.environ, NPROC="2", GENS="2", RUN_DIR=str(tmp_path / "c4"), FKS_DIST_BACKEND="gloo",
               PORT=str(34000 + os.getpid() % 1000), OMP_NUM_THREADS="1", GLOO_SOCKET_IFNAME="lo",
               CONFIG="configs/config4_rehearsal.json", DEVICE_ARGS="--device cpu")
    r = subprocess.run(["bash", os.path.join(REPO, "tools", "run_config4.sh")], env=env, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["ranks"] == 2 and out["islands_per_rank"] == 1 and out["generations"] == 2
    assert (tmp_path / "c4" / "metrics.rank1.jsonl").exists()


def test_device_workload_requires_one_gpu_model_per_node(default_workload):
    """The kernels keep one GPU-milli total per node (NodeRegs::gmt1): a node
    whose GPUs differ is rejected up front (UnsupportedWorkload -> CPU
    engines), never replayed with a wrong total."""
    import copy
    from funsearch_kubernetes_simulator_amd.ops.hip_engine import UnsupportedWorkload, prepare_device_workload
    prepare_device_workload(default_workload)            # OpenB: one model per node
    w = copy.deepcopy(default_workload)
    a, b = int(w.cluster.gpu_start[0]), int(w.cluster.gpu_start[1])
    assert b - a >= 2
    w.cluster.gpu_milli_total[a + 1] = 500
    with pytest.raises(UnsupportedWorkload, match="milli totals"):
        prepare_device_workload(w)


def test_one_rank_group_collectives_equal_local(tmp_path):
    """FKS_DIST_GROUP=1 creates a one-rank process group (gloo here, RCCL on the
    GPU box: tests/test_gpu_rccl.py); the collective helpers then go through it
    and return what the local path returns."""
    import subprocess
    import sys
    script = tmp_path / "one.py"
    script.write_text(
        "import json, numpy as np\n"
        "from funsearch_kubernetes_simulator_amd.parallel import dist\n"
        "ctx = dist.init_distributed(backend='gloo', use_gpu=False, force_group=True)\n"
        "x = np.arange(12.0).reshape(3, 4)\n"
        "h = dist.all_gather_array_async(x)\n"
        "g = h.wait()\n"
        "out = {'group': ctx.group, 'distributed': ctx.distributed, 'backend': ctx.backend,\n"
        "       'gather': bool(np.array_equal(g, x[None])), 'bytes': dist.all_gather_bytes(b'abc') == [b'abc'],\n"
        "       'max': dist.all_reduce_max(2.5), 'sum': dist.all_reduce_sum(1.5)}\n"
        "dist.barrier()\n"
        "dist.shutdown()\n"
        "print(json.dumps(out))\n")
    env = dict(os.environ, PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
               WORLD_SIZE="1", RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29400 + os.getpid() % 300),
               GLOO_SOCKET_IFNAME="lo")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out == {"group": True, "distributed": False, "backend": "gloo", "gather": True, "bytes": True,
                   "max": 2.5, "sum": 1.5}
