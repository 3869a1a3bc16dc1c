"""Program-path throughput: FunSearch candidate *programs* (not parametric
family members) evaluated exactly, as the evolution loop produces them.

`mutation_children` draws offline-mutation children (funsearch/llm.py
`MutationClient`, the LLM stand-in of the config-3 runs) of the reference and
seed programs; `measure_native` times them through the MI355X native backend
(JIT compile + k_replay_native) -- the number to compare with the reference's
program evals/s (15.84), next to the parametric headline."""

from __future__ import annotations

import random
import time
from typing import List

from ..funsearch.llm import MutationClient
from ..models.library import reference_policies, seed_policies
from ..policy.compiler import CompiledPolicy, CompileError, compile_policy
from ..policy.template import PolicyTemplate


def mutation_children(n: int, seed: int = 0, device_only: bool = True) -> List[CompiledPolicy]:
    client = MutationClient(seed)
    parents = list(reference_policies().values()) + list(seed_policies().values())
    out: List[CompiledPolicy] = []
    seen = set()
    rng = random.Random(seed)
    tries = 0
    while len(out) < n and tries < 50 * n:
        tries += 1
        pa = rng.sample(parents, 2)
        prompt = PolicyTemplate.create_prompt_for_llm([(pa[0], 0.45), (pa[1], 0.44)], "feedback")
        resp = client.chat.completions.create(model="m", messages=[{"role": "user", "content": prompt}])
        code = PolicyTemplate.fill_template(resp.choices[0].message.content)
        if code in seen:
            continue
        try:
            p = compile_policy(code)
        except CompileError:
            continue
        if device_only and not p.device_ok:
            continue
        seen.add(code)
        out.append(p)
        if rng.random() < 0.3:
            parents.append(code)
    return out


def measure_native(dev, progs: List[CompiledPolicy]) -> dict:
    """Evaluate `progs` natively twice: the first pass pays the JIT for every
    new shape, the second finds them all cached (pure device time)."""
    t0 = time.perf_counter()
    batch = dev.submit_native(0, progs)
    t1 = time.perf_counter()
    tab = dev.wait(0)
    t2 = time.perf_counter()
    dev.submit_native(0, progs)
    tab2 = dev.wait(0)
    t3 = time.perf_counter()
    n = len(progs)
    info = dev.info()
    kernel = ({0: "k_replay_native_duo (two waves per program)"}.get(info.get("native_rows_last"),
              f"k_replay_rows_native ({info.get('native_rows_last')} per wave)")
              if info.get("native_waves_last") else "k_replay_native")
    return {"programs": n, "kernel": kernel, "native": int(batch.ok.sum()), "new_shapes": int(batch.compiled),
            "jit_s": round(t1 - t0, 3), "device_s": round(t2 - t1, 3),
            "evals_per_s_incl_jit": round(n / (t2 - t0), 1), "evals_per_s_cached": round(n / (t3 - t2), 1),
            "events": int(tab[:, 8].sum()), "repeat_identical": bool((tab == tab2).all())}


def novel_children(n: int, seed: int = 0, exclude=()) -> List[CompiledPolicy]:
    """`n` mutation children with pairwise-distinct shapes (`shape_key`),
    none in `exclude` (e.g. the shapes a compiler already holds): every one is
    a JIT compile, as with a real LLM, which almost never repeats a program's
    structure."""
    from ..policy.native_codegen import shape_key
    out, keys = [], set(exclude)
    s = seed
    while len(out) < n:
        for p in mutation_children(2 * (n - len(out)) + 8, seed=s):
            k = shape_key(p)
            if k not in keys:
                keys.add(k)
                out.append(p)
                if len(out) == n:
                    break
        s += 7919
    return out


def measure_novel(dev, workload, n: int = 256, compile_batches: int = 4, seed: int = 0,
                  cpu_threads: int = 0) -> dict:
    """Novel-program throughput: `n` programs, every one a new shape, JIT
    included, against the CPU VM on the same batch (bit-identical rows asserted
    over programs neither engine defers).  Also the compile time of
    `compile_batches` batches of 64 fresh shapes (median logged)."""
    import numpy as np
    from ..engine import COLS
    from ..ops import cpu_engine as ce
    progs = novel_children(n + 64 * compile_batches, seed, exclude=set(dev.native_compiler._shapes))
    main, extra = progs[:n], progs[n:]
    t64 = []
    for i in range(compile_batches):
        b = dev.submit_native(0, extra[64 * i:64 * (i + 1)])
        dev.wait(0)
        t64.append(b.compile_s)
    t0 = time.perf_counter()
    batch = dev.submit_native(0, main)
    t1 = time.perf_counter()
    tab = dev.wait(0)
    t2 = time.perf_counter()
    threads = cpu_threads or ce.default_threads()
    c0 = time.perf_counter()
    vm = ce.simulate_program_batch(workload, main, threads=threads)
    c1 = time.perf_counter()
    skip = (100, 101)
    exc, vexc = tab[:, COLS["exc"]].astype(int), vm[:, COLS["exc"]].astype(int)
    cmp = ~np.isin(exc, skip) & ~np.isin(vexc, skip)
    if not dev.options.get("trace_hash", True):
        # the device skipped the per-event trace hash (bench.py turns it off): compare the rest
        tab, vm = tab[:, :COLS["trace_hash_hi"]], vm[:, :COLS["trace_hash_hi"]]
    dev_rate, vm_rate = n / (t2 - t0), n / (c1 - c0)
    st = dev.native_compiler.stats
    return {"programs": n, "new_shapes": int(batch.compiled), "native": int(batch.ok.sum()),
            "jit_tier": getattr(dev.native_compiler, "tier", "?"),
            "jit_s": round(t1 - t0, 4), "device_s": round(t2 - t1, 4),
            "evals_per_s_incl_jit": round(dev_rate, 1),
            "cpu_vm_evals_per_s": round(vm_rate, 1), "cpu_vm_threads": threads,
            "vs_cpu_vm": round(dev_rate / vm_rate, 2),
            "compile_s_per_64_batch": [round(x, 4) for x in t64],
            "compile_s_per_64_median": round(float(np.median(t64)), 4) if t64 else None,
            "baseline_shapes": int(st.get("baseline_shapes", 0)), "llvm_shapes": int(st.get("llvm_shapes", 0)),
            "compared": int(cmp.sum()), "bit_identical": bool((tab[cmp] == vm[cmp]).all())}


def _novel_worker(args):
    n, seed = args
    return novel_children(n, seed)


def novel_children_parallel(n: int, seed: int = 0, workers: int = 8, exclude=()) -> List[CompiledPolicy]:
    """`novel_children` generated in `workers` spawned processes (the offline
    mutator + bytecode compiler run ~9 ms a program on one core); shapes are
    deduplicated across workers, and the shortfall is made up serially."""
    import concurrent.futures
    import multiprocessing
    from ..policy.native_codegen import shape_key
    workers = max(1, min(workers, n // 64 or 1))
    per = -(-n // workers) + 16
    keys, out = set(exclude), []
    if workers > 1:
        with concurrent.futures.ProcessPoolExecutor(workers, mp_context=multiprocessing.get_context("spawn")) as ex:
            parts = list(ex.map(_novel_worker, [(per, seed + 104729 * (w + 1)) for w in range(workers)]))
    else:
        parts = [novel_children(per, seed)]
    for part in parts:
        for p in part:
            k = shape_key(p)
            if k not in keys and len(out) < n:
                keys.add(k)
                out.append(p)
    if len(out) < n:
        out += novel_children(n - len(out), seed + 7, exclude=keys)
    return out


def measure_novel_large(dev, workload, n: int = 2048, seed: int = 0, compare: int = 128, cpu_threads: int = 0,
                        workers: int = 8) -> dict:
    """LLM-scale batch of `n` programs, every one a new shape, JIT included:
    split over the device's slots, each chunk compiled (C++ generator, host
    threads), loaded and launched while the previous chunks replay, with the
    two-wave kernel's heap top sized for all `n` in flight.  The first
    `compare` programs are checked against the CPU VM, row for row."""
    import numpy as np
    from ..engine import COLS
    from ..ops import cpu_engine as ce
    progs = novel_children_parallel(n, seed, workers, exclude=set(dev.native_compiler._shapes))
    slots = max(1, dev.n_slots)
    size = -(-n // slots)
    chunks = [progs[i:i + size] for i in range(0, n, size)]
    dev.set_options(native_inflight=n)
    try:
        t0 = time.perf_counter()
        batches = [dev.submit_native(s, c) for s, c in enumerate(chunks)]
        t_sub = time.perf_counter()
        tabs = [dev.wait(s) for s in range(len(chunks))]
        t1 = time.perf_counter()
        info = dev.info()
        # the same programs again: every shape cached (device time only)
        for s, c in enumerate(chunks):
            dev.submit_native(s, c)
        tabs2 = [dev.wait(s) for s in range(len(chunks))]
        t2 = time.perf_counter()
    finally:
        dev.set_options(native_inflight=0)
    tab, tab2 = np.concatenate(tabs), np.concatenate(tabs2)
    threads = cpu_threads or ce.default_threads()
    sub = progs[:compare]
    vm = ce.simulate_program_batch(workload, sub, threads=threads)
    a, b = tab[:compare], vm
    skip = (100, 101, 102, 103)
    cmp = ~np.isin(a[:, COLS["exc"]].astype(int), skip) & ~np.isin(b[:, COLS["exc"]].astype(int), skip)
    if not dev.options.get("trace_hash", True):
        a, b = a[:, :COLS["trace_hash_hi"]], b[:, :COLS["trace_hash_hi"]]
    return {"programs": n, "chunks": len(chunks), "new_shapes": int(sum(x.compiled for x in batches)),
            "native": int(sum(x.ok.sum() for x in batches)),
            "jit_s": round(sum(x.compile_s for x in batches), 4), "load_s": round(sum(x.load_s for x in batches), 4),
            "submit_s": round(t_sub - t0, 4), "wall_s": round(t1 - t0, 4),
            "evals_per_s_incl_jit": round(n / (t1 - t0), 1), "evals_per_s_cached": round(n / (t2 - t1), 1),
            "duo_heap_top": info.get("native_duo_top_last"), "duo_programs_per_cu": info.get("native_duo_per_cu_last"),
            "resident_capacity": int(info.get("native_duo_per_cu_last", 0)) * int(info.get("num_cus", 0)),
            "repeat_identical": bool((tab == tab2).all()),
            "compared": int(cmp.sum()), "bit_identical": bool((a[cmp] == b[cmp]).all())}


# ---------------------------------------------------------------------------- evolved programs
#: 2,048 offline-mutation children of the best programs of an evolved steady-state
#: population (data/populations/config3_steady_r4f_islands.json, tools/population_bench.py
#: --save-sources): the programs the search evaluates late in a run (long bodies,
#: ~12 GPU-list loops), frozen so every commit replays the same set
EVOLVED_SET = "config3_steady_r4f_children2048.json.gz"


def save_program_set(path: str, sources) -> None:
    """Program texts as template bodies where they are template-shaped
    (gzip JSON; `load_program_set` restores the exact text)."""
    import gzip
    import json
    from ..parallel.dist import program_body
    items = []
    for src in sources:
        body, templ = program_body(src)
        items.append({"b": body} if templ else {"s": src})
    with gzip.open(path, "wt", encoding="utf-8") as f:
        json.dump({"format": "fks-program-set-v1", "programs": items}, f)


def load_program_set(path: str) -> List[str]:
    import gzip
    import json
    from ..policy.template import PolicyTemplate
    with gzip.open(path, "rt", encoding="utf-8") as f:
        d = json.load(f)
    return [PolicyTemplate.fill_template(it["b"]) if "b" in it else it["s"] for it in d["programs"]]


def _compile_worker(sources):
    out = []
    for src in sources:
        try:
            out.append(compile_policy(src))
        except CompileError:
            out.append(None)
    return out


def evolved_children(n: int = 2048, workers: int = 8) -> List[CompiledPolicy]:
    """The frozen evolved-population children (EVOLVED_SET), compiled in
    `workers` spawned processes; device-capable ones, in file order."""
    import concurrent.futures
    import multiprocessing
    import os
    from .._paths import DATA_DIR
    srcs = load_program_set(os.path.join(DATA_DIR, "populations", EVOLVED_SET))[:n]
    if workers > 1 and len(srcs) > 64:
        parts = [srcs[i::workers] for i in range(workers)]
        with concurrent.futures.ProcessPoolExecutor(workers, mp_context=multiprocessing.get_context("spawn")) as ex:
            res = list(ex.map(_compile_worker, parts))
        progs = [None] * len(srcs)
        for w, part in enumerate(res):
            for j, p in enumerate(part):
                progs[w + j * workers] = p
    else:
        progs = _compile_worker(srcs)
    return [p for p in progs if p is not None and p.device_ok]


def service_rolling(dev, progs, seconds: float, chunk: int = 256, slots: int = 16, ref=None) -> dict:
    """Sustained programs/s through the resident program service
    (`DeviceEvaluator.start_service`), driven like the steady loop: `slots`
    batches of `chunk` programs in flight, each replaced when it completes;
    the first pass over `progs` is checked against `ref` rows."""
    import numpy as np
    n = len(progs)
    info = dev.start_service(slots=max(16384, 4 * chunk * slots), share=1.0)
    base = dev.SERVICE_SLOT_BASE
    nxt, done, inflight, lat = 0, 0, {}, []
    first = [None] * (-(-n // chunk))
    try:
        t0 = time.perf_counter()
        while True:
            for s in range(slots):
                if s not in inflight and time.perf_counter() - t0 < seconds:
                    lo = nxt % n
                    part = progs[lo:lo + chunk] if lo + chunk <= n else progs[lo:] + progs[:lo + chunk - n]
                    dev.submit_native(base + s, part)
                    inflight[s] = (time.perf_counter(), nxt)
                    nxt += chunk
            if not inflight:
                break
            busy = True
            for s in list(inflight):
                if dev.ready(base + s):
                    tab = dev.wait(base + s)
                    t_sub, at = inflight.pop(s)
                    lat.append(time.perf_counter() - t_sub)
                    if at + chunk <= n and at % chunk == 0:
                        first[at // chunk] = tab
                    done += chunk
                    busy = False
            if busy:
                time.sleep(0.0005)
        wall = time.perf_counter() - t0
    finally:
        dev.stop_service()
    rec = {"seconds": round(wall, 3), "programs": done, "evals_per_s": round(done / wall, 1), "chunk": chunk,
           "batches_in_flight": slots, "resident_workgroups": int(info["blocks"]),
           "batch_latency_mean_s": round(float(np.mean(lat)), 4) if lat else None}
    if ref is not None:
        parts = [(k, t) for k, t in enumerate(first) if t is not None]
        rec["checked"] = sum(len(t) for _, t in parts)
        rec["bit_identical"] = all(bool((t == ref[k * chunk:k * chunk + len(t)]).all()) for k, t in parts)
    return rec


def measure_evolved(dev, workload, n: int = 2048, compare: int = 128, cpu_threads: int = 0,
                    service_s: float = 0.0) -> dict:
    """The evolved-population children (EVOLVED_SET) at LLM-batch scale: split
    over the device's slots, all in flight at once, JIT included (first pass)
    and cached (second pass); mean replayed events, exception fraction, and the
    first `compare` rows checked against the CPU VM.  service_s > 0: also the
    sustained rate through the resident program service (`service_rolling`)."""
    import numpy as np
    from ..engine import COLS
    from ..ops import cpu_engine as ce
    t_c = time.perf_counter()
    progs = evolved_children(n)
    t_compile = time.perf_counter() - t_c
    n = len(progs)
    slots = max(1, dev.n_slots)
    size = -(-n // slots)
    chunks = [progs[i:i + size] for i in range(0, n, size)]
    dev.set_options(native_inflight=n)
    try:
        t0 = time.perf_counter()
        batches = [dev.submit_native(s, c) for s, c in enumerate(chunks)]
        tabs = [dev.wait(s) for s in range(len(chunks))]
        t1 = time.perf_counter()
        for s, c in enumerate(chunks):
            dev.submit_native(s, c)
        tabs2 = [dev.wait(s) for s in range(len(chunks))]
        t2 = time.perf_counter()
    finally:
        dev.set_options(native_inflight=0)
    tab, tab2 = np.concatenate(tabs), np.concatenate(tabs2)
    threads = cpu_threads or ce.default_threads()
    sub = progs[:compare]
    vm = ce.simulate_program_batch(workload, sub, threads=threads)
    skip = (100, 101)
    exc, vexc = tab[:compare, COLS["exc"]].astype(int), vm[:, COLS["exc"]].astype(int)
    cmp = ~np.isin(exc, skip) & ~np.isin(vexc, skip)
    a, b = tab[:compare], vm
    if not dev.options.get("trace_hash", True):
        a, b = a[:, :COLS["trace_hash_hi"]], b[:, :COLS["trace_hash_hi"]]
    st = dev.native_compiler.stats
    svc = service_rolling(dev, progs, service_s, ref=tab2) if service_s > 0 else None
    return {"programs": n, "source": f"data/populations/{EVOLVED_SET}", "bytecode_compile_s": round(t_compile, 3),
            "native": int(sum(int(b.ok.sum()) for b in batches)),
            "new_shapes": int(sum(int(b.compiled) for b in batches)),
            "evals_per_s_incl_jit": round(n / (t1 - t0), 1), "evals_per_s_cached": round(n / (t2 - t1), 1),
            "mean_events": round(float(tab[:, COLS["n_events"]].mean()), 1),
            "exception_fraction": round(float((tab[:, COLS["exc"]] != 0).mean()), 4),
            "repeat_identical": bool((tab == tab2).all()),
            "compared_vs_cpu_vm": int(cmp.sum()), "bit_identical": bool((a[cmp] == b[cmp]).all()),
            "baseline_shapes_total": int(st.get("baseline_shapes", 0)),
            **({"service": svc} if svc is not None else {})}
