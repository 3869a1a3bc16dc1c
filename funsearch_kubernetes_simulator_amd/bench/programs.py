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
