"""Baseline program JIT (csrc/jit, ops/gcnjit.py) on the CPU: gfx950 encodings
against the ROCm assembler, generated code against the CPU VM through the
wave64 emulator (full replays and random single events), and the code-object
skeleton's layout / relocation arithmetic."""
import os
import random
import shutil
import subprocess

import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
from funsearch_kubernetes_simulator_amd.ops import gcnjit
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy
from funsearch_kubernetes_simulator_amd.policy.native_codegen import constant_block

from program_corpus import programs

MC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin", "llvm-mc")
have_mc = pytest.mark.skipif(not os.path.exists(MC), reason="ROCm llvm-mc not installed")
SKIP_EXC = (100, 101)   # UNSUPPORTED / BUDGET: the next engine decides


@pytest.fixture(scope="module")
def corpus():
    from funsearch_kubernetes_simulator_amd.bench.programs import mutation_children
    return programs() + mutation_children(24, seed=5)


def test_every_corpus_program_compiles(corpus):
    declined = []
    for p in corpus:
        code, why = gcnjit.compile_program(p)
        if code is None:
            declined.append(why)
        else:
            assert code.words.size > 10 and code.info["vgprs"] <= 128 and code.info["sgprs"] <= 96
    assert not declined, declined


@have_mc
def test_opcode_table_is_what_llvm_mc_assembles(tmp_path):
    """gcn_opcodes.inc regenerated from the assembler equals the checked-in table."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen", os.path.join(os.path.dirname(__file__), "..", "tools",
                                                                      "gen_gcn_opcodes.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    gen.OUT = str(tmp_path / "ops.inc")
    gen.main()
    ours = open(os.path.join(os.path.dirname(__file__), "..", "csrc", "jit", "gcn_opcodes.inc")).read()
    assert open(gen.OUT).read() == ours


@have_mc
def test_generated_code_round_trips_through_llvm_mc(corpus):
    """Every generated word decodes to a valid gfx950 instruction and
    re-assembles to the same bytes (canonical encodings, no stray bits)."""
    for p in corpus[::3]:
        code, why = gcnjit.compile_program(p)
        assert code is not None, why
        words = code.words.copy()
        for lo, hi, _ in code.relocs.reshape(-1, 3):   # as the loader patches them (never inline-encodable)
            words[int(lo)], words[int(hi)] = 0x12345678, 0xFFFFF000
        raw = words.tobytes()
        txt = " ".join(f"0x{b:02x}" for b in raw)
        dis = subprocess.run([MC, "-disassemble", "-triple=amdgcn-amd-amdhsa", "-mcpu=gfx950"], input=txt,
                             capture_output=True, text=True)
        assert dis.returncode == 0 and not dis.stderr.strip(), dis.stderr[:2000]
        # branch offsets are printed as immediates: re-assembling the listing gives the same words
        asm = "\n".join(line.strip() for line in dis.stdout.splitlines() if line.strip() and not line.strip().startswith("."))
        re = subprocess.run([MC, "-triple=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-show-encoding"], input=asm,
                            capture_output=True, text=True)
        assert re.returncode == 0, re.stderr[:2000]
        out = bytearray()
        for line in re.stdout.splitlines():
            if "encoding: [" in line:
                out += bytes(int(x, 16) for x in line.split("encoding: [")[1].rstrip("]").split(","))
        assert bytes(out) == raw


@have_mc
def test_no_integer_inline_constants_in_f64_value_operands(corpus):
    """In a 64-bit float operand an integer inline constant is a bit pattern
    (1 -> 4.9e-324), not a converted value: generated f64 arithmetic / compares
    use the float inline constants (0.5, 1.0, 2.0, 4.0, ...) or 0 only."""
    import re
    bodies = ["x = node.cpu_milli_left / node.cpu_milli_total\n    return (1 - x) * 2.0 + (x > 1) * 4 - (x < 0.5) * 3"]
    progs = list(corpus[::4]) + [compile_policy("def priority_function(pod, node):\n    " + b + "\n") for b in bodies]
    bad = []
    for p in progs:
        code, why = gcnjit.compile_program(p)
        assert code is not None, why
        words = code.words.copy()
        for lo, hi, _ in code.relocs.reshape(-1, 3):
            words[int(lo)], words[int(hi)] = 0x12345678, 0xFFFFF000
        txt = " ".join(f"0x{b:02x}" for b in words.tobytes())
        dis = subprocess.run([MC, "-disassemble", "-triple=amdgcn-amd-amdhsa", "-mcpu=gfx950"], input=txt,
                             capture_output=True, text=True).stdout
        for line in dis.splitlines():
            line = line.strip()
            op = line.split(" ")[0]
            if not op.startswith("v_") or "_f64" not in op or op.startswith(("v_ldexp_f64", "v_cmp_class_f64")):
                continue
            for tok in re.split(r"[ ,]+", line)[1:]:
                if re.fullmatch(r"-?\d+", tok) and int(tok) != 0:
                    bad.append(line)
    assert not bad, bad[:5]


def test_emulated_replays_equal_cpu_vm(default_workload, corpus):
    """Full replays of the 8,152-pod trace with the generated machine code on
    the wave64 emulator: rows bit-identical to the CPU VM."""
    budget = 1 << 16   # runaway loops end quickly on both (BUDGET rows are skipped)
    vm_all = ce.simulate_program_batch(default_workload, corpus, ce.SimOptions(budget=budget))
    # the emulator runs ~10^7 instructions / s: replays with millions of events
    # (a repush-heavy program, 2M events) are left to the GPU tests
    keep = [i for i in range(0, len(corpus), 2) if vm_all[i, 8] < 60000]
    progs = [corpus[i] for i in keep]
    vm = vm_all[keep]
    emu = gcnjit.emulate_programs(default_workload, progs, budget, ce.SimOptions(budget=budget))
    compared = 0
    for i, p in enumerate(progs):
        if int(emu[i, 10]) in SKIP_EXC or int(vm[i, 10]) in SKIP_EXC:
            continue
        assert np.array_equal(emu[i], vm[i]), (i, p.source[-300:], emu[i], vm[i])
        compared += 1
    assert len(keep) >= len(corpus) // 2 - 4 and compared >= len(progs) - 4


def test_emulated_replays_without_prologue_equal_cpu_vm(default_workload, corpus):
    """Full replays as the device runs them: the feasibility prologue compiled
    out and the program called for feasible nodes only -- rows bit-identical
    to the CPU VM running the whole program on every node."""
    budget = 1 << 16
    progs = [p for p in corpus if gcnjit.elide_range(p)[1]][::2]
    assert len(progs) >= 8
    vm = ce.simulate_program_batch(default_workload, progs, ce.SimOptions(budget=budget))
    keep = [i for i in range(len(progs)) if vm[i, 8] < 60000]
    progs, vm = [progs[i] for i in keep], vm[keep]
    emu = gcnjit.emulate_programs(default_workload, progs, budget, ce.SimOptions(budget=budget), elide=True)
    compared = 0
    for i, p in enumerate(progs):
        if int(emu[i, 10]) in SKIP_EXC or int(vm[i, 10]) in SKIP_EXC:
            continue
        assert np.array_equal(emu[i], vm[i]), (i, p.source[-300:], emu[i], vm[i])
        compared += 1
    assert compared >= len(progs) - 2


def _finish(kind, v):
    if kind == "exc":
        return -v
    if kind == "none":
        return -4
    if kind == "int":
        return max(0, v)
    if v != v or not v > 0:
        return 0
    if v == float("inf"):
        return -3
    if v >= 2 ** 63:
        return -100
    return int(v)


def _random_event(rng, n=16):
    node, gl, gt, gm = [], [], [], []
    for _ in range(n):
        ct = rng.choice([32000, 64000, 96000, 128000])
        mt = rng.choice([131072, 262144, 786432])
        ng = rng.choice([0, 1, 2, 4, 8])
        gls = [rng.choice([0, 1000, rng.randint(0, 1000)]) for _ in range(ng)] + [0] * (8 - ng)
        node += [rng.randint(0, ct), ct, rng.randint(0, mt), mt, sum(1 for x in gls[:ng] if x == 1000), ng]
        gl += gls
        gt += [1000] * ng + [0] * (8 - ng)
        gm += [16384] * ng + [0] * (8 - ng)
    pod = [rng.choice([0, 1000, 4000, rng.randint(0, 96000)]), rng.choice([0, 1024, rng.randint(0, 400000)]),
           rng.choice([0, 0, 1, 1, 2, 8]), rng.choice([0, 1000, rng.randint(0, 1000)]), rng.randint(0, 10 ** 7),
           rng.randint(0, 10 ** 6)]
    pod[3] = 1000 if pod[2] > 1 else (0 if pod[2] == 0 else pod[3])
    return node, gl, gt, gm, pod


def test_single_events_equal_cpu_vm_on_random_states(corpus):
    """One emulated wave (lanes = 16 nodes, divergent control flow) per random
    cluster state vs the VM per node: int(max(0, score)) or the exception."""
    m = ce.native()
    rng = random.Random(3)
    for p in corpus[::2]:
        kc = constant_block(p, 1 << 16).tolist()
        lit = gcnjit.literal_mask(p).tolist()
        for _ in range(6):
            node, gl, gt, gm, pod = _random_event(rng)
            emu = m.gcn_emu_event(p.code, list(map(int, p.ctag)), lit, list(map(int, p.iconst)),
                                  list(map(float, p.fconst)), kc, node, gl, gt, gm, pod)
            podd = dict(cpu_milli=pod[0], memory_mib=pod[1], num_gpu=pod[2], gpu_milli=pod[3], creation_time=pod[4],
                        duration_time=pod[5])
            for n in range(16):
                nd = dict(cpu_milli_left=node[6 * n], cpu_milli_total=node[6 * n + 1], memory_mib_left=node[6 * n + 2],
                          memory_mib_total=node[6 * n + 3], gpu_left=node[6 * n + 4])
                ng = node[6 * n + 5]
                k, v = m.score_program_once(p.code, list(p.fconst), list(p.iconst), list(p.ctag), podd, nd,
                                            gl[8 * n:8 * n + ng], gt[8 * n:8 * n + ng], gm[8 * n:8 * n + ng])
                ref = _finish(k, v)
                if ref in (-100, -101) or emu[n] in (-100, -101):
                    continue
                assert emu[n] == ref, (p.source[-300:], n, pod, node[6 * n:6 * n + 6], (k, v), emu[n])


def _check_bodies(bodies, seed, events=8):
    """Each body as a program: one emulated wave per random event == the VM per node."""
    m = ce.native()
    rng = random.Random(seed)
    for body in bodies:
        p = compile_policy("def priority_function(pod, node):\n    " + body + "\n")
        kc = constant_block(p, 1 << 16).tolist()
        for _ in range(events):
            node, gl, gt, gm, pod = _random_event(rng)
            emu = m.gcn_emu_event(p.code, list(map(int, p.ctag)), gcnjit.literal_mask(p).tolist(),
                                  list(map(int, p.iconst)), list(map(float, p.fconst)), kc, node, gl, gt, gm, pod)
            podd = dict(cpu_milli=pod[0], memory_mib=pod[1], num_gpu=pod[2], gpu_milli=pod[3], creation_time=pod[4],
                        duration_time=pod[5])
            for n in range(16):
                nd = dict(cpu_milli_left=node[6 * n], cpu_milli_total=node[6 * n + 1], memory_mib_left=node[6 * n + 2],
                          memory_mib_total=node[6 * n + 3], gpu_left=node[6 * n + 4])
                ng = node[6 * n + 5]
                k, v = m.score_program_once(p.code, list(p.fconst), list(p.iconst), list(p.ctag), podd, nd,
                                            gl[8 * n:8 * n + ng], gt[8 * n:8 * n + ng], gm[8 * n:8 * n + ng])
                ref = _finish(k, v)
                if ref in (-100, -101) or emu[n] in (-100, -101):
                    continue
                assert emu[n] == ref, (body, n, (k, v), emu[n])


GPU_LOOP_BODIES = [
    # node.gpus loops: counter-indexed GPU fields (GPR index mode), unchecked GETs
    "c = 0\n    for gpu in node.gpus:\n        if gpu.gpu_milli_left >= pod.gpu_milli:\n            c += 1\n"
    "    return c * 10 + 1",
    "return sum(g.gpu_milli_left for g in node.gpus) + 3 * len([g for g in node.gpus if g.gpu_milli_total > 0])",
    "return max(g.gpu_milli_total - g.gpu_milli_left for g in node.gpus)",
    "t = 0\n    for i, g in enumerate(node.gpus):\n        t += i * g.gpu_milli_left + g.memory_mib_left % 7\n    return t",
    # the outer element inside an inner loop, and after its loop (per-lane last GPU)
    "t = 0\n    for g in node.gpus:\n        for h in node.gpus:\n            if h.gpu_milli_left > g.gpu_milli_left:\n"
    "                t += g.gpu_milli_total - h.gpu_milli_left\n    return t",
    "t = 1\n    g = node.gpus[0]\n    for g in node.gpus:\n        t += 1\n    return t * 1000 + g.gpu_milli_left",
    # the loop variable reassigned in the body; loops over other lists
    "t = 0\n    for g in node.gpus:\n        if g.gpu_milli_left < 500:\n            g = node.gpus[0]\n"
    "        t += g.gpu_milli_left\n    return t",
    "a = [g for g in node.gpus if g.gpu_milli_left > 100]\n    t = 0\n    for g in a:\n"
    "        t += g.gpu_milli_total - g.gpu_milli_left\n    return t + len(a)",
    "gs = node.gpus\n    if pod.num_gpu > 1:\n        gs = gs[1:]\n    t = 0\n    for g in gs:\n"
    "        t += g.gpu_milli_left\n    return t",
    "t = 0\n    for g in node.gpus:\n        if g.gpu_milli_left == 0:\n            continue\n        if t > 1500:\n"
    "            break\n        t += g.gpu_milli_left\n    return t",
    "s = sorted(node.gpus, key=lambda g: -g.gpu_milli_left)\n    return s[0].gpu_milli_left * 2 + s[-1].gpu_milli_total",
]


SMALL_POW_BODIES = [
    "x = node.cpu_milli_left / node.cpu_milli_total\n    return (x ** 2 + x ** 3 - x ** 1) * 1e6",
    "x = (node.memory_mib_left - pod.memory_mib) / 7.0\n    return x ** 3 + x ** 2 * 3.5 + (x - 1) ** 1",
    "x = (pod.cpu_milli - node.cpu_milli_left) * 1e-300\n    return (x ** 2) * 1e300 + (x * 1e150) ** 3",
    "x = 0.0 if node.gpu_left == 0 else node.cpu_milli_left / node.gpu_left\n    return x ** 2 - node.cpu_milli_left ** 2 / 1e3",
    "x = float(2 ** (node.gpu_left + 1))\n    return x ** 2 + x ** 3 + x ** 1",
    "x = node.cpu_milli_left * 1e200\n    return min(x ** 2, 1e300) + min(x ** 3, 1e308)",
]


def test_small_integer_powers_equal_cpu_vm():
    """float ** 1 / 2 / 3 inlined by the JIT (glibc pow's 0.52-ULP bound:
    lanes near a rounding boundary, zeros, powers of two, underflow and
    overflow take the runtime pow) == the VM, which runs glibc's pow."""
    _check_bodies(SMALL_POW_BODIES, seed=31, events=12)


def test_elided_feasibility_prologue_equals_cpu_vm_on_feasible_nodes(corpus):
    """Code compiled without the template's feasibility prologue (the kernels
    call such programs for feasible nodes only) scores every feasible node as
    the whole program does on the VM; a body that reads the prologue's GPU
    count keeps its prologue."""
    m = ce.native()
    rng = random.Random(41)
    elided = 0
    for p in corpus:
        lo, hi = gcnjit.elide_range(p)
        if not hi:
            continue
        r = m.gcn_compile_many([(p.code, np.asarray(p.ctag, np.uint8), gcnjit.literal_mask(p),
                                 np.asarray(p.iconst, np.int64), np.asarray(p.fconst, np.float64), lo, hi)], 1)[0]
        assert r["ok"], r["reason"]
        if not r["elided"]:
            continue
        elided += 1
        kc = constant_block(p, 1 << 16).tolist()
        for _ in range(4):
            node, gl, gt, gm, pod = _random_event(rng)
            emu = m.gcn_emu_event(p.code, list(map(int, p.ctag)), gcnjit.literal_mask(p).tolist(),
                                  list(map(int, p.iconst)), list(map(float, p.fconst)), kc, node, gl, gt, gm, pod,
                                  elide_lo=lo, elide_hi=hi)
            podd = dict(cpu_milli=pod[0], memory_mib=pod[1], num_gpu=pod[2], gpu_milli=pod[3], creation_time=pod[4],
                        duration_time=pod[5])
            for n in range(16):
                nd = dict(cpu_milli_left=node[6 * n], cpu_milli_total=node[6 * n + 1], memory_mib_left=node[6 * n + 2],
                          memory_mib_total=node[6 * n + 3], gpu_left=node[6 * n + 4])
                ng = node[6 * n + 5]
                free = sum(1 for j in range(ng) if gl[8 * n + j] >= pod[3])
                feasible = (pod[0] <= nd["cpu_milli_left"] and pod[1] <= nd["memory_mib_left"] and
                            pod[2] <= nd["gpu_left"] and (pod[2] == 0 or free >= pod[2]))
                if not feasible:
                    continue
                k, v = m.score_program_once(p.code, list(p.fconst), list(p.iconst), list(p.ctag), podd, nd,
                                            gl[8 * n:8 * n + ng], gt[8 * n:8 * n + ng], gm[8 * n:8 * n + ng])
                ref = _finish(k, v)
                if ref in (-100, -101) or emu[n] in (-100, -101):
                    continue
                assert emu[n] == ref, (p.source[-300:], n, (k, v), emu[n])
    assert elided >= 10
    from funsearch_kubernetes_simulator_amd.policy.template import PolicyTemplate
    reads = compile_policy(PolicyTemplate.TEMPLATE.replace(
        "{llm_generated_logic}", "score = 100 + (available_gpus if pod.num_gpu > 0 else 0)"))
    lo, hi = gcnjit.elide_range(reads)
    assert hi > lo
    r = m.gcn_compile_many([(reads.code, np.asarray(reads.ctag, np.uint8), gcnjit.literal_mask(reads),
                             np.asarray(reads.iconst, np.int64), np.asarray(reads.fconst, np.float64), lo, hi)], 1)[0]
    assert r["ok"] and not r["elided"]


def test_runaway_loop_raises_budget():
    """The loop budget is one counter per wave (kc[0], capped): a program that
    never leaves its loop raises BUDGET in every lane (the next engine decides)."""
    m = ce.native()
    p = compile_policy("def priority_function(pod, node):\n    x = 0\n    while x >= 0:\n"
                       "        x = (x + 1) % 7\n    return x\n")
    node, gl, gt, gm, pod = _random_event(random.Random(5))
    for budget in (1 << 10, 1 << 16, 0):   # (0: unlimited -> the per-call cap)
        kc = constant_block(p, budget).tolist()
        emu = m.gcn_emu_event(p.code, list(map(int, p.ctag)), gcnjit.literal_mask(p).tolist(),
                              list(map(int, p.iconst)), list(map(float, p.fconst)), kc, node, gl, gt, gm, pod)
        assert list(emu) == [-101] * 16


def test_exhausted_budget_stays_exhausted():
    """Lanes that were outside EXEC when the budget ran out (here: the other
    branch of an if) must not get a wrapped ~2^32 budget for a later loop:
    they raise BUDGET within the cap like every other lane."""
    m = ce.native()
    p = compile_policy("def priority_function(pod, node):\n    x = 0\n"
                       "    if node.cpu_milli_left % 2 == 0:\n        while x >= 0:\n"
                       "            x = (x + 1) % 7\n    y = 0\n    for i in range(5000):\n"
                       "        y += 1\n    return x + y\n")
    rng = random.Random(11)
    for _ in range(20):
        node, gl, gt, gm, pod = _random_event(rng)
        even = [node[6 * j] % 2 == 0 for j in range(16)]
        if any(even) and not all(even):
            break
    else:
        raise AssertionError("no mixed event")
    kc = constant_block(p, 1 << 10).tolist()
    emu = m.gcn_emu_event(p.code, list(map(int, p.ctag)), gcnjit.literal_mask(p).tolist(),
                          list(map(int, p.iconst)), list(map(float, p.fconst)), kc, node, gl, gt, gm, pod)
    assert list(emu) == [-101] * 16
    # with a budget above both loops' needs, the odd lanes finish
    p2 = compile_policy(p.source.replace("while x >= 0", "while x >= 0 and x < 3"))
    kc = constant_block(p2, 1 << 20).tolist()
    emu = m.gcn_emu_event(p2.code, list(map(int, p2.ctag)), gcnjit.literal_mask(p2).tolist(),
                          list(map(int, p2.iconst)), list(map(float, p2.fconst)), kc, node, gl, gt, gm, pod)
    assert list(emu) == [5003 if e else 5000 for e in even]


@pytest.mark.parametrize("unroll", [True, False])
def test_gpu_list_loops_equal_cpu_vm(unroll):
    """The compiler's GPU-list loop skeletons (bytecode LOOP_INDEX): unchecked
    gets, 32-bit counters and, for node.gpus, fields read with the counter in
    GPR index mode -- and the cases that must not take that path (outer
    element in an inner loop, after the loop, reassigned, other lists); node.gpus
    loops both unrolled (the default) and rolled."""
    m = ce.native()
    old = m.gcn_set_unroll_cap(0 if not unroll else 1600)
    try:
        _check_bodies(GPU_LOOP_BODIES, seed=21)
    finally:
        m.gcn_set_unroll_cap(old)


@have_mc
def _disassemble(code):
    txt = " ".join(f"0x{b:02x}" for b in code.words.tobytes())
    return subprocess.run([MC, "-disassemble", "-triple=amdgcn-amd-amdhsa", "-mcpu=gfx950"], input=txt,
                          capture_output=True, text=True).stdout


@have_mc
def test_node_gpus_loop_indexes_fields_uniformly():
    """Rolled (unrolling off): the counter-indexed field read in GPR index mode;
    unrolled (the default): eight guarded copies, each reading its GPU's field
    straight from the argument VGPR, no counter, no back edge."""
    m = ce.native()
    p = compile_policy("def priority_function(pod, node):\n    " + GPU_LOOP_BODIES[0] + "\n")
    old = m.gcn_set_unroll_cap(0)
    try:
        code, why = gcnjit.compile_program(p)
    finally:
        m.gcn_set_unroll_cap(old)
    assert code is not None, why
    dis = _disassemble(code)
    assert dis.count("s_set_gpr_idx_on") == 1 and dis.count("s_set_gpr_idx_off") == 1
    assert "v_cmp_lt_i32" in dis
    code, why = gcnjit.compile_program(p)
    assert code is not None, why
    assert code.info["unrolled"] == 1
    dis = _disassemble(code)
    assert "s_set_gpr_idx_on" not in dis and "s_cbranch_scc0" not in dis   # (no budget charge: no back edge)
    for k in range(8):
        assert f"v_mov_b32_e32 v{{}}, v{5 + k}".split("{}")[1] in dis


def test_evolved_population_compiles_natively():
    """Register pressure on real evolved programs (a steady-mode population:
    long, bloated bodies): the baseline JIT takes nearly all of them (a decline
    sends a program to the device VM)."""
    import json
    pops = os.path.join(os.path.dirname(__file__), "..", "data", "populations")
    codes = []

    def walk(o):
        if isinstance(o, dict):
            if isinstance(o.get("code"), str):
                codes.append(o["code"])
            for v in o.values():
                walk(v)
        elif isinstance(o, list):
            if len(o) == 2 and isinstance(o[0], str) and isinstance(o[1], (int, float)):
                codes.append(o[0])   # [code, score] members
            else:
                for v in o:
                    walk(v)
    for name in ("config3_steady_r4_islands.json", "config3_steady_r4f_islands.json"):
        walk(json.load(open(os.path.join(pops, name))))
    codes = sorted(set(codes))
    assert len(codes) >= 48
    declined = []
    for src in codes:
        p = compile_policy(src)
        if not p.device_ok:
            continue
        code, why = gcnjit.compile_program(p)
        if code is None:
            declined.append(why)
    assert len(declined) <= len(codes) // 32, declined


def test_dynamic_types_runtime_calls_and_lists():
    """Programs whose registers change type at run time (runtime-library calls,
    tag bits), GPU-list slicing / insertion / sorting, and exceptions."""
    bodies = [
        "s = 0.0\n    if pod.cpu_milli > 30000:\n        s = int(pod.cpu_milli * 0.05)\n    s = max(1, s)\n"
        "    if node.cpu_milli_left > pod.cpu_milli * 2:\n        s += 54.111\n    return max(1, int(s))",
        "x = node.cpu_milli_left ** 0.5 + (node.memory_mib_left % 7) // 2\n    return x",
        "g = sorted(node.gpus, key=lambda g: g.gpu_milli_left)[:2]\n    t = 0\n"
        "    for q in g:\n        t += q.gpu_milli_left\n    return t + len(g) * 3",
        "v = node.cpu_milli_left / (node.gpu_left - 1)\n    return v",
        "a = [g for g in node.gpus if g.gpu_milli_left > 100]\n    return max(1, len(a) * 100 - node.gpus[0].gpu_milli_left)",
        "r = round(node.memory_mib_left / 3.0) + abs(pod.cpu_milli - node.cpu_milli_left)\n    return -r if r % 2 else r",
    ]
    _check_bodies(bodies, seed=11)


def test_skeleton_layout_and_relocations():
    if not shutil.which(gcnjit.CLANG) and not os.path.exists(gcnjit.CLANG):
        pytest.skip("ROCm clang not installed")
    sk = gcnjit.Skeleton.load(gcnjit.SKELETON_SIZES[0])
    assert sk.arena_vaddr % gcnjit.PROGRAM_ALIGN == 0 and sk.capacity > 200_000
    assert sk.image[sk.arena_off:sk.arena_off + 4] == bytes.fromhex("000081bf")   # s_endpgm filler
    p = compile_policy("def priority_function(pod, node):\n    return node.cpu_milli_left ** 0.5\n")
    code, _ = gcnjit.compile_program(p)
    assert code.relocs.size == 3 * code.info["calls"] and code.info["calls"] == 1
    lo, hi, pc = (int(x) for x in code.relocs[:3])
    # the two literal slots follow s_add_u32 / s_addc_u32 words of the runtime-table address
    assert code.words[lo - 1] >> 23 == 0x100 and code.words[hi - 1] >> 23 == 0x104
    assert pc % 4 == 0 and pc < code.words.size * 4


def test_llvm_tier_disk_cache(tmp_path, monkeypatch):
    """LLVM-tier code objects persist on disk (shared by ranks / restarts):
    the second build of the same module is a cache hit with the same image."""
    from funsearch_kubernetes_simulator_amd.ops import jit
    if not os.path.exists(jit.CLANG):
        pytest.skip("ROCm clang not installed")
    monkeypatch.setenv("FKS_JIT_CACHE", str(tmp_path / "cache"))
    p = compile_policy("def priority_function(pod, node):\n    return node.cpu_milli_left - pod.cpu_milli // 3\n")
    a = jit.compile_device_module([p])
    b = jit.compile_device_module([p])
    assert not a.cached and b.cached and a.image == b.image and a.resources == b.resources
    assert b.compile_s < a.compile_s
    assert len(list((tmp_path / "cache").glob("*.co"))) == 1
    # a cached image whose bytes no longer match its recorded sha256 is a miss
    co = next((tmp_path / "cache").glob("*.co"))
    raw = bytearray(co.read_bytes())
    raw[-1] ^= 0xFF
    co.write_bytes(bytes(raw))
    assert not jit.compile_device_module([p]).cached
    monkeypatch.setenv("FKS_JIT_CACHE", "off")
    assert not jit.compile_device_module([p]).cached


def test_skeleton_provenance_rebuilds_stale_files(tmp_path, monkeypatch):
    """A skeleton is reused only if built from the current source and its bytes
    are unchanged; an edited source or a modified file triggers a rebuild."""
    if not os.path.exists(gcnjit.CLANG):
        pytest.skip("ROCm clang not installed")
    monkeypatch.setattr(gcnjit, "skeleton_path", lambda size: tmp_path / f"skel_{size >> 10}k.co")
    size = gcnjit.SKELETON_SIZES[0]
    path = gcnjit.build_skeleton(size)
    assert gcnjit.skeleton_is_current(size)
    raw = bytearray(path.read_bytes())
    raw[100] ^= 0xFF
    path.write_bytes(bytes(raw))
    assert not gcnjit.skeleton_is_current(size)
    gcnjit.build_skeleton(size)
    assert gcnjit.skeleton_is_current(size)
    monkeypatch.setattr(gcnjit, "SKELETON_SOURCE", gcnjit.SKELETON_SOURCE + "// edited\n")
    assert not gcnjit.skeleton_is_current(size)


def test_per_lane_pods_several_rows_in_one_call(corpus):
    """The four-programs-per-wave row kernel can call one shape for several
    DPP rows at once, each row with its own pod: every pod field is per lane."""
    m = ce.native()
    rng = random.Random(17)
    for p in corpus[::3]:
        kc = constant_block(p, 1 << 16).tolist()
        lit = gcnjit.literal_mask(p).tolist()
        node, gl, gt, gm, _ = _random_event(rng, n=64)
        pods = [_random_event(rng, n=1)[4] for _ in range(4)]          # one pod per 16-lane row
        per_lane = [x for l in range(64) for x in pods[l // 16]]
        emu = m.gcn_emu_event(p.code, list(map(int, p.ctag)), lit, list(map(int, p.iconst)),
                              list(map(float, p.fconst)), kc, node, gl, gt, gm, per_lane)
        for n in range(0, 64, 5):
            pod = pods[n // 16]
            podd = dict(cpu_milli=pod[0], memory_mib=pod[1], num_gpu=pod[2], gpu_milli=pod[3], creation_time=pod[4],
                        duration_time=pod[5])
            nd = dict(cpu_milli_left=node[6 * n], cpu_milli_total=node[6 * n + 1], memory_mib_left=node[6 * n + 2],
                      memory_mib_total=node[6 * n + 3], gpu_left=node[6 * n + 4])
            ng = node[6 * n + 5]
            k, v = m.score_program_once(p.code, list(p.fconst), list(p.iconst), list(p.ctag), podd, nd,
                                        gl[8 * n:8 * n + ng], gt[8 * n:8 * n + ng], gm[8 * n:8 * n + ng])
            ref = _finish(k, v)
            if ref in (-100, -101) or emu[n] in (-100, -101):
                continue
            assert emu[n] == ref, (p.source[-300:], n, pod, (k, v), emu[n])


@pytest.mark.parametrize("cap", [2, 3])
def test_spilled_registers_equal_cpu_vm(corpus, cap):
    """Register pressure beyond the pairs: with the pool capped at `cap` pairs
    ordinary programs spill virtual registers to per-lane scratch slots
    (reloaded per instruction, stored back after, the runtime calls' save area
    above the slots).  Emulated single events stay equal to the VM."""
    m = ce.native()
    rng = random.Random(17 + cap)
    progs = corpus[::3] + [compile_policy("def priority_function(pod, node):\n    " + b + "\n") for b in (
        "s = 0.0\n    if pod.cpu_milli > 30000:\n        s = int(pod.cpu_milli * 0.05)\n    s = max(1, s)\n"
        "    if node.cpu_milli_left > pod.cpu_milli * 2:\n        s += 54.111\n    return max(1, int(s))",
        "x = node.cpu_milli_left ** 0.5 + (node.memory_mib_left % 7) // 2\n    return x",
        "g = sorted(node.gpus, key=lambda g: g.gpu_milli_left)[:2]\n    t = 0\n"
        "    for q in g:\n        t += q.gpu_milli_left\n    return t + len(g) * 3",
        "a = node.cpu_milli_left; b = node.memory_mib_left; c = node.gpu_left; d = pod.cpu_milli\n"
        "    e = a * 2 + b; f = b - c * 3; g2 = (a + d) / max(1, b); h = e * f - g2\n"
        "    return a + b + c + d + e + f + g2 + h")]
    m.gcn_set_pair_cap(cap)
    try:
        spilled = 0
        for p in progs:
            info = m.gcn_compile(p.code, list(map(int, p.ctag)), gcnjit.literal_mask(p).tolist(),
                                 list(map(int, p.iconst)), list(map(float, p.fconst)))
            if not info["ok"]:
                assert "VGPR" in info["reason"] or "spilled register" in info["reason"], info["reason"]
                continue
            spilled += info["spills"] > 0
            kc = constant_block(p, 1 << 16).tolist()
            for _ in range(4):
                node, gl, gt, gm, pod = _random_event(rng)
                emu = m.gcn_emu_event(p.code, list(map(int, p.ctag)), gcnjit.literal_mask(p).tolist(),
                                      list(map(int, p.iconst)), list(map(float, p.fconst)), kc, node, gl, gt, gm, pod)
                podd = dict(cpu_milli=pod[0], memory_mib=pod[1], num_gpu=pod[2], gpu_milli=pod[3],
                            creation_time=pod[4], duration_time=pod[5])
                for n in range(16):
                    nd = dict(cpu_milli_left=node[6 * n], cpu_milli_total=node[6 * n + 1],
                              memory_mib_left=node[6 * n + 2], memory_mib_total=node[6 * n + 3],
                              gpu_left=node[6 * n + 4])
                    ng = node[6 * n + 5]
                    k, v = m.score_program_once(p.code, list(p.fconst), list(p.iconst), list(p.ctag), podd, nd,
                                                gl[8 * n:8 * n + ng], gt[8 * n:8 * n + ng], gm[8 * n:8 * n + ng])
                    ref = _finish(k, v)
                    if ref in (-100, -101) or emu[n] in (-100, -101):
                        continue
                    assert emu[n] == ref, (p.source[-300:], n, (k, v), emu[n], info["spills"])
        assert spilled >= len(progs) // 4, (spilled, len(progs))
    finally:
        m.gcn_set_pair_cap(0)


@have_mc
def test_spilled_code_round_trips_through_llvm_mc(corpus):
    """Spill slots and the runtime calls' saves and restores encode
    as the assembler does (scratch_*_dword at s32 offsets)."""
    m = ce.native()
    m.gcn_set_pair_cap(2)
    try:
        done = 0
        for p in corpus[::4]:
            code, _ = gcnjit.compile_program(p)
            if code is None or code.info["spills"] == 0:
                continue
            words = code.words.copy()
            for lo, hi, _ in code.relocs.reshape(-1, 3):
                words[int(lo)], words[int(hi)] = 0x12345678, 0xFFFFF000
            raw = words.tobytes()
            dis = subprocess.run([MC, "-disassemble", "-triple=amdgcn-amd-amdhsa", "-mcpu=gfx950"],
                                 input=" ".join(f"0x{b:02x}" for b in raw), capture_output=True, text=True)
            assert dis.returncode == 0 and not dis.stderr.strip(), dis.stderr[:2000]
            asm = "\n".join(ln.strip() for ln in dis.stdout.splitlines() if ln.strip() and not ln.strip().startswith("."))
            assert "scratch_load_dword" in asm and "scratch_store_dword" in asm
            re = subprocess.run([MC, "-triple=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-show-encoding"], input=asm,
                                capture_output=True, text=True)
            out = bytearray()
            for line in re.stdout.splitlines():
                if "encoding: [" in line:
                    out += bytes(int(x, 16) for x in line.split("encoding: [")[1].rstrip("]").split(","))
            assert bytes(out) == raw
            done += 1
        assert done >= 3
    finally:
        m.gcn_set_pair_cap(0)
