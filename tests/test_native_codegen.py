"""Native program backend (policy/native_codegen.py) on the CPU.

The generated C++ is the code the MI355X JIT compiles; built for the host with
g++ (FKS_HOST_JIT) and replayed by the C++ oracle engine it must reproduce the
CPU bytecode VM row for row -- score, every utilisation mean, snapshot and
fragmentation counts, exception class and the event-trace hash -- on the FULL
8,152-pod trace for every program of the corpus."""
import numpy as np
import pytest

from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
from funsearch_kubernetes_simulator_amd.policy.bytecode import Exc
from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy
from funsearch_kubernetes_simulator_amd.policy.native_codegen import (I, F, IF_, infer_types, module_source,
                                                                      shape_key, _loop_structure)
from funsearch_kubernetes_simulator_amd.policy.bytecode import unpack_code

from program_corpus import programs


def test_native_equals_vm_full_trace(default_workload):
    progs = programs()
    assert len(progs) >= 40
    nat = ce.simulate_native_batch(default_workload, progs, threads=8)
    vm = ce.simulate_program_batch(default_workload, progs, threads=8)
    for i, p in enumerate(progs):
        if int(vm[i, 10]) in (Exc.UNSUPPORTED, Exc.BUDGET) or int(nat[i, 10]) in (Exc.UNSUPPORTED, Exc.BUDGET):
            continue   # engines defer these to the next engine by design
        assert np.array_equal(nat[i], vm[i]), (i, p.source[-400:], nat[i], vm[i])


def test_constants_are_data_shapes_shared():
    a = compile_policy("def priority_function(pod, node):\n    return 1000 - node.cpu_milli_left * 0.25\n")
    b = compile_policy("def priority_function(pod, node):\n    return 2000 - node.cpu_milli_left * 0.75\n")
    c = compile_policy("def priority_function(pod, node):\n    return 1000.0 - node.cpu_milli_left * 0.25\n")
    assert shape_key(a) == shape_key(b)       # same code, other constants: one compiled function
    assert shape_key(a) != shape_key(c)       # a constant's int/float tag is part of the shape


def test_type_inference_proves_static_types():
    p = compile_policy("def priority_function(pod, node):\n"
                       "    x = pod.cpu_milli + 1\n"
                       "    y = x / 2\n"
                       "    z = x if node.gpu_left > 0 else y\n"
                       "    return z\n")
    code = unpack_code(p.code)
    types = infer_types(code, _loop_structure(code), p.ctag)
    seen = set()
    for pc, st in enumerate(types):
        seen.update(st.values())
    assert I in seen and F in seen and IF_ in seen   # z really is int-or-float; x and y are not


def test_module_source_compiles_for_host(tmp_path):
    from funsearch_kubernetes_simulator_amd.ops.jit import compile_host_module
    progs = programs()[:8]
    path = compile_host_module(progs, str(tmp_path / "m.so"))
    assert (tmp_path / "m.so").exists()
    src = module_source(progs)
    assert "fks_jit_table" in src and src.count("extern \"C\" __device__ __noinline__ int64_t fks_prog_") == 8


def test_node_gpus_index_specialisation_matches_vm(default_workload):
    """`for g in node.gpus` / `node.gpus[i]` on an unmodified GPU list are lowered
    to direct GPU indices (no 4-bit list unpacking): negative indices, index
    errors, len() and lists rebuilt in a branch must behave exactly as the VM."""
    srcs = [
        "def priority_function(pod, node):\n    return len(node.gpus) * 10 + node.gpus[-1].gpu_milli_left if node.gpus else 1\n",
        "def priority_function(pod, node):\n    gs = node.gpus\n    s = 0\n    for i in range(len(gs)):\n"
        "        s += gs[i].gpu_milli_left * (i + 1)\n    return s\n",
        "def priority_function(pod, node):\n    return node.gpus[3].gpu_milli_left + 1\n",        # IndexError on small nodes
        "def priority_function(pod, node):\n    gs = node.gpus\n    if pod.num_gpu > 1:\n        gs = gs[1:]\n"
        "    t = 0\n    for g in gs:\n        t += g.gpu_milli_left\n    return t + len(gs)\n",
        "def priority_function(pod, node):\n    best = 0\n    for g in node.gpus:\n        for h in node.gpus:\n"
        "            best = max(best, g.gpu_milli_left - h.gpu_milli_left)\n    return best + 1\n",
    ]
    progs = [compile_policy(s) for s in srcs]
    nat = ce.simulate_native_batch(default_workload, progs, threads=4)
    vm = ce.simulate_program_batch(default_workload, progs, threads=4)
    assert np.array_equal(nat, vm)
