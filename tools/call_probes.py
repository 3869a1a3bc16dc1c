"""Call-cost probes of the native program path: small programs that repeat
one construct (dependent float arithmetic, if-blocks, GPU aggregates,
divisions, ...) behind the template's feasibility prologue, so the per-event
cycles of the scoring wave's call (tools/duo_phase.py --probes, on the GPU)
divided by the executed wave instructions per event (tools/jit_profile.py
--set probes, on the CPU emulator) give a cycles-per-instruction figure for
each construct.

    python tools/call_probes.py            # lists the probes
"""
from __future__ import annotations

FEAS = """def priority_function(pod, node):
    if (pod.cpu_milli > node.cpu_milli_left or
        pod.memory_mib > node.memory_mib_left or
        pod.num_gpu > node.gpu_left):
        return 0
    if pod.num_gpu > 0:
        available_gpus = 0
        for gpu in node.gpus:
            if gpu.gpu_milli_left >= pod.gpu_milli:
                available_gpus += 1
        if available_gpus < pod.num_gpu:
            return 0
"""


def _rep(lines, n):
    return "".join("    " + ln.format(i=i, k=1.0 + 0.01 * i) + "\n" for i in range(n) for ln in lines)


PROBES = {
    # nothing but the (elided) prologue and a return: the fixed call cost
    "empty": FEAS + "    return 1\n",
    # 64 dependent float multiply-adds
    "fchain": FEAS + "    s = node.cpu_milli_left * 0.5\n" + _rep(["s = s * {k} + 0.25"], 64) + "    return s\n",
    # 64 independent-ish int adds (int64, overflow-checked or not)
    "ichain": FEAS + "    s = node.cpu_milli_left\n" + _rep(["s = s + node.memory_mib_left - {i}"], 32) + "    return s\n",
    # 32 if-blocks with a float add each (divergent across nodes)
    "ifs": FEAS + "    s = 0.0\n" + _rep(["if node.cpu_milli_left > {i} * 1000:", "    s += {k}"], 32) + "    return s\n",
    # 16 float divisions
    "divs": FEAS + "    s = 0.0\n" + _rep(["s += node.cpu_milli_left / max(1, pod.cpu_milli + {i})"], 16) + "    return s\n",
    # 8 GPU aggregates over node.gpus (generator expressions)
    "gsum": FEAS + "    s = 0.0\n" + _rep(["s += sum(g.gpu_milli_left - pod.gpu_milli + {i} for g in node.gpus"
                                           " if g.gpu_milli_left >= pod.gpu_milli) / 1000"], 8) + "    return s\n",
    "gmax": FEAS + "    s = 0\n" + _rep(["s += max(g.gpu_milli_left + {i} for g in node.gpus) if node.gpus else 0"], 8) + "    return s\n",
    "gcount": FEAS + "    s = 0\n" + _rep(["s += sum(1 for g in node.gpus if 0 < g.gpu_milli_left < {i} * 100 + 100)"], 8)
    + "    return s\n",
    # min / max builtins over scalars, abs
    "minmax": FEAS + "    s = 0.0\n" + _rep(["s += min(node.cpu_milli_left / 1000, max(pod.cpu_milli, {i}) / 100)"], 16)
    + "    return s\n",
    # float ** and math.exp / log through the runtime library
    "pow": FEAS + "    s = 0.0\n" + _rep(["s += (node.cpu_milli_left + {i}) ** 0.5"], 8) + "    return s\n",
}


def probe_sources():
    return dict(PROBES)


if __name__ == "__main__":
    for k, v in PROBES.items():
        print(f"== {k}\n{v}")
