"""Dynamic instruction mix of baseline-JIT code (ops/gcnjit.py) over full
replays on the wave64 emulator: executed wave instructions per opcode, per
replayed event, for a program set (the reference seeds, offline-mutation
children, or children of an evolved population).  Shows where the scoring
wave's call time goes without a GPU.

    python tools/jit_profile.py --set children --programs 24
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="children", choices=["children", "reference", "population", "probes"])
    ap.add_argument("--programs", type=int, default=24)
    ap.add_argument("--ck", default="data/populations/config3_steady_r4_islands.json")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--no-elide", action="store_true", help="keep the feasibility prologue (call every node)")
    a = ap.parse_args()
    from funsearch_kubernetes_simulator_amd.ops import gcnjit
    from funsearch_kubernetes_simulator_amd.policy.compiler import compile_policy
    if a.set == "children":
        from funsearch_kubernetes_simulator_amd.bench.programs import mutation_children
        progs = mutation_children(a.programs, 0)
    elif a.set == "reference":
        from funsearch_kubernetes_simulator_amd.models.library import reference_policies
        progs = [compile_policy(s) for s in reference_policies().values()]
    elif a.set == "probes":
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from call_probes import probe_sources
        for name, src in probe_sources().items():
            p = compile_policy(src)
            if gcnjit.compile_program(p)[0] is None:
                print(json.dumps({"probe": name, "declined": True}))
                continue
            _profile(name, [p], a)
        return
    else:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from population_bench import _programs
        progs = _programs(a.ck, a.programs, 7)
    progs = [p for p in progs if gcnjit.compile_program(p)[0] is not None]
    _profile(a.set, progs, a)


def _profile(name, progs, a) -> None:
    from funsearch_kubernetes_simulator_amd.core import load_default_workload
    from funsearch_kubernetes_simulator_amd.ops import cpu_engine as ce
    from funsearch_kubernetes_simulator_amd.ops import gcnjit
    w = load_default_workload()
    budget = 1 << 16
    ce.native().gcn_emu_profile(True)
    tab = gcnjit.emulate_programs(w, progs, budget, ce.SimOptions(budget=budget), elide=not a.no_elide)
    counts = ce.native().gcn_emu_profile_counts()
    ce.native().gcn_emu_profile(False)
    from funsearch_kubernetes_simulator_amd.policy.bytecode import Op
    events = float(tab[:, 8].sum())
    by_bc = {}
    for k, v in list(counts.items()):
        if k.startswith("bc:"):
            code = int(k[3:])
            by_bc[Op(code).name if code in Op._value2member_map_ else "prologue/epilogue"] = v
            del counts[k]
    total = sum(v for k, v in counts.items() if k != "LABEL")
    rows = sorted(((k, v) for k, v in counts.items() if k != "LABEL"), key=lambda kv: -kv[1])
    print(json.dumps({"set": name, "programs": len(progs), "events": int(events),
                      "insns_per_event": round(total / events, 1)}), flush=True)
    if a.top <= 0:
        return
    for k, v in rows[:a.top]:
        print(f"{k:28s} {v / events:9.2f} per event  {100.0 * v / total:5.1f}%")
    print("-- by the bytecode op they lower (labels included)")
    tb = sum(by_bc.values())
    for k, v in sorted(by_bc.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"{k:28s} {v / events:9.2f} per event  {100.0 * v / tb:5.1f}%")

if __name__ == "__main__":
    main()
