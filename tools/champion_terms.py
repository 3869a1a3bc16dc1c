"""Which score terms of a champion program came from a family rendering?

    python tools/champion_terms.py POLICY.json|POLICY.py [...]

A policy body's *terms* are its top-level statements after `score = 0.0`
(each adds to, scales or sets `score`, possibly under a condition).  A term
counts as a family term when, with every numeric literal replaced by `C`, it
equals a statement of some family rendering (`models.families.to_program` of
`random_linear`, `feature_linear`, `composite_linear` -- what the family
coupler injects into the islands).  Prints per policy the number of terms,
how many match a family statement, and the fraction that does not.
"""
from __future__ import annotations

import ast
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

_NUM = re.compile(r"(?<![\w.])\d+(?:\.\d+)?(?:e[-+]?\d+)?(?![\w.])")


def _norm(stmt: str) -> str:
    return _NUM.sub("C", re.sub(r"\s+", " ", stmt.strip()))


def terms(code: str) -> list:
    fn = next(n for n in ast.parse(code).body if isinstance(n, ast.FunctionDef))
    lines = code.splitlines()
    out, started = [], False
    for st in fn.body:
        seg = "\n".join(lines[st.lineno - 1:st.end_lineno])
        if not started:
            if isinstance(st, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "score" for t in st.targets):
                started = True
            continue
        if isinstance(st, ast.Return):
            break
        out.append(seg)
    return out


def family_terms() -> set:
    import numpy as np
    from funsearch_kubernetes_simulator_amd.models.families import WEIGHTS, to_program
    from funsearch_kubernetes_simulator_amd.models.families import SAMPLERS
    out = set()
    rng = np.random.default_rng(0)
    for fam in ("random_linear", "feature_linear", "composite_linear"):
        # many weight vectors (signs, zeros): every statement form the renderer emits
        ws = list(SAMPLERS[fam](200, rng)) + [np.linspace(-1.5, 1.6, WEIGHTS), np.zeros(WEIGHTS)]
        ws += [np.where(rng.random(WEIGHTS) < 0.5, 0.0, rng.normal(size=WEIGHTS)) for _ in range(200)]
        for w in ws:
            code = to_program(fam, w)
            fn = next(n for n in ast.parse(code).body if isinstance(n, ast.FunctionDef))
            lines = code.splitlines()
            for st in fn.body:
                out.add(_norm("\n".join(lines[st.lineno - 1:st.end_lineno])))
    return out


def main() -> None:
    fam = family_terms()
    for path in sys.argv[1:]:
        text = open(path).read()
        code = json.loads(text).get("code", text) if path.endswith(".json") else text
        ts = terms(code)
        hit = sum(_norm(t) in fam for t in ts)
        print(json.dumps({"policy": os.path.basename(path), "terms": len(ts), "family_terms": hit,
                          "non_family_fraction": round(1 - hit / max(1, len(ts)), 4)}))


if __name__ == "__main__":
    main()
