"""Bundled policy programs (program-text format).

* ``reference`` - the five policies of the reference's comparison harness
  (`tests/test_scheduler.py:20-218`): first-fit, best-fit and the three
  published FunSearch champions, with their exact reference scores;
* ``seeds`` - the seed programs of the reference search loop
  (`funsearch/funsearch_integration.py:217-431`).

Stored as JSON under ``data/policies`` (the same text a results JSON holds).
"""

from __future__ import annotations

import json
from functools import lru_cache
from typing import Dict

from .._paths import POLICIES_DIR


@lru_cache(maxsize=None)
def _load(name: str) -> Dict[str, dict]:
    with open(POLICIES_DIR / f"{name}.json") as fh:
        return {p["name"]: p for p in json.load(fh)["policies"]}


def reference_policies() -> Dict[str, str]:
    """name -> program text, in the reference's comparison order."""
    return {k: v["code"] for k, v in _load("reference_policies").items()}


def reference_scores() -> Dict[str, float]:
    return {k: v["score"] for k, v in _load("reference_policies").items()}


def seed_policies() -> Dict[str, str]:
    return {k: v["code"] for k, v in _load("seed_policies").items()}


def policy(name: str) -> str:
    for table in ("reference_policies", "seed_policies"):
        if name in _load(table):
            return _load(table)[name]["code"]
    raise KeyError(name)


def discovered_policies() -> Dict[str, dict]:
    """Policies found by this framework's searches, stored in the reference's
    results-JSON schema (`save_best_policy`: score, generation, code,
    timestamp; plus family / weights / results) under
    ``data/policies/discovered``.  file stem -> record."""
    out: Dict[str, dict] = {}
    d = POLICIES_DIR / "discovered"
    if d.is_dir():
        for f in sorted(d.glob("*.json")):
            with open(f) as fh:
                out[f.stem] = json.load(fh)
    return out
