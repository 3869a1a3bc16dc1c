"""Filesystem locations of bundled data, built native artefacts and outputs."""

from __future__ import annotations

import os
from pathlib import Path

PACKAGE_DIR = Path(__file__).resolve().parent
REPO_DIR = PACKAGE_DIR.parent

#: Bundled OpenB trace assets (copied from the reference's benchmarks/traces).
DATA_DIR = Path(os.environ.get("FKS_DATA_DIR", REPO_DIR / "data"))
TRACES_DIR = DATA_DIR / "traces"
POLICIES_DIR = DATA_DIR / "policies"

#: In-tree native extension output directory (built by ops/build.py).
NATIVE_DIR = PACKAGE_DIR / "ops"
CSRC_DIR = REPO_DIR / "csrc"

DEFAULT_NODE_FILE = "gpu_models_filtered.csv"
DEFAULT_POD_FILE = "openb_pod_list_default.csv"


def resolve_traces_dir(traces_dir: "str | os.PathLike | None") -> Path:
    """Resolve a traces directory.

    The reference resolves ``"benchmarks/traces"`` against the current working
    directory (`benchmarks/parser.py:12`), which breaks as soon as a script is
    started elsewhere.  Here an explicit directory that exists wins; the
    reference's default spelling, or ``None``, maps to the bundled copy.
    """
    if traces_dir is None:
        return TRACES_DIR
    p = Path(traces_dir)
    if p.is_dir():
        return p
    if str(traces_dir).rstrip("/") in ("benchmarks/traces", "traces"):
        return TRACES_DIR
    return p
