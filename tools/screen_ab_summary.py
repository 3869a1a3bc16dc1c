#!/usr/bin/env python3
"""Summary of tools/screen_ab.sh: median best score per arm, per-seed wins,
surrogate/exact Spearman rank correlations."""
import json
import sys

import numpy as np


def main() -> None:
    rows = [json.loads(l) for l in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/screen_ab/ab.jsonl")]
    arms = {}
    for r in rows:
        arms.setdefault(r["k"], {})[r["seed"]] = r
    seeds = sorted(set(arms.get(1, {})) & set(arms.get(4, {})))
    base = [arms[1][s]["best_score"] for s in seeds]
    scr = [arms[4][s]["best_score"] for s in seeds]
    rho = [x for s in seeds for x in (arms[4][s]["screen"] or {}).get("spearman", [])]
    out = {"seeds": seeds, "exact_only_best": base, "screened_best": scr,
           "median_exact_only": float(np.median(base)) if base else None,
           "median_screened": float(np.median(scr)) if scr else None,
           "screened_wins": int(sum(b < a for a, b in zip(scr, base))),
           "spearman_median": float(np.median(rho)) if rho else None,
           "spearman_range": [float(min(rho)), float(max(rho))] if rho else None,
           "exact_evals_per_s": {k: float(np.median([arms[k][s]["value"] for s in seeds])) for k in (1, 4)}}
    out["verdict"] = ("screen wins on the median" if out["median_screened"] is not None
                      and out["median_screened"] > out["median_exact_only"] else "exact-only wins on the median")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
