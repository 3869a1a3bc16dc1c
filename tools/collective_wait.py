#!/usr/bin/env python3
"""Per-rank collective wait of a multi-rank island run, from its JSONL logs.

    python tools/collective_wait.py runs/c4r/metrics.rank*.jsonl

Reads each rank's last ``generation`` (pipelined / lock-step) or
``steady_final`` / ``steady_status`` record and prints the wall time the rank
spent blocked in collectives (`funsearch/migration.py` ``wait_s``) as a
fraction of its run time; exits 1 if any rank is at or above ``--limit``.
"""
import argparse
import json
import sys


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("logs", nargs="+")
    ap.add_argument("--limit", type=float, default=0.05)
    a = ap.parse_args()
    rows = []
    for path in a.logs:
        last = None
        migrations = 0
        for line in open(path):
            r = json.loads(line)
            if r.get("kind") in ("migration", "steady_migration"):
                migrations += 1
            if "collective_wait_s" in r and r.get("kind") in ("generation", "steady_status", "steady_final"):
                last = r
        if last is None:
            continue
        frac = last.get("collective_wait_frac")
        rows.append({"log": path, "rank": last.get("rank"), "generation": last.get("generation"),
                     "migrations": migrations, "collective_wait_s": last["collective_wait_s"],
                     "collective_wait_frac": frac})
    worst = max((r["collective_wait_frac"] or 0.0) for r in rows) if rows else None
    print(json.dumps({"ranks": len(rows), "max_collective_wait_frac": worst, "limit": a.limit, "per_rank": rows}))
    sys.exit(0 if rows and worst < a.limit else 1)


if __name__ == "__main__":
    main()
