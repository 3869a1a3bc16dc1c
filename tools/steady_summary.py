"""Compact timeline of a steady-state run's status records.

    python tools/steady_summary.py STEADY_LOG_OR_METRICS_JSONL [--final-only]

One line per `steady_status` (and the `steady_final`): wall time, evaluations,
evals/s, programs in flight (time-weighted mean), queued children, producer
tasks and CPU ms per child, host fallbacks / shed children, polish batches,
best score, distinct island bests, generation, main-thread phase seconds,
module-load seconds and the device-busy fraction; then the final record in
full.  Used for the profiles/r4_config3_steady_*.txt summaries.
"""

from __future__ import annotations

import json
import sys


def main() -> None:
    path = sys.argv[1]
    final_only = "--final-only" in sys.argv
    last = None
    for line in open(path):
        line = line.strip()
        if not line.startswith("{"):
            continue
        try:
            r = json.loads(line)
        except ValueError:
            continue
        if r.get("kind") not in ("steady_status", "steady_final"):
            continue
        last = r
        if final_only and r["kind"] != "steady_final":
            continue
        ph = {k: round(v, 1) for k, v in r.get("main_phase_s", {}).items()}
        print(f"{r['wall_s']:8.1f}s evals {r['evaluations']:7d} {r['evals_per_s']:8.1f}/s "
              f"all {r.get('all_evals_per_s', 0):8.1f}/s occ~{r.get('occupancy_mean') or 0:.3f} "
              f"inflight~{r.get('inflight_mean', 0):6.0f} queued {r.get('queued', 0):4d} "
              f"Mcyc/child {r.get('mcycles_per_child', 0):6.1f} cost_rej {r.get('cost_rejected', 0)} "
              f"tasks {r.get('producer_tasks', 0):2d} ms/child {r.get('producer_ms_per_child', 0):5.2f} "
              f"fallback {r.get('host_fallback', 0)} shed {r.get('shed', 0)} "
              f"polish {r.get('polish_batches', 0)}/{r.get('polish_improved', 0)} "
              f"best {r['best']:.6f} distinct {r.get('distinct_island_bests', 0)} gen {r['generation']} "
              f"phases {ph} load_s {r.get('jit', {}).get('load_s')} busy {r.get('device_busy')}")
    if last is not None:
        print(json.dumps(last))
    # children merged per 100 s window (from the status records' evaluations)
    st = []
    for line in open(path):
        if '"steady_status"' in line or '"steady_final"' in line:
            try:
                r = json.loads(line.strip())
            except ValueError:
                continue
            if r.get("kind") in ("steady_status", "steady_final"):
                # (the drain after the wall limit -- no producer task, nothing
                # queued, the last replays finishing -- is not part of a window)
                if st and r.get("producer_tasks", 1) == 0 and r.get("queued", 1) == 0:
                    continue
                st.append((r["wall_s"], r["evaluations"], r.get("evaluations", 0) + r.get("polish_evals", 0)))
    if st:
        print("# 100 s windows: children / s, all program evals / s (children + polish variants)")
        w0, e0, a0 = 0.0, 0, 0
        for k, (t, e, a) in enumerate(st):
            last_rec = k == len(st) - 1
            if t - w0 >= 99.5 or (last_rec and t - w0 >= 30):
                print(f"  [{w0:6.0f}, {t:6.0f}) s: {(e - e0) / (t - w0):8.1f} children/s {(a - a0) / (t - w0):8.1f} all/s")
                w0, e0, a0 = t, e, a
    # steady_batch records by quintile of the run: device seconds per batch
    # (child batches only), the ready queue, and the replayed events per program
    bs = []
    for line in open(path):
        if '"steady_batch"' not in line:
            continue
        try:
            r = json.loads(line.strip())
        except ValueError:
            continue
        bs.append(r)
    if bs:
        q = max(1, len(bs) // 5)
        print("# steady_batch quintiles: batches, device_s mean, queued mean, events mean / max per program,"
              " device Mcycles per replay (mean of batch means / mean of batch maxima)")
        for i in range(5):
            part = bs[i * q:(i + 1) * q] if i < 4 else bs[4 * q:]
            if not part:
                continue
            dm = sum(r["device_s"] for r in part) / len(part)
            qm = sum(r.get("queued", 0) for r in part) / len(part)
            em = sum(r.get("events_mean", 0) for r in part) / len(part)
            ex = max(r.get("events_max", 0) for r in part)
            cm = sum(r.get("mcycles_mean", 0) for r in part) / len(part)
            cx = sum(r.get("mcycles_max", 0) for r in part) / len(part)
            print(f"Q{i + 1}: {len(part):4d} batches  device_s {dm:7.3f}  queued {qm:6.1f}  events mean {em:9.0f} max {ex}"
                  f"  Mcycles {cm:7.1f} / {cx:7.1f}")


if __name__ == "__main__":
    main()
