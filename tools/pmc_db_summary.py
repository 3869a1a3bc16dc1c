"""Per-policy-event PMC summary of a rocprofv3 rocpd database (`--pmc` pass of
bench.py, tools/gpu_check.sh `pmc=`): sums every counter over the row-kernel
dispatches and divides by the replayed policy-events of those launches (the
bench JSON line's events_per_s x the dispatches' summed wall / the launches'
concurrency is not needed: events come from the bench's own table sums).

    python tools/pmc_db_summary.py DB [DB ...] --events-per-dispatch N [--kernel replay_rows]

VALU issue model (CDNA4): a wave64 VALU op occupies its SIMD (16 lanes) for 4
cycles, so a CU's 4 SIMDs issue at most 1 VALU wave-instruction per cycle;
SQ_ACTIVE_INST_VALU counts quad-cycles a wave spends on VALU instructions."""
import argparse
import collections
import sqlite3


def load(db, kernel):
    c = sqlite3.connect(db)
    agg = collections.defaultdict(float)
    disp = set()
    dur = {}
    for name, did, ctr, val, s, e in c.execute(
            "select kernel_name, dispatch_id, counter_name, value, start, end from counters_collection"):
        if kernel in name:
            agg[ctr] += float(val)
            disp.add(did)
            dur[did] = e - s
    return agg, len(disp), sum(dur.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--kernel", default="replay_rows")
    ap.add_argument("--events", type=float, required=True, help="policy-events replayed by the matched dispatches")
    ap.add_argument("--cus", type=int, default=256)
    a = ap.parse_args()
    tot = {}
    nd = 0
    for db in a.dbs:
        agg, n, _ = load(db, a.kernel)
        nd = max(nd, n)
        tot.update(agg)
    ev = a.events
    print(f"# {nd} dispatches of *{a.kernel}*, {ev:.4g} policy-events")
    for k in sorted(tot):
        print(f"{k:<28} {tot[k]:>14.4g}   per policy-event {tot[k] / ev:>10.2f}")
    if "SQ_ACTIVE_INST_VALU" in tot and "GRBM_GUI_ACTIVE" in tot:
        gui = tot["GRBM_GUI_ACTIVE"]
        print(f"# VALU busy (rocprof's VALUBusy: 100*ACTIVE_INST_VALU/CUs/GRBM_GUI_ACTIVE, x4 quad-cycles / 4 SIMDs)"
              f" = {100 * tot['SQ_ACTIVE_INST_VALU'] * 4 / 4 / a.cus / gui:.1f} %")
    if "SQ_THREAD_CYCLES_VALU" in tot and "SQ_ACTIVE_INST_VALU" in tot:
        print(f"# VALU lane utilisation (THREAD_CYCLES_VALU / (ACTIVE_INST_VALU*4*64)... rocprof VALUUtil ="
              f" THREAD_CYCLES/(ACTIVE_INST_VALU*64)) = {100 * tot['SQ_THREAD_CYCLES_VALU'] / (tot['SQ_ACTIVE_INST_VALU'] * 64):.1f} %")
    if "SQ_INSTS_VALU" in tot and "GRBM_GUI_ACTIVE" in tot:
        print(f"# VALU wave-instructions per CU-cycle = {tot['SQ_INSTS_VALU'] / a.cus / tot['GRBM_GUI_ACTIVE']:.3f}"
              f" (issue ceiling 1.0: 4 SIMDs x 1 wave64 op / 4 cycles)")


if __name__ == "__main__":
    main()
