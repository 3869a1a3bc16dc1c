"""Per-kernel time summary of a rocprofv3 rocpd database (`--kernel-trace`,
the SQLite output rocprofv3 7.x writes by default; tools/gpu_check.sh `prof`):
dispatches, total / mean / max duration and share of the summed kernel time,
plus each kernel's launch shape and register counts.

    python tools/kernel_stats_db.py gpurun_out/NAME/prof/run_results.db [--top 15]
"""
import argparse
import sqlite3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), max(duration), max(grid_x), max(workgroup_x), "
        "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(lds_size), max(scratch_size) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print(f"# {a.db}: {sum(r[1] for r in rows)} dispatches, {total / 1e6:.3f} ms of kernel time")
    print(f"{'share':>6} {'calls':>6} {'total_ms':>10} {'mean_us':>10} {'max_us':>10}  grid  wg  vgpr agpr sgpr  lds  scratch  kernel")
    for name, n, tot, avg, mx, gx, wx, vg, ag, sg, lds, scr in rows[:a.top]:
        short = name if len(name) < 90 else name[:87] + "..."
        print(f"{100 * tot / total:5.1f}% {n:6d} {tot / 1e6:10.3f} {avg / 1e3:10.1f} {mx / 1e3:10.1f}  {gx} {wx} "
              f"{vg} {ag} {sg} {lds} {scr}  {short}")


if __name__ == "__main__":
    main()
