"""Per-policy-event PMC summary of a rocprofv3 counter-collection CSV from tools/pmc_driver.py.

    python tools/pmc_summary.py gpurun_out/r3h/pmc1/run_counter_collection.csv gpurun_out/r3h/pmc1.log [kernel-substring]

Sums every counter over the dispatches of the big launch (grid > 100k threads, the kernel-name
substring, default "replay_rows") and divides by the policy-events the driver reported (its JSON
line's "events").  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* are in quad-cycles (x4 = cycles).
"""
import collections
import csv
import json
import sys


def main() -> None:
    csv_path, log_path = sys.argv[1], sys.argv[2]
    sub = sys.argv[3] if len(sys.argv) > 3 else "replay_rows"
    events = None
    for line in open(log_path):
        line = line.strip()
        if line.startswith("{") and '"events"' in line:
            events = json.loads(line)["events"]
    agg = collections.defaultdict(float)
    kernel = ""
    for r in csv.DictReader(open(csv_path)):
        if sub in r["Kernel_Name"] and int(r["Grid_Size"]) > 100000:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            kernel = r["Kernel_Name"]
    print(f"# kernel {kernel[:100]}")
    print(f"# policy-events {events:.6g}")
    for k, v in sorted(agg.items()):
        print(f"{k:<24} {v:>16.4g}   per policy-event {v / events:>10.2f}")
    if "GRBM_GUI_ACTIVE" in agg and "SQ_INSTS_VALU" in agg:
        cyc = agg["GRBM_GUI_ACTIVE"] / 8
        print(f"# elapsed ~{cyc:.4g} cycles per XCD; VALU instructions per SIMD-cycle "
              f"{agg['SQ_INSTS_VALU'] / 1024 / cyc:.3f}")


if __name__ == "__main__":
    main()
