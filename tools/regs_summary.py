"""Summarise `-Rpass-analysis=kernel-resource-usage` remarks (stdin): one line per kernel."""
import re
import sys

cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        print()
        print(cur[-50:], end=" ")
        continue
    m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]): (\d+)",
                  line)
    if m and cur:
        name = m.group(1).split()[0] + ("_spill" if "Spill" in m.group(1) else "")
        print(f"{name}={m.group(2)}", end=" ")
    if "error" in line:
        print(line, end="")
print()
