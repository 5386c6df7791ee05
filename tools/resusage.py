"""Per-kernel register / LDS / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (stdin)."""
import re
import subprocess
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        cur = {"name": name}
        rows.append(cur)
        continue
    m = re.search(r"(VGPRs|AGPRs|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split(" [")[0]] = int(m.group(2))
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if pat in r["name"]:
        print(f"{r.get('VGPRs',0):4d}v {r.get('VGPRs Spill',0):3d}vs {r.get('SGPRs Spill',0):3d}ss "
              f"{r.get('LDS Size',0):7d}B occ{r.get('Occupancy',0)}  {r['name'][:110]}")
