"""Per-kernel scan of a device assembly listing (hipcc --cuda-device-only -S):
MFMA count, scratch (spill) instructions and how many of them sit between
the first and the last MFMA (inside the K loop), global loads, s_barriers.

    python tools/isa_scan.py /tmp/c3.s [name-substring]
"""
import re
import subprocess
import sys

src = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\w+):\s*(?:;.*)?$", src, re.M)]
for i, (pos, name) in enumerate(starts):
    end = starts[i + 1][0] if i + 1 < len(starts) else len(src)
    body = src[pos:end].split("\n")
    try:
        dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    except OSError:
        dn = name
    if pat not in dn:
        continue
    mf = [j for j, l in enumerate(body) if "v_mfma" in l]
    sc = [j for j, l in enumerate(body) if "scratch_" in l]
    inl = [j for j in sc if mf and mf[0] < j < mf[-1]]
    gl = sum(1 for l in body if "global_load_dwordx4" in l)
    bar = sum(1 for l in body if "s_barrier" in l)
    print(f"mfma {len(mf):5d} scratch {len(sc):3d} in-loop {len(inl):3d} gload4 {gl:4d} "
          f"barrier {bar:3d}  {dn[:120]}")
