"""Per-kernel register / scratch / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (stdin)."""
import re
import subprocess
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("sgpr", r"TotalSGPRs: (\d+)"),
                     ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                     ("sspill", r"SGPRs Spill: (\d+)"), ("vspill", r"VGPRs Spill: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
names = [r["name"] for r in rows]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
for r, d in zip(rows, dem):
    d = re.sub(r"\(.*", "", d)
    print(f"{d[:70]:70s} vgpr={r.get('vgpr')} sgpr={r.get('sgpr')} scratch={r.get('scratch')} "
          f"occ={r.get('occ')} sspill={r.get('sspill')} vspill={r.get('vspill')}")
