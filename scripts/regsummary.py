"""Per-kernel VGPR/AGPR/SGPR spill summary from hipcc -Rpass-analysis=kernel-resource-usage output."""
import re
import subprocess
import sys

rows, cur = {}, None
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    dn = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip().replace("(anonymous namespace)::", "").split("(")[0]
    print(f"{dn:58s} VGPR {v.get('VGPRs')} AGPR {v.get('AGPRs')} SGPR {v.get('TotalSGPRs')} sgpr_spill {v.get('SGPRs Spill')} "
          f"vgpr_spill {v.get('VGPRs Spill')} scratch {v.get('ScratchSize [bytes/lane]')} occ {v.get('Occupancy [waves/SIMD]')}")
