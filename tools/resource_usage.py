"""Per-kernel registers / scratch / occupancy / LDS from a `hipcc -Rpass-analysis=kernel-resource-usage`
log: python tools/resource_usage.py <log> [name-filter ...]"""
import re
import sys

txt = open(sys.argv[1]).read()
flt = sys.argv[2:]
for b in re.split(r"remark: Function Name: ", txt)[1:]:
    name = b.split("\n")[0]
    if flt and not any(f in name for f in flt):
        continue

    def g(key):
        m = re.search(re.escape(key) + r": (\S+)", b)
        return m.group(1) if m else "?"
    print(f"{name[:64]:64s} VGPR={g('VGPRs'):>4s} SGPR={g('SGPRs'):>4s} scratch={g('ScratchSize [bytes/lane]'):>4s} "
          f"occ={g('Occupancy [waves/SIMD]'):>2s} LDS={g('LDS Size [bytes/block]')}")
