"""Tabulate hipcc -Rpass-analysis=kernel-resource-usage remarks: VGPRs, scratch, occupancy, spills."""
import re
import sys

txt = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for b in re.split(r"remark: Function Name: ", txt)[1:]:
    name = b.split()[0]
    if pat not in name:
        continue

    def g(k):
        m = re.search(re.escape(k) + r": (\d+)", b)
        return m.group(1) if m else "?"
    print("%-64s V%4s scr%4s occ%3s vsp%4s ssp%4s" % (name[:64], g("VGPRs"), g("ScratchSize [bytes/lane]"),
                                                     g("Occupancy [waves/SIMD]"), g("VGPRs Spill"), g("SGPRs Spill")))
