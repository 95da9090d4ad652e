"""Print VGPR/AGPR/spill/LDS metadata per kernel from a hipcc --save-temps .s file."""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
meta = s[s.find("amdhsa.kernels:"):]
for blk in meta.split("\n  - ")[1:]:
    def g(k):
        m = re.search(r"\." + k + r":\s+(\S+)", blk)
        return m.group(1) if m else "?"
    name = g("name")
    if pat in name:
        print(f"vgpr={g('vgpr_count'):>4} agpr={g('agpr_count'):>4} vspill={g('vgpr_spill_count'):>3} "
              f"lds={g('group_segment_fixed_size'):>6} {name[:110]}")
