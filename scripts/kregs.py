"""Register / spill / LDS table of the kernels in a hipcc -save-temps .s file
(the amdhsa metadata block): python scripts/kregs.py file.s [name-filter]."""
import re
import sys

txt = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
meta = txt[txt.find("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    f = dict(re.findall(r"\.(\w+):\s+([^\n]+)", blk))
    name = f.get("name", "?")
    if flt not in name:
        continue
    print(f"{name[:70]:70s} vgpr {f.get('vgpr_count', '?'):>4} agpr {f.get('agpr_count', '?'):>4} "
          f"spill {f.get('vgpr_spill_count', '?'):>4} lds {f.get('group_segment_fixed_size', '?'):>6}")
