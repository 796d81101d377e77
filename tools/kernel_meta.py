"""Print VGPR / spill / LDS metadata of the kernels in a hipcc -S assembly file.

    python tools/kernel_meta.py file.s [name-substring]
"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.findall(r"(- \.agpr_count.*?\.wavefront_size)", s, re.S):
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if pat not in name:
        continue
    get = lambda k: (re.search(r"\.%s:\s+(\d+)" % k, blk) or [None, "?"])[1]
    print(f"{name[:70]:70s} vgpr {get('vgpr_count'):>4} agpr {get('agpr_count'):>3} "
          f"spill {get('vgpr_spill_count'):>3} lds {get('group_segment_fixed_size')}")
