#!/usr/bin/env python3
"""Per-kernel VGPR / spill / scratch summary of an amdgcn .s (save-temps) file."""
import re
import sys

txt = open(sys.argv[1]).read()
for m in re.finditer(r"\.name:\s+(\S+)\n(?:.*\n)*?.*?\.vgpr_count:\s+(\d+)\n\s+\.vgpr_spill_count:\s+(\d+)", txt):
    pass
for blk in txt.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    v = re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1)
    sp = re.search(r"\.vgpr_spill_count:\s+(\d+)", blk).group(1)
    pr = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk).group(1)
    print(f"{name[:60]:60s} vgpr {v:>4} spill {sp:>3} scratch {pr:>3}")
