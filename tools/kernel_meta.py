"""Reads `llvm-readelf --notes` of a gfx950 code object on stdin, prints one line per kernel
(tools/kernel_meta.sh)."""
import re
import sys

txt = sys.stdin.read()
for blk in txt.split("  - .agpr_count:")[1:]:
    blk = ".agpr_count:" + blk

    def g(k):
        m = re.search(r"\." + k + r":\s+(\S+)", blk)
        return m.group(1) if m else "?"

    print(f"{g('name'):34s} vgpr={g('vgpr_count'):>4s} agpr={g('agpr_count'):>4s} sgpr={g('sgpr_count'):>4s} "
          f"scratch={g('private_segment_fixed_size'):>6s} vspill={g('vgpr_spill_count'):>5s} "
          f"sspill={g('sgpr_spill_count'):>4s} dynstack={g('uses_dynamic_stack')}")
