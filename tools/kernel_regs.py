#!/usr/bin/env python3
"""Register / LDS / scratch summary of the kernels in a hipcc -save-temps device assembly file
(the amdhsa.kernels metadata): python tools/kernel_regs.py file.s [name-substring]"""
import re
import sys


def main():
    text = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    meta = text[text.index("amdhsa.kernels:"):]
    for block in re.split(r"\n  - ", meta)[1:]:
        name = re.search(r"\.name:\s+(\S+)", block)
        if not name or sub not in name.group(1):
            continue
        f = {k: re.search(rf"\.{k}:\s+(\d+)", block) for k in
             ("vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size", "private_segment_fixed_size",
              "vgpr_spill_count")}
        vals = {k: int(v.group(1)) if v else None for k, v in f.items()}
        print(f"{name.group(1)[:70]:70s} vgpr {vals['vgpr_count']} agpr {vals['agpr_count']} "
              f"spill {vals['vgpr_spill_count']} lds {vals['group_segment_fixed_size']} "
              f"scratch {vals['private_segment_fixed_size']}")


if __name__ == "__main__":
    main()
