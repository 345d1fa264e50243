"""Print VGPR/SGPR/LDS/scratch per kernel from a hipcc --cuda-device-only -S listing."""
import re
import sys

text = open(sys.argv[1]).read()
meta = text[text.find("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    def f(k):
        m = re.search(r"\." + k + r":\s+(\S+)", blk)
        return m.group(1) if m else "?"
    print(f"{f('name')[:60]:60s} vgpr {f('vgpr_count'):>4s} sgpr {f('sgpr_count'):>4s} "
          f"lds {f('group_segment_fixed_size'):>6s} scratch {f('private_segment_fixed_size'):>4s}")
