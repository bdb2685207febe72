"""Print VGPR/SGPR/LDS/scratch of the kernels in a gfx950 assembly file
(`make -C pyactivestorage_amd/csrc asm` writes build/pyas/inst_f32.s)."""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "build/pyas/inst_f32.s"
pat = sys.argv[2] if len(sys.argv) > 2 else ""
s = open(path).read()
for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", s, re.S):
    name, body = m.group(1), m.group(2)
    if pat not in name:
        continue
    get = lambda k: re.search(r"\.amdhsa_%s (\d+)" % k, body).group(1)
    print(f"{name[:70]:70s} vgpr {get('next_free_vgpr'):>4} sgpr {get('next_free_sgpr'):>4} "
          f"lds {get('group_segment_fixed_size'):>6} scratch {get('private_segment_fixed_size')}")
