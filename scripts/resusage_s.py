"""VGPR / SGPR / LDS / scratch per kernel from a device .s file (diagnostic)."""
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", s, re.S):
    name, body = m.group(1), m.group(2)
    if len(sys.argv) > 2 and not re.search(sys.argv[2], name):
        continue
    g = lambda k: (re.search(r"\.amdhsa_" + k + r"\s+(\d+)", body) or [None, "?"])[1]
    short = re.sub(r"_ZN2rm12_GLOBAL__N_1\d+", "", name)[:48]
    print("%-48s vgpr=%-4s agpr_off=%-4s sgpr=%-4s lds=%-6s scratch=%s" % (
        short, g("next_free_vgpr"), g("accum_offset"), g("next_free_sgpr"), g("group_segment_fixed_size"),
        g("private_segment_fixed_size")))
