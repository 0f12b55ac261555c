"""Static instruction mix of kernels in a device assembly file (hipcc --cuda-device-only -S).

usage: python tools/asmstat.py file.s SUBSTRING [SUBSTRING...]
Prints, per matching kernel: instruction count, top opcodes, VGPR/AGPR/SGPR use, LDS and scratch."""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
keys = sys.argv[2:]
for m in re.finditer(r"^(_Z\w+):", s, re.M):
    name = m.group(1)
    if not any(k in name for k in keys):
        continue
    end = s.find(".Lfunc_end", m.end())
    body = s[m.end():end]
    ins = []
    for line in body.split("\n"):
        t = line.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        ins.append(t.split()[0])
    c = Counter(ins)
    meta_i = s.find(".amdhsa_kernel " + name)
    meta = s[meta_i:s.find(".end_amdhsa_kernel", meta_i)]

    def g(k):
        mm = re.search(re.escape(k) + r"\s+(\d+)", meta)
        return mm.group(1) if mm else "?"

    print(f"{name[:90]}\n  instrs {len(ins)}  vgpr {g('.amdhsa_next_free_vgpr')}  accum_offset "
          f"{g('.amdhsa_accum_offset')}  sgpr {g('.amdhsa_next_free_sgpr')}  lds {g('.amdhsa_group_segment_fixed_size')}"
          f"  scratch {g('.amdhsa_private_segment_fixed_size')}")
    groups = Counter()
    for op, n in c.items():
        k = ("mfma" if "mfma" in op else "global_load" if op.startswith(("global_load", "buffer_load")) else
             "global_store" if op.startswith(("global_store", "buffer_store")) else
             "atomic" if "atomic" in op else "ds_read" if op.startswith("ds_read") else
             "ds_write" if op.startswith("ds_write") else "s_waitcnt" if op == "s_waitcnt" else
             "salu" if op.startswith("s_") else "valu" if op.startswith("v_") else "other")
        groups[k] += n
    print("  classes", dict(groups.most_common()))
    print("  top", c.most_common(18))
