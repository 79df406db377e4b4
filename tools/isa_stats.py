#!/usr/bin/env python3
"""Instruction mix of one kernel in a device assembly listing (hipcc
--cuda-device-only -S): counts by class, static (not executed) counts.

    python tools/isa_stats.py engine.s <mangled-name-substring>
"""
import collections
import re
import sys

path, sub = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(sub) + r"\S*:\s*(;.*)?$", l))
name = lines[start].split(":")[0]
cnt = collections.Counter()
ops = collections.Counter()
for l in lines[start + 1:]:
    if l.startswith(".Lfunc_end") or re.match(r"^_Z\S+:", l):
        break
    t = l.strip()
    if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
        continue
    op = t.split()[0]
    ops[op] += 1
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        cnt["vmem_load"] += 1
    elif op.startswith(("global_store", "buffer_store", "flat_store")):
        cnt["vmem_store"] += 1
    elif op.startswith("s_load") or op.startswith("s_buffer_load"):
        cnt["smem_load"] += 1
    elif op.startswith("s_waitcnt"):
        cnt["waitcnt"] += 1
    elif op.startswith("v_"):
        cnt["valu"] += 1
        if "f64" in op:
            cnt["valu_f64"] += 1
    elif op.startswith("s_"):
        cnt["salu"] += 1
    elif op.startswith("ds_"):
        cnt["lds"] += 1
    else:
        cnt["other"] += 1
print(name)
print(dict(cnt))
print(ops.most_common(40))
