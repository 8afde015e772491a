#!/usr/bin/env python3
"""Instruction mix of the hottest loop (the backward-branch region with the most f64 ops) of
each blind-rotation kernel in a --save-temps gfx950 .s file (no GPU needed).
Usage: tools/loop_mix.py FILE.s [name-substring ...]"""
import collections
import re
import sys

txt = open(sys.argv[1]).read()
pats = sys.argv[2:] or ["blind_rotate"]
for m in re.finditer(r"^(_Z\S*):\s*;", txt, re.M):
    nm = m.group(1)
    if not any(p in nm for p in pats):
        continue
    end = txt.index(".Lfunc_end", m.end())
    lines = [l.strip() for l in txt[m.end():end].split("\n")]
    labels = {l.split(":")[0]: i for i, l in enumerate(lines) if re.match(r"^\.LBB\d+_\d+:", l)}
    best = None
    for i, l in enumerate(lines):
        b = re.match(r"s_(?:cbranch_\w+|branch) (\.LBB\d+_\d+)", l)
        if b and b.group(1) in labels and labels[b.group(1)] < i:
            n = sum("_f64" in x for x in lines[labels[b.group(1)]:i])
            if not best or n > best[0]:
                best = (n, labels[b.group(1)], i)
    if not best:
        continue
    c = collections.Counter()
    for l in lines[best[1]:best[2]]:
        if not l or l.startswith((".", ";")):
            continue
        op = l.split()[0]
        if op.startswith("v_"):
            c["VALU"] += 1
            if "_f64" in op:
                c["f64"] += 1
            elif "permlane" in op:
                c["permlane"] += 1
            elif "dpp" in l:
                c["dpp"] += 1
            elif op.startswith("v_mov") or op.startswith("v_accvgpr"):
                c["mov"] += 1
            elif op.startswith("v_cndmask"):
                c["cndmask"] += 1
            else:
                c["int/other"] += 1
        elif op.startswith("ds_"):
            c["ds"] += 1
        elif op.startswith(("global_", "buffer_")):
            c["vmem"] += 1
        elif op.startswith("scratch_"):
            c["scratch"] += 1
        elif op.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        elif op.startswith("s_barrier"):
            c["barrier"] += 1
        elif op.startswith("s_nop"):
            c["nop"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    print(nm[:60], dict(c))
