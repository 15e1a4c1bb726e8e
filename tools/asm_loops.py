#!/usr/bin/env python3
"""Loops of one kernel in a `make asm` listing: for every backward branch, the loop's line span, its
instruction count and its scratch (spill) loads/stores -- to see whether spills sit on a hot loop.
Measurement tooling only. Usage: python tools/asm_loops.py LISTING.s SYMBOL [min_instrs]"""
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 40
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
labels = {}
for i in range(start, end):
    m = re.match(r"^(\.LBB\d+_\d+):", lines[i])
    if m:
        labels[m.group(1)] = i
tot = sum(1 for i in range(start, end) if "scratch_" in lines[i])
print(f"{sym}: lines {start}-{end}, scratch ops {tot}")
for i in range(start, end):
    m = re.match(r"^\s*s_cbranch_\w+\s+(\.LBB\d+_\d+)|^\s*s_branch\s+(\.LBB\d+_\d+)", lines[i])
    if not m:
        continue
    lab = m.group(1) or m.group(2)
    j = labels.get(lab)
    if j is None or j > i:
        continue
    body = [l for l in lines[j:i + 1] if l.strip() and not l.strip().startswith(";") and not l.startswith(".")]
    if len(body) < mn:
        continue
    sc = sum(1 for l in body if "scratch_" in l)
    rl = sum(1 for l in body if "v_readlane" in l or "v_writelane" in l)
    print(f"loop {lab} lines {j}-{i}: {len(body)} instrs, scratch {sc}, readlane/writelane {rl}")
