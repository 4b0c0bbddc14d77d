"""Report scratch (spill) instructions and loop back-edges per kernel in a hipcc -S listing.

usage: python tools/asm_spills.py file.s [kernel-substring ...]
"""
import re
import sys

s = open(sys.argv[1]).read()
pats = sys.argv[2:] or [""]
for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
  name = m.group(1)
  if not any(p in name for p in pats):
    continue
  j = s.index(".Lfunc_end", m.end())
  body = s[m.start():j].split("\n")
  labels = {l.split(":")[0]: k for k, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
  spills = [k for k, l in enumerate(body) if "scratch_" in l]
  loops = []
  for k, l in enumerate(body):
    b = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
    if b and labels.get(b.group(1), 1 << 30) < k:
      loops.append((labels[b.group(1)], k))
  inloop = [k for k in spills if any(a <= k <= b for a, b in loops)]
  print(f"{name}: {len(body)} lines, {len(spills)} scratch ops, {len(inloop)} inside loops")
  for a, b in loops:
    n = sum(1 for k in spills if a <= k <= b)
    print(f"   loop {a}-{b} ({b - a} lines): {n} scratch ops")
