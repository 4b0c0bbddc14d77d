"""Per-kernel SQ counter summary from a rocprofv3 --pmc CSV directory (latency vs issue bound).

usage: python tools/sq_counters.py <pmc_dir>
"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
  for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "mjw" not in k:
      continue
    k = k.split("(")[0].replace("void ", "")
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[k][r["Counter_Name"]] += 1
for k, c in acc.items():
  n = max(cnt[k].values())
  avg = {name: v / cnt[k][name] for name, v in c.items()}
  print(k, f"({n} dispatches)")
  for name in sorted(avg):
    print(f"   {name:24s} {avg[name]:16.0f}")
  wc = avg.get("SQ_WAVE_CYCLES")
  if wc:
    for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
      if name in avg:
        print(f"   {name} / WAVE_CYCLES = {avg[name] / wc:.3f}")
  if "SQ_WAVES" in avg and "SQ_INSTS_VALU" in avg:
    print(f"   VALU insts per wave = {avg['SQ_INSTS_VALU'] / avg['SQ_WAVES']:.0f}, "
          f"LDS {avg.get('SQ_INSTS_LDS', 0) / avg['SQ_WAVES']:.0f}, SALU {avg.get('SQ_INSTS_SALU', 0) / avg['SQ_WAVES']:.0f}")
