"""Per-kernel rocprofv3 durations over the bench's timed window (not the whole run).

usage: python tools/kernel_window.py <stats_dir> <warmup> <steps> [out.json]

`bench.py --steps K --warmup W` runs W warm-up steps, K timed steps (graph replays) and then -- from the
state saved before the timed region -- the same K steps again eagerly for its HIP-event trace.  The step
kernel `mjw::reset_counters_kernel` is launched once per step, so the kernel-trace CSV (ordered by start
time) splits into steps at its dispatches: steps [W, W+K) are the timed window, [W+K, W+2K) its traced
re-run.  This prints the average duration per launch and per step of every kernel in both windows, so the
bench line's `roofline.kernel_ms` (from the re-run) can be checked against rocprof's own clock on the
identical steps.
"""
import collections
import csv
import glob
import json
import os
import sys

STEP_KERNEL = "mjw::reset_counters_kernel"


def kname(full):
  s = full.strip()
  if s.startswith("void "):
    s = s[5:]
  depth = 0
  for i, ch in enumerate(s):
    if ch == "<":
      depth += 1
    elif ch == ">":
      depth -= 1
    elif ch == "(" and depth == 0:
      return s[:i]
  return s


def dispatches(stats_dir):
  """[(start_ns, end_ns, kernel)] of every mjw dispatch, in start order."""
  out = []
  for f in glob.glob(os.path.join(stats_dir, "**", "*kernel_trace.csv"), recursive=True):
    with open(f) as fh:
      for r in csv.DictReader(fh):
        k = kname(r.get("Kernel_Name", ""))
        if "mjw" not in k:
          continue
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
  out.sort()
  return out


def split_steps(disp):
  """Dispatch lists per step (a step starts at each STEP_KERNEL dispatch; the ctrl-noise launch before it
  belongs to the previous step's list and is dropped by the caller's filter)."""
  steps, cur = [], None
  for d in disp:
    if d[2] == STEP_KERNEL:
      cur = []
      steps.append(cur)
    if cur is not None:
      cur.append(d)
  return steps


def window(steps, lo, hi):
  per = collections.defaultdict(list)
  nstep = 0
  for s in steps[lo:hi]:
    nstep += 1
    for t0, t1, k in s:
      if "ctrl_noise" in k:
        continue
      per[k].append((t1 - t0) * 1e-6)
  res = {}
  for k, v in sorted(per.items()):
    res[k] = {"avg_ms_per_launch": sum(v) / len(v), "launches_per_step": len(v) / max(1, nstep),
              "ms_per_step": sum(v) / max(1, nstep)}
  # wall span of the window's steps: first dispatch start to last dispatch end
  span = None
  if steps[lo:hi]:
    span = (steps[lo:hi][-1][-1][1] - steps[lo:hi][0][0][0]) * 1e-6 / max(1, nstep)
  return {"steps": nstep, "kernels": res, "kernel_sum_ms_per_step": sum(e["ms_per_step"] for e in res.values()),
          "span_ms_per_step": span}


def main():
  stats_dir, warm, nsteps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
  steps = split_steps(dispatches(stats_dir))
  res = {"steps_found": len(steps), "warmup": warm, "timed_steps": nsteps,
         "timed": window(steps, warm, warm + nsteps), "trace": window(steps, warm + nsteps, warm + 2 * nsteps)}
  txt = json.dumps(res, indent=1)
  if len(sys.argv) > 4:
    with open(sys.argv[4], "w") as fh:
      fh.write(txt)
  print(txt)


if __name__ == "__main__":
  main()
