"""Summarise rocprofv3 CSV output into profiles/: per-kernel HBM traffic and time, per launch and per step.

usage: python tools/pmc_traffic.py <stats_dir> <fetch_dir> <write_dir> <out.json> [worlds per launch] [solver] [model] [tail steps]
  tail steps: average the counters over the last N steps only (the passes warm up first)
  stats_dir : rocprofv3 --kernel-trace --stats --output-format csv output directory
  fetch_dir : rocprofv3 --pmc FETCH_SIZE --output-format csv output directory
  write_dir : rocprofv3 --pmc WRITE_SIZE --output-format csv output directory

Traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes (MI355X_MICROARCH.md HBM section: units
are KB; FETCH_SIZE counts half the bytes of wide streaming reads on gfx950), averaged over the dispatches of
each kernel (keyed by its demangled name without arguments, e.g. `mjw::sp::solve_kernel<1>`; the template
instances stay separate).

Per step: the number of steps in a PMC run is the dispatch count of `mjw::reset_counters_kernel`, which the
step launches exactly once; each kernel contributes dispatches / steps launches per step, and the step's
traffic is the sum over kernels of launches_per_step * bytes_per_launch.  Each kernel keeps its own
rocprof average duration (`avg_ns`, from the kernel-trace pass of the same command).
"""
import collections
import csv
import glob
import json
import os
import sys

STEP_KERNEL = "mjw::reset_counters_kernel"


def kname(full):
  """'void mjw::dense_kernel<7, false>(mjw_model_t, mjw_data_t, int)' -> 'mjw::dense_kernel<7, false>'."""
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


def rows(d, pattern):
  out = []
  for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
    with open(f) as fh:
      out += list(csv.DictReader(fh))
  return out


def counter(d, name):
  """{kernel: [values per dispatch, in dispatch order]} of one PMC counter."""
  vals = collections.defaultdict(list)
  for r in sorted(rows(d, "*counter_collection.csv"), key=lambda r: int(r.get("Dispatch_Id", 0) or 0)):
    if r.get("Counter_Name") != name:
      continue
    k = kname(r.get("Kernel_Name", ""))
    if "mjw" in k:
      vals[k].append(float(r["Counter_Value"]))
  return vals


def tail(vals, steps, tail_steps):
  """The dispatches of the last `tail_steps` of `steps` steps (all when tail_steps is 0)."""
  if not tail_steps or not steps or tail_steps >= steps:
    return vals
  return {k: v[len(v) - max(1, round(len(v) * tail_steps / steps)):] for k, v in vals.items()}


def bench_window(d):
  """nefc / ncon means of the bench line a PMC pass ran (its trace pass = the tail window the counters are
  averaged over, profile_model.sh), from the JSON line in <pass dir>.log."""
  try:
    with open(d.rstrip("/") + ".log") as fh:
      lines = [ln for ln in fh if ln.startswith("{")]
    rec = json.loads(lines[-1])
    c = rec["config"]
    return {"nefc_mean": c["nefc_mean"], "ncon_mean": c["ncon_mean"], "trace_steps": c.get("trace_steps")}
  except (OSError, IndexError, KeyError, ValueError):
    return None


def summarise(stats_dir, fetch_dir, write_dir, nworld, solver, model, csrc_sha, tail_steps=0):
  fetch = counter(fetch_dir, "FETCH_SIZE")
  write = counter(write_dir, "WRITE_SIZE")
  stats = {kname(r["Name"]): r for r in rows(stats_dir, "*kernel_stats.csv")}
  fetch = tail(fetch, len(fetch.get(STEP_KERNEL, [])), tail_steps)
  write = tail(write, len(write.get(STEP_KERNEL, [])), tail_steps)
  steps_f = len(fetch.get(STEP_KERNEL, []))
  steps_w = len(write.get(STEP_KERNEL, []))
  res = {"nworld": nworld, "solver": solver, "model": model, "csrc_sha": csrc_sha,
         "unit_note": "FETCH/WRITE_SIZE in KB per dispatch; hbm bytes = (2*FETCH + WRITE)*1024; per step = "
                      "sum over kernels of (dispatches / steps) * bytes per launch, steps = dispatches of " + STEP_KERNEL,
         "steps": [steps_f, steps_w], "tail_steps": tail_steps,
         # the counted window's constraint / contact sizes (the FETCH and WRITE passes run the same
         # deterministic steps): bench.py prices the window's algorithmic bytes with them
         "window": {"fetch": bench_window(fetch_dir), "write": bench_window(write_dir)}, "kernels": {}}
  total = 0.0
  for k in sorted(set(fetch) | set(write)):
    f, w = fetch.get(k, []), write.get(k, [])
    fa = sum(f) / len(f) if f else None
    wa = sum(w) / len(w) if w else None
    per_launch = (2 * fa + wa) * 1024 if fa is not None and wa is not None else None
    lps = len(f) / steps_f if steps_f else None
    st = stats.get(k)
    ent = {"fetch_size_kb": fa, "write_size_kb": wa, "dispatches": [len(f), len(w)], "hbm_bytes_per_launch": per_launch,
           "launches_per_step": lps,
           "hbm_bytes_per_step": per_launch * lps if per_launch is not None and lps is not None else None,
           "avg_ns": float(st["AverageNs"]) if st else None, "calls_in_stats_pass": int(st["Calls"]) if st else None}
    res["kernels"][k] = ent
    if ent["hbm_bytes_per_step"] is not None and k != STEP_KERNEL:
      total += ent["hbm_bytes_per_step"]
  res["hbm_bytes_per_step_total"] = total
  return res


def main():
  stats_dir, fetch_dir, write_dir, out = sys.argv[1:5]
  nworld = int(sys.argv[5]) if len(sys.argv) > 5 else 8192
  solver = sys.argv[6] if len(sys.argv) > 6 else "CG"
  model = sys.argv[7] if len(sys.argv) > 7 else "humanoid"
  tail_steps = int(sys.argv[8]) if len(sys.argv) > 8 else 0
  sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
  from mujoco_warp_amd import build as _build

  res = summarise(stats_dir, fetch_dir, write_dir, nworld, solver, model, _build.sources_hash(), tail_steps)
  with open(out, "w") as fh:
    json.dump(res, fh, indent=1)
  print(json.dumps(res, indent=1))


if __name__ == "__main__":
  main()
