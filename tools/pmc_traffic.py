"""Summarise rocprofv3 CSV output into profiles/: kernel-trace stats + per-kernel HBM traffic.

usage: python tools/pmc_traffic.py <stats_dir> <fetch_dir> <write_dir> <out.json> [worlds per launch] [solver] [model]
  model     : humanoid (default: the dense path's kernels) or a sparse-path model (cloth, aloha_cloth)
  stats_dir : rocprofv3 --kernel-trace --stats --output-format csv output directory
  fetch_dir : rocprofv3 --pmc FETCH_SIZE --output-format csv output directory
  write_dir : rocprofv3 --pmc WRITE_SIZE --output-format csv output directory
Traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes (MI355X_MICROARCH.md HBM section:
FETCH_SIZE counts half the bytes of wide streaming reads on gfx950; units are KB), averaged over
the dispatches of each kernel.
"""
import csv
import glob
import json
import os
import sys

KERNELS = {"forward": "mjw_kernel<79", "dense": "dense_kernel<7, false>"}
SPARSE_KERNELS = {"forward": "sp::forward_kernel", "solve": "sp::solve_kernel", "ccd": "sp::ccd_kernel", "euler": "sp::euler_kernel"}


def rows(d, pattern):
  out = []
  for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
    with open(f) as fh:
      out += list(csv.DictReader(fh))
  return out


def counter_avg(d, counter):
  vals = {k: [] for k in KERNELS}
  for r in rows(d, "*counter_collection.csv"):
    name = r.get("Kernel_Name", "")
    if r.get("Counter_Name") != counter:
      continue
    for k, pat in KERNELS.items():
      if pat in name.replace("mjw::", ""):
        vals[k].append(float(r["Counter_Value"]))
  return {k: (sum(v) / len(v) if v else None, len(v)) for k, v in vals.items()}


def main():
  global KERNELS
  stats_dir, fetch_dir, write_dir, out = sys.argv[1:5]
  nworld = int(sys.argv[5]) if len(sys.argv) > 5 else 8192
  solver = sys.argv[6] if len(sys.argv) > 6 else "CG"
  model = sys.argv[7] if len(sys.argv) > 7 else "humanoid"
  if model != "humanoid" and model in ("cloth", "aloha_cloth"):
    KERNELS = SPARSE_KERNELS
  fetch = counter_avg(fetch_dir, "FETCH_SIZE")
  write = counter_avg(write_dir, "WRITE_SIZE")
  stats = rows(stats_dir, "*kernel_stats.csv")
  sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
  from mujoco_warp_amd import build as _build

  res = {"nworld": nworld, "solver": solver, "model": model, "csrc_sha": _build.sources_hash(), "unit_note": "FETCH/WRITE_SIZE in KB per dispatch; hbm bytes = (2*FETCH + WRITE)*1024",
         "kernels": {}}
  for k, pat in KERNELS.items():
    f, nf = fetch[k]
    w, nw = write[k]
    st = [r for r in stats if pat in r.get("Name", "").replace("mjw::", "")]
    res["kernels"][k] = {
      "pattern": pat,
      "fetch_size_kb": f, "write_size_kb": w, "dispatches": [nf, nw],
      "hbm_bytes_per_launch": (2 * f + w) * 1024 if f is not None and w is not None else None,
      "avg_ns_rocprof": float(st[0]["AverageNs"]) if st else None,
    }
  if KERNELS is SPARSE_KERNELS:
    # per step: every forward-stage launch (frames / collision / rows / velocity) and one solve
    k = res["kernels"]
    nfwd = k["forward"]["dispatches"][0] / max(1, k["solve"]["dispatches"][0])
    parts = [k["forward"]["hbm_bytes_per_launch"], k["solve"]["hbm_bytes_per_launch"]]
    if None not in parts:
      k["forward"]["hbm_bytes_per_step_forward_plus_solve"] = nfwd * parts[0] + parts[1]
  with open(out, "w") as fh:
    json.dump(res, fh, indent=1)
  print(json.dumps(res, indent=1))


if __name__ == "__main__":
  main()
