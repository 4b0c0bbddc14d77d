"""Measurement bookkeeping on CPU: the per-step aggregation of rocprofv3 PMC summaries
(tools/pmc_traffic.py) and bench.py's choice of the dominant kernel group for `roofline`."""

import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _write(path, header, rows):
  os.makedirs(os.path.dirname(path), exist_ok=True)
  with open(path, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(header)
    w.writerows(rows)


def _pmc_dirs(tmp_path):
  """A sparse-path-like PMC run of 15 steps: 4 forward-stage launches, one index build and one CG launch
  per step (the round-2 bookkeeping took dispatches(forward) / dispatches(solve) = 60 / 30 = 2)."""
  launches = [("void mjw::sp::forward_kernel<256>(mjw_model_t, mjw_data_t, int)", 10.0, 1.0),
              ("void mjw::sp::forward_kernel<1024>(mjw_model_t, mjw_data_t, int)", 20.0, 2.0),
              ("void mjw::sp::forward_kernel<2048>(mjw_model_t, mjw_data_t, int)", 30.0, 3.0),
              ("void mjw::sp::forward_kernel<2>(mjw_model_t, mjw_data_t, int)", 40.0, 4.0),
              ("void mjw::sp::solve_kernel<0>(mjw_model_t, mjw_data_t)", 100.0, 10.0),
              ("void mjw::sp::solve_kernel<1>(mjw_model_t, mjw_data_t)", 1000.0, 100.0),
              ("mjw::sp::euler_kernel(mjw_model_t, mjw_data_t)", 5.0, 5.0),
              ("mjw::reset_counters_kernel(int*, int*)", 0.0, 0.0)]
  hdr = ["Kernel_Name", "Counter_Name", "Counter_Value"]
  fetch = [[n, "FETCH_SIZE", f] for _ in range(15) for n, f, w in launches]
  write = [[n, "WRITE_SIZE", w] for _ in range(15) for n, f, w in launches]
  _write(str(tmp_path / "fetch" / "x" / "run_counter_collection.csv"), hdr, fetch)
  _write(str(tmp_path / "write" / "x" / "run_counter_collection.csv"), hdr, write)
  stats = [[n, 15, 1000.0 * (i + 1)] for i, (n, f, w) in enumerate(launches)]
  _write(str(tmp_path / "stats" / "x" / "run_kernel_stats.csv"), ["Name", "Calls", "AverageNs"], stats)


def test_pmc_per_step_aggregation(tmp_path):
  import pmc_traffic

  _pmc_dirs(tmp_path)
  res = pmc_traffic.summarise(str(tmp_path / "stats"), str(tmp_path / "fetch"), str(tmp_path / "write"), 1024, "CG",
                              "aloha_cloth", "sha")
  k = res["kernels"]
  assert res["steps"] == [15, 15]
  # template instances stay separate, each with its own rocprof duration
  assert k["mjw::sp::solve_kernel<0>"]["hbm_bytes_per_launch"] == (2 * 100 + 10) * 1024
  assert k["mjw::sp::solve_kernel<1>"]["hbm_bytes_per_launch"] == (2 * 1000 + 100) * 1024
  assert k["mjw::sp::solve_kernel<0>"]["avg_ns"] == 5000.0 and k["mjw::sp::solve_kernel<1>"]["avg_ns"] == 6000.0
  assert all(v["launches_per_step"] == 1.0 for v in k.values())
  expect = sum((2 * f + w) * 1024 for f, w in [(10, 1), (20, 2), (30, 3), (40, 4), (100, 10), (1000, 100), (5, 5)])
  assert res["hbm_bytes_per_step_total"] == expect


def test_roofline_names_the_dominant_group():
  import bench

  # humanoid-like trace: dense kernel slower than the forward kernel
  dur = [[("mjw::reset_counters_kernel", 0.004), ("mjw::mjw_kernel<79, false>", 0.280), ("mjw::dense_kernel<7, false, false>", 0.290)]] * 3
  tab = bench.kernel_table(dur, False)
  pmc = {"mjw::dense_kernel<7, false, false>": {"bytes_per_launch": 95e6}, "mjw::mjw_kernel<79, false>": {"bytes_per_launch": 157e6}}
  r = bench.roofline_record(tab, {"forward": 18170.0, "dense": 3930.0}, 8192, pmc, "pmc_x.json")
  assert r["kernel"] == "mjw::dense_kernel<7, false, false>" and r["group"] == "dense"
  assert abs(r["kernel_ms"] - 0.290) < 1e-12
  assert abs(r["achieved"] - 3930.0 * 8192 / 0.290e-3 / 1e9) < 1e-9
  assert r["traffic"] == 95e6 and abs(r["groups"]["dense"]["traffic_over_alg"] - 95e6 / (3930.0 * 8192)) < 1e-12
  assert r["groups"]["forward"]["traffic_per_step"] == 157e6

  # sparse: four forward launches and two solve launches per step; the solve group dominates
  dur = [[("mjw::reset_counters_kernel", 0.004), ("mjw::sp::forward_kernel<256>", 0.4), ("mjw::sp::forward_kernel<1024>", 2.9),
          ("mjw::sp::forward_kernel<2048>", 1.3), ("mjw::sp::forward_kernel<2>", 0.85), ("mjw::sp::solve_kernel<0>", 1.8),
          ("mjw::sp::solve_kernel<1>", 16.6), ("mjw::sp::euler_kernel", 0.15)]]
  tab = bench.kernel_table(dur, True)
  r = bench.roofline_record(tab, {"forward": 3e6, "solve": 0.2e6, "euler": 0.03e6}, 1024, None, "none")
  assert r["group"] == "solve" and r["kernel"] == "mjw::sp::solve_kernel<0> + mjw::sp::solve_kernel<1>"
  assert abs(r["kernel_ms"] - 18.4) < 1e-9 and r["traffic"] is None
  assert abs(r["groups"]["forward"]["ms_per_step"] - 5.45) < 1e-9


def test_gpus_defaults_to_world_size(monkeypatch):
  import bench

  monkeypatch.setenv("WORLD_SIZE", "4")
  monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "3"])
  assert bench.parse().gpus == 4
  monkeypatch.delenv("WORLD_SIZE")
  assert bench.parse().gpus == 1
