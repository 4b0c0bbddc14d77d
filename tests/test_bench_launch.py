"""bench.py as the driver runs it: `--gpus N` starts N ranks itself (one process per GPU, gloo barrier,
no collective on the data path), weak and strong sharding, hipGraph replay.

On the 1-GPU box the two ranks share the device round-robin; each rank's final qpos must equal the
matching world range of a single-process run of the same global worlds (ctrl noise is indexed by global
world id through world_offset)."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, timeout=240):
  env = dict(os.environ)
  env.pop("WORLD_SIZE", None)
  env.pop("RANK", None)
  env.pop("LOCAL_RANK", None)
  out = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
  assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
  lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
  assert len(lines) == 1, out.stdout
  return json.loads(lines[0])


def test_launcher_command_without_gpu(monkeypatch):
  """`--gpus 2` with no WORLD_SIZE re-launches itself through torch.distributed.run (parent never touches HIP)."""
  sys.path.insert(0, ROOT)
  import bench

  seen = {}

  def fake_call(cmd, env=None):
    seen["cmd"], seen["env"] = cmd, env
    return 0

  monkeypatch.setattr(subprocess, "call", fake_call)
  monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
  assert bench.launch_ranks(2) == 0
  cmd = seen["cmd"]
  assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=2" in cmd
  assert "127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "2", "--steps", "3"]
  assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


@pytest.mark.gpu
@pytest.mark.parametrize("model,per_rank", [("humanoid", 256), ("apollo", 64)])
def test_gpu_bench_two_ranks_weak_equals_single(tmp_path, model, per_rank):
  """C2 and C4 (apollo: Newton, sensors, box-box CCD) sharded over two ranks: each rank's worlds
  bitwise equal to the same global worlds of one 2 x per_rank run."""
  common = ["--model", model, "--steps", "5", "--warmup", "2", "--cpu-baseline", "0", "--graph", "0"]
  two = _run(["--gpus", "2", "--nworld", str(per_rank), "--dump-qpos", str(tmp_path / "two")] + common)
  assert two["n_gpus"] == 2 and two["scaling"] == "weak"
  assert two["config"]["nworld_total"] == 2 * per_rank and two["config"]["converged_worlds"] == 2 * per_rank
  one = _run(["--gpus", "1", "--nworld", str(2 * per_rank), "--dump-qpos", str(tmp_path / "one")] + common)
  assert one["n_gpus"] == 1
  q1 = np.load(tmp_path / "one" / "qpos_rank0.npz")["qpos"]
  for r in range(2):
    z = np.load(tmp_path / "two" / f"qpos_rank{r}.npz")
    off = int(z["offset"])
    assert off == per_rank * r
    np.testing.assert_array_equal(z["qpos"], q1[off:off + per_rank])


@pytest.mark.gpu
def test_gpu_bench_two_ranks_strong_and_graph(tmp_path):
  common = ["--steps", "5", "--warmup", "2", "--cpu-baseline", "0", "--nworld", "301", "--trace-steps", "2"]
  strong = _run(["--gpus", "2", "--scaling", "strong", "--graph", "0", "--dump-qpos", str(tmp_path / "s")] + common)
  assert strong["scaling"] == "strong" and strong["config"]["nworld_total"] == 301
  # graph replay over two stream shards of one rank: the timed region is replays only, the kernel times
  # come from the 2-step eager trace pass after it (same number of steps as the strong run's)
  graph = _run(["--gpus", "1", "--graph", "1", "--streams", "2", "--dump-qpos", str(tmp_path / "g")] + common)
  assert graph["config"]["graph"] is True and graph["config"]["streams"] == 2
  assert graph["config"]["timed_region"] == "graph replays only" and graph["config"]["trace_steps"] == 2
  qg = np.load(tmp_path / "g" / "qpos_rank0.npz")["qpos"]
  got = [np.load(tmp_path / "s" / f"qpos_rank{r}.npz") for r in range(2)]
  assert [int(z["offset"]) for z in got] == [0, 151]
  np.testing.assert_array_equal(np.concatenate([z["qpos"] for z in got]), qg)


def test_pmc_traffic_is_bound_to_the_kernel_sources(tmp_path):
  """bench.py reports `roofline.traffic` only from a PMC summary of the same workload taken on a build of
  the current kernel sources (csrc_sha == build.sources_hash())."""
  sys.path.insert(0, ROOT)
  import bench
  from mujoco_warp_amd import build

  pmc = {"nworld": 8192, "solver": "CG", "model": "humanoid", "csrc_sha": build.sources_hash(),
         "kernels": {"mjw::dense_kernel<7, false>": {"hbm_bytes_per_launch": 123.0, "hbm_bytes_per_step": 123.0, "launches_per_step": 1.0}}}
  f = tmp_path / "pmc_humanoid_r99.json"
  f.write_text(json.dumps(pmc))
  assert bench.pmc_traffic(str(f), "humanoid", 8192, "CG")[0]["mjw::dense_kernel<7, false>"]["bytes_per_launch"] == 123.0
  assert bench.pmc_traffic(str(f), "humanoid", 4096, "CG")[0] is None  # other workload
  pmc["csrc_sha"] = "0" * 16
  f.write_text(json.dumps(pmc))
  traffic, why = bench.pmc_traffic(str(f), "humanoid", 8192, "CG")
  assert traffic is None and "predates" in why
  assert bench.pmc_traffic(str(tmp_path / "missing.json"), "humanoid", 8192, "CG")[0] is None


def test_pmc_traffic_ratio_uses_the_pmc_window(tmp_path):
  """traffic_over_alg divides the PMC bytes by the algorithmic bytes at the counted window's own nefc / ncon
  (tools/pmc_traffic.py records them from the PMC passes' bench lines), not at the trace pass's."""
  sys.path.insert(0, ROOT)
  import bench
  from mujoco_warp_amd import build

  k = "mjw::mjw_kernel<79, false, false>"
  pmc = {"nworld": 8, "solver": "CG", "model": "humanoid", "csrc_sha": build.sources_hash(),
         "window": {"fetch": {"nefc_mean": 10.0, "ncon_mean": 2.0}},
         "kernels": {k: {"hbm_bytes_per_launch": 8000.0, "hbm_bytes_per_step": 8000.0, "launches_per_step": 1.0}}}
  f = tmp_path / "pmc_humanoid_r99.json"
  f.write_text(json.dumps(pmc))
  traffic, src = bench.pmc_traffic(str(f), "humanoid", 8, "CG")
  tab = {k: {"ms_per_step": 1.0, "launches_per_step": 1.0, "group": "forward"}}
  alg_at = lambda ne, nc: {"forward": 100.0 * ne + nc}
  rec = bench.roofline_record(tab, alg_at(30.0, 5.0), 8, traffic, src, alg_at)
  assert rec["groups"]["forward"]["traffic_over_alg"] == 8000.0 / (8 * 1002.0)
  assert rec["groups"]["forward"]["alg_bytes_per_env_step"] == 3005.0
