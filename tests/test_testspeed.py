"""testspeed mirror (reference mujoco_warp/testspeed.py): flags, function discovery, metrics/output."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_flags_and_function_discovery():
  from mujoco_warp_amd import testspeed

  a = testspeed.parse(["models/humanoid.xml", "--nworld", "16", "-o", "opt.solver=cg", "-o", "opt.iterations=5", "--format", "json"])
  assert a.nworld == 16 and a.override == ["opt.solver=cg", "opt.iterations=5"] and a.format == "json"
  assert a.function == "step" and a.nstep == 1000 and a.keyframe == 0 and a.num_buckets == 10
  funcs = testspeed._funcs()
  # testspeed.py:46-50 discovers the (m, d) entry points
  for name in ("step", "forward", "fwd_position", "fwd_velocity", "fwd_actuation", "solve", "euler"):
    assert name in funcs


def test_metrics_and_buckets():
  from mujoco_warp_amd import testspeed

  a = testspeed.parse(["models/apptronik_apollo/scene_flat.xml", "--nworld", "4", "--nstep", "10"])
  trace = {"step": ([2.0], {"forward kernel": ([1.0], {})})}
  met = testspeed.collect_metrics(a, object(), object(), a.mjcf, 0.5, 2.0, trace, [8] * 10, [20] * 10, [np.array([3, 5])] * 10, 4)
  assert met["benchmark"] == "apptronik_apollo_flat"
  assert met["steps_per_second"] == 40 / 2.0 and met["converged_worlds"] == 4
  assert met["step"] == 1e6 * 2.0 / 40 and met["step.forward kernel"] == 1e6 * 1.0 / 40
  assert met["ncon_mean"] == 2.0 and met["nefc_p95"] == 20 and met["solver_niter_mean"] == 4.0
  rows = testspeed._buckets(list(range(10)), 10, 3)
  assert [r[2] for r in rows] == [0, 4, 7]


@pytest.mark.gpu
def test_gpu_testspeed_runs_humanoid():
  out = subprocess.run([sys.executable, "-m", "mujoco_warp_amd.testspeed", "models/humanoid.xml", "--nworld", "256", "--nstep", "20",
                        "-o", "opt.solver=cg", "--measure_alloc", "--measure_solver", "--event_trace", "--format", "json"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
  assert out.returncode == 0, out.stderr[-3000:]
  met = json.loads(out.stdout.strip().splitlines()[-1])
  assert met["converged_worlds"] == 256 and met["steps_per_second"] > 0
  assert met["ncon_mean"] > 0 and met["nefc_mean"] > 0 and met["solver_niter_mean"] > 0
  assert met["step.forward kernel"] > 0
  human = subprocess.run([sys.executable, "-m", "mujoco_warp_amd.testspeed", "models/humanoid.xml", "--nworld", "64", "--nstep", "10",
                          "--measure_alloc"], capture_output=True, text=True, timeout=240, cwd=ROOT)
  assert human.returncode == 0, human.stderr[-3000:]
  assert "Total steps per second" in human.stdout and "nefc alloc" in human.stdout
