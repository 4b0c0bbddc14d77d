"""testspeed: benchmark the batched step on an MJCF (mirror of mujoco_warp/testspeed.py).

Usage: python -m mujoco_warp_amd.testspeed <mjcf XML path> [flags]

Example:
  python -m mujoco_warp_amd.testspeed models/humanoid.xml --nworld 8192 -o "opt.solver=cg"

Flags, metrics and output formats follow the reference CLI (testspeed.py:46-78 flags, :112-161
_collect_metrics, :164-282 output): the function is one of the package's `(m, d)` entry points,
state starts from `--keyframe`, every step applies the benchmark's OU + Halton control noise around
the keyframe controls (benchmark.py:41-83), and the function is captured once as a hipGraph and
replayed per step with only the replay timed (benchmark.py:123-155).  `--event_trace` replaces the
reference's per-@event_scope Warp events (warp_util.py:25-119) with HIP events around the step's
kernels (the forward kernel, then factor / solve / integrate): the work of this path is two
fused launches, not ~100 scoped Warp launches.
"""

from __future__ import annotations

import argparse
import inspect
import json
import os
import sys
import time

import numpy as np


def _funcs():
  import mujoco_warp_amd as mjw

  return {n: f for n, f in inspect.getmembers(mjw, inspect.isfunction) if set(inspect.signature(f).parameters.keys()) == {"m", "d"}}


def parse(argv=None):
  p = argparse.ArgumentParser(prog="testspeed", description=__doc__.splitlines()[0])
  p.add_argument("mjcf", help="MJCF XML path")
  p.add_argument("--function", default="step", help="the function to benchmark (an (m, d) entry point)")
  p.add_argument("--nstep", type=int, default=1000, help="number of steps per rollout")
  p.add_argument("--nworld", type=int, default=8192, help="number of parallel rollouts")
  p.add_argument("--nconmax", type=int, default=None, help="override maximum number of contacts per world")
  p.add_argument("--njmax", type=int, default=None, help="override maximum number of constraints per world")
  p.add_argument("--njmax_nnz", type=int, default=None, help="override maximum number of non-zeros in constraint Jacobian")
  p.add_argument("--nccdmax", type=int, default=None, help="override maximum number of CCD contacts per world")
  p.add_argument("-o", "--override", action="append", default=[], help="Model overrides (notation: foo.bar = baz)")
  p.add_argument("--keyframe", type=int, default=0, help="keyframe to initialize simulation.")
  p.add_argument("--event_trace", action="store_true", help="print an event trace report")
  p.add_argument("--measure_alloc", action="store_true", help="print a report of contacts and constraints per step")
  p.add_argument("--measure_solver", action="store_true", help="print a report of solver iterations per step")
  p.add_argument("--num_buckets", type=int, default=10, help="number of buckets to summarize rollout measurements")
  p.add_argument("--device", default=None, help="override the default device (cuda:N)")
  p.add_argument("--memory", action="store_true", help="print memory report")
  p.add_argument("--format", default="human", choices=["human", "short", "json"], help="output format for results")
  p.add_argument("--info", action="store_true", help="print Model and Data info")
  return p.parse_args(argv)


def benchmark(fn, m, d, nstep, center=None, event_trace=False, measure_alloc=False, measure_solver_niter=False):
  """benchmark.py:86-171: capture `fn(m, d)` as a hipGraph, then per step launch the control noise,
  replay the graph and time the replay alone.  Returns (capture time, run time, trace, nacon, nefc,
  solver_niter, converged worlds)."""
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd.forward import step_timed

  dev = d.qpos.device
  trace = {}
  nacon, nefc, solver_niter = [], [], []
  cap_beg = time.perf_counter()
  s = torch.cuda.Stream(device=dev)
  s.wait_stream(torch.cuda.current_stream(dev))
  graph = torch.cuda.CUDAGraph()
  with torch.cuda.graph(graph, stream=s):
    fn(m, d)
  torch.cuda.synchronize(dev)
  cap_duration = time.perf_counter() - cap_beg
  ev = None
  if event_trace:
    ev = tuple(torch.cuda.Event(enable_timing=True) for _ in range(3))
    for e in ev:
      e.record()
  t_fwd = t_rest = 0.0
  time_vec = np.zeros(nstep)
  for i in range(nstep):
    mjw.ctrl_noise(m, d, i, center=center)
    torch.cuda.synchronize(dev)
    run_beg = time.perf_counter()
    graph.replay()
    torch.cuda.synchronize(dev)
    time_vec[i] = time.perf_counter() - run_beg
    if measure_alloc:
      nacon.append(max(int(d.nacon[0]), int(d.ncollision[0])))
      nefc.append(int(d.nefc.max()))
    if measure_solver_niter:
      solver_niter.append(d.solver_niter.cpu().numpy())
  if ev is not None and fn is mjw.step:
    # kernel split of the step: the rollout continues eagerly for nstep // 10 untimed steps with HIP
    # events around the kernels of each, scaled to the timed rollout
    n_ev = max(1, nstep // 10)
    for i in range(n_ev):
      mjw.ctrl_noise(m, d, nstep + i, center=center)
      step_timed(m, d, *ev)
      torch.cuda.synchronize(dev)
      t_fwd += ev[0].elapsed_time(ev[1]) * 1e-3
      t_rest += ev[1].elapsed_time(ev[2]) * 1e-3
    scale = nstep / n_ev
    total = float(np.sum(time_vec))
    trace = {"step": ([total], {"forward kernel": ([t_fwd * scale], {}), "factor/solve/integrate kernel(s)": ([t_rest * scale], {})})}
  nsuccess = int((~torch.isnan(d.qpos).any(dim=1)).sum())
  return cap_duration, float(np.sum(time_vec)), trace, nacon, nefc, solver_niter, nsuccess


def _memory(obj, prefix=""):
  import torch

  out = []
  for k, v in vars(obj).items():
    if isinstance(v, torch.Tensor):
      out.append((prefix + k, v.numel() * v.element_size()))
    elif hasattr(v, "__dict__") and type(v).__module__.startswith("mujoco_warp_amd") and not callable(v):
      out.extend(_memory(v, prefix + k + "."))
  return out


def collect_metrics(args, m, d, path, jit_time, run_time, trace, nacon, nefc, solver_niter, nsuccess):
  """testspeed.py:112-161."""
  steps = args.nworld * args.nstep
  base = os.path.basename(path)
  stem = os.path.splitext(base)[0]
  metrics = {
    "benchmark": os.path.basename(os.path.dirname(os.path.abspath(path))) + stem.replace("scene", "") if base.startswith("scene") else stem,
    "jit_duration": jit_time,
    "run_time": run_time,
    "steps_per_second": steps / run_time,
    "converged_worlds": int(nsuccess),
  }

  def flatten_trace(prefix, tr):
    for k, (times, sub) in tr.items():
      for i, t in enumerate(times):
        metrics[f"{prefix}{k}{f'[{i}]' if len(times) > 1 else ''}"] = 1e6 * t / steps
      flatten_trace(f"{prefix}{k}.", sub)

  flatten_trace("", trace)
  if args.memory:
    metrics.update({"model_memory": sum(c for _, c in _memory(m)), "data_memory": sum(c for _, c in _memory(d))})
  if nacon and nefc:
    metrics.update({
      "ncon_mean": np.mean(nacon) / args.nworld,
      "ncon_p95": np.percentile(nacon, 95) / args.nworld,
      "nefc_mean": np.mean(nefc),
      "nefc_p95": np.percentile(nefc, 95),
    })
  if solver_niter:
    metrics.update({"solver_niter_mean": np.mean(solver_niter), "solver_niter_p95": np.percentile(solver_niter, 95)})
  return metrics


def _buckets(values, nstep, nbucket):
  idx, rows = 0, []
  for i in range(nbucket):
    size = nstep // nbucket + (i < (nstep % nbucket))
    arr = np.array(values[idx:idx + size])
    if arr.size:
      rows.append([np.mean(arr), np.std(arr), np.min(arr), np.max(arr)])
    idx += size
  return rows


def _print_table(matrix, headers, title):
  ncol = len(headers)
  widths = [max([len(f"{row[i]:g}") for row in matrix] + [len(headers[i])]) for i in range(ncol)]
  print(f"\n{title}:\n")
  print("  ".join(f"{headers[i]:<{widths[i]}}" for i in range(ncol)))
  print("-" * sum(widths) + "--" * 3)
  for row in matrix:
    print("  ".join(f"{row[i]:{widths[i]}g}" for i in range(ncol)))


def output_human(args, m, d, mjm, jit_time, run_time, trace, nacon, nefc, solver_niter, nsuccess):
  """testspeed.py:164-282."""
  steps = args.nworld * args.nstep
  timestep = float(m.opt.timestep.reshape(-1)[0])
  print(f"""
Summary for {args.nworld} parallel rollouts

Total JIT time: {jit_time:.2f} s
Total simulation time: {run_time:.2f} s
Total steps per second: {steps / run_time:,.0f}
Total realtime factor: {steps * timestep / run_time:,.2f} x
Total time per step: {1e9 * run_time / steps:.2f} ns
Total converged worlds: {nsuccess} / {d.nworld}""")
  if trace:
    print("\nEvent trace:\n")

    def show(tr, indent):
      for k, (times, sub) in tr.items():
        print("  " * indent + f"{k}: " + ", ".join(f"{1e6 * t / steps:.2f}" for t in times))
        show(sub, indent + 1)

    show(trace, 0)
  if nacon and nefc:
    _print_table(_buckets(nacon, args.nstep, args.num_buckets), ("mean", "std", "min", "max"), "nacon alloc")
    _print_table(_buckets(nefc, args.nstep, args.num_buckets), ("mean", "std", "min", "max"), "nefc alloc")
  if solver_niter:
    _print_table(_buckets(solver_niter, args.nstep, args.num_buckets), ("mean", "std", "min", "max"), "solver niter")
  if args.memory:
    for obj, name in ((m, "\nModel"), (d, "Data")):
      mem = _memory(obj)
      total = sum(c for _, c in mem)
      print(f"{name} memory {total / 1024**2:.2f} MiB:")
      for field, c in mem:
        if total and c / total >= 0.01:
          print(f" {field}: {c / 1024**2:.2f} MiB ({100 * c / total:.2f}%)")


def main(argv=None):
  args = parse(argv)
  import torch

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf

  funcs = _funcs()
  if args.function not in funcs:
    raise SystemExit(f"--function must be one of {sorted(funcs)}")
  if not torch.cuda.is_available():
    raise SystemExit("testspeed available for gpu only")  # testspeed.py:300-301
  dev = torch.device(args.device or "cuda")
  if args.format == "human":
    print(f"Loading model from: {args.mjcf}...\n")
  mjm = mjcf.load_model(args.mjcf)
  mjd = mjcf.MjData(mjm)
  center = None
  if mjm.nkey > 0 and args.keyframe > -1:
    mjcf.reset_data_keyframe(mjm, mjd, args.keyframe)
    center = torch.as_tensor(np.asarray(mjd.ctrl, dtype=np.float32), device=dev)
  mjw.override_model(mjm, args.override)
  m = mjw.put_model(mjm, device=dev)
  mjw.override_model(m, args.override)
  d = mjw.put_data(mjm, mjd, nworld=args.nworld, nconmax=args.nconmax, njmax=args.njmax, njmax_nnz=args.njmax_nnz,
                   nccdmax=args.nccdmax, device=dev, m=m)
  if args.format == "human":
    sizes = [f"{n}: {getattr(mjm, n)}" for n in ("nq", "nv", "nu", "nbody", "ngeom") if getattr(mjm, n) > 0]
    print("Model\n  " + " ".join(sizes))
    print(f"Option\n  integrator: {mjw.IntegratorType(int(m.opt.integrator)).name}\n  cone: {mjw.ConeType(int(m.opt.cone)).name}\n"
          f"  solver: {mjw.SolverType(int(m.opt.solver)).name} iterations: {int(m.opt.iterations)} ls_iterations: {int(m.opt.ls_iterations)}\n"
          f"  is_sparse: {bool(m.is_sparse)}")
    print(f"Data\n  nworld: {d.nworld} naconmax: {d.naconmax} njmax: {d.njmax}\n")
    print(f"Rolling out {args.nstep} steps at dt = {float(m.opt.timestep.reshape(-1)[0]):g}...")
  fn = funcs[args.function]
  res = benchmark(fn, m, d, args.nstep, center, args.event_trace, args.measure_alloc, args.measure_solver)
  if args.format == "human":
    output_human(args, m, d, mjm, *res)
  else:
    metrics = collect_metrics(args, m, d, args.mjcf, *res)
    if args.format == "json":
      del metrics["benchmark"]
      print(json.dumps(metrics))
    else:
      bench = metrics.pop("benchmark")
      w = max(len(k) for k in metrics) + len(bench)
      for k, v in metrics.items():
        print(f"{bench}:{k:<{w}} {v}")


if __name__ == "__main__":
  main(sys.argv[1:])
