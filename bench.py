"""Benchmark: env-steps/s of the batched humanoid step (BASELINE.json metric).

Workload (BASELINE.json configs[1]): benchmarks/humanoid/humanoid.xml, nworld=8192
per GPU, fp32, Euler + CG (opt.solver override), nconmax=24, njmax=64
(benchmarks/config.txt:21), state from keyframe 0 ("squat"), qvel = warmstart = 0,
and before every step the reference's Ornstein-Uhlenbeck + Halton control noise
(_src/benchmark.py:41-83, std 0.01, rate 0.1, global world ids).  One "step" =
ctrl_noise + mjw.step over all worlds; the timed region contains exactly K steps
(ctrl_noise included, i.e. slightly conservative vs the reference which times
only the graph replay).

Multi-GPU: one process per GPU (torch.distributed.run, or `--gpus N` alone, which
starts the N ranks itself); each rank owns 8192 worlds (weak scaling, world ids
offset by rank) or `--scaling strong` splits --nworld over the ranks; no
collective on the data path: a gloo (host) barrier + max-over-ranks of the
elapsed time brackets the timed region.

A step is a counter reset and two kernels on the torch stream: the forward kernel
mjw::mjw_kernel<79, ...> (kinematics, com, crb/qM, collision, constraint rows,
transmission, velocity, rne, actuation, qfrc_smooth) and the dense kernel
mjw::dense_kernel<7, ...> (Cholesky + M^-1, CG solve, Euler).  As in the
reference's benchmark (benchmark.py:123-155) the step is captured once as a
hipGraph (after the first warmup step) and replayed every step, the control noise
launched before each replay; the timed region holds graph replays only.  The whole
Data state is saved right before it; after it the state is restored and the same
steps (same state, same control-noise indices, so bitwise the same work) run again
eagerly through mjw_step_trace, which records a HIP event on that stream after every
kernel launch and so times each kernel over exactly the timed window.  The record
checks that the traced kernel sum per step is <= 1.03 x the timed ms/step.

Also reported: `roofline` for the dominant kernel group -- the one with the most
time per step (the forward kernel on the humanoid, the CG solve on the sparse path):
its algorithmic bytes per env-step (SURVEY.md 8(d)'s B_alg split by the kernel that
writes each output, DESIGN.md 3.5, at the trace pass's nefc / ncon) x worlds per
launch over its HIP-event time vs the 8 TB/s HBM peak, and its traffic from the
committed rocprofv3 PMC passes ((2 FETCH_SIZE + WRITE_SIZE) KB -> B, summed per step
over the group's launches, with the PMC window's own algorithmic bytes for the
ratio); every group's figures side by side in `roofline.kernels`; and `cpu_baseline`
(the fp64 C oracle, OpenMP over worlds on the box's CPU share, bounded sample, rank 0).
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (whole node), humanoid.xml nworld=8192 at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec


# benchmark configurations (BASELINE.json configs; benchmarks/config.txt sizes)
MODELS = {
  # C2, the headline: humanoid, Euler + CG override, keyframe 0 ("squat")
  "humanoid": dict(path="models/humanoid.xml", nworld=8192, nconmax=24, njmax=64, solver="CG", key=0),
  # C3: franka (implicitfast, model-default Newton), no keyframe -> ctrl noise around ctrlrange midpoints
  "franka": dict(path="models/franka_emika_panda/scene.xml", nworld=16384, nconmax=1, njmax=5, solver=None, key=None),
  # C4: apollo (Euler, model-default Newton, IMU sensors, box-box CCD), keyframe "stand"
  "apollo": dict(path="models/apptronik_apollo/scene_flat.xml", nworld=4096, nconmax=16, njmax=64, solver=None, key=0),
  # C5 stand-in: the reference's `cloth` benchmark (benchmarks/cloth/scene.xml, config.txt:19: nconmax 200,
  # njmax 3000, 100 steps) -- the same 30x30 flex towel as aloha_cloth over a mannequin instead of the
  # mesh arms; sparse path (mjw_sparse.hip), CG, starts from qpos0 (towel falls onto the mannequin)
  "cloth": dict(path="models/cloth/scene.xml", nworld=1024, nconmax=200, njmax=3000, solver=None, key=None, steps=100,
                cpu_worlds=16, cpu_steps=8),
  # C5: aloha_cloth (benchmarks/aloha_cloth/scene.xml: two mesh arms + the 30x30 towel lying on the
  # table), keyframe "neutral_pose", 100 steps (config.txt:13).  The towel's 1682 triangles touch the
  # table box twice each (3364 contacts, ~16k rows), so config.txt's nconmax 920 / njmax 6300 would
  # truncate both; this run sizes them so that nothing is dropped
  "aloha_cloth": dict(path="models/aloha_cloth/scene.xml", nworld=1024, nconmax=4096, njmax=16384, solver=None, key=0, steps=100,
                      cpu_worlds=16, cpu_steps=2),
}


def step_words(mjm, nv_pad, sparse=False):
  """Algorithmic words per env-step of SURVEY.md 8(d), from the model sizes: (state inputs, fixed
  Data-contract outputs of the forward kernels, fixed outputs of the dense kernel).  For the
  humanoid: 233 + 3012 + 925 = 4170 words.  Sparse models store qM / qLD as nM ancestor entries
  and add the flex outputs (vertex positions, edge length / velocity / Jacobian)."""
  nq, nv, nu, nb, nj, ng = mjm.nq, mjm.nv, mjm.nu, mjm.nbody, mjm.njnt, mjm.ngeom
  nJmom = nu  # joint transmissions: one moment entry per actuator
  w_in = nq + nv + nu + nv + nv + 6 * nb + 1  # qpos qvel ctrl qacc_warmstart qfrc_applied xfrc_applied time
  kin = nb * (3 + 4 + 9 + 3 + 9) + nj * 6 + ng * 12 + mjm.nsite * 12
  camlight = mjm.ncam * 12 + mjm.nlight * 6
  com = 3 * nb + 10 * nb + 6 * nv
  crb = 10 * nb + (int(mjm.nM) if sparse else nv_pad * nv_pad)
  trn = nu + nJmom + 3 * nu
  vel = 6 * nb + 6 * nv + nu
  passive = 3 * nv
  rne = nv + 12 * nb
  act = nu + 2 * nv
  sensors = getattr(mjm, "nsensordata", 0)
  flex = 3 * getattr(mjm, "nflexvert", 0) + 8 * getattr(mjm, "nflexedge", 0)
  fwd_out = kin + camlight + com + crb + trn + vel + passive + rne + act + sensors + flex + 2
  dense_out = (int(mjm.nM) if sparse else nv * nv) + nv + (3 * nv + 5) + (nq + 2 * nv + 1)  # qLD, qacc_smooth, solver, integrator
  return w_in, fwd_out, dense_out


def b_alg_parts(words, nefc_mean, ncon_mean, nv_pad):
  """(forward, dense) algorithmic bytes per env-step: per constraint row 10 scalars + a J row of
  nv_pad (2 of them, force / state, written by the dense kernel), per contact 38 words."""
  w_in, fwd_out, dense_out = words
  fwd = 4.0 * (w_in + fwd_out + (8.0 + nv_pad) * nefc_mean + 38.0 * ncon_mean)
  dense = 4.0 * (dense_out + 2.0 * nefc_mean)
  return fwd, dense


def b_alg_groups(mjm, words, nefc_mean, ncon_mean, row_words, sparse):
  """Algorithmic bytes per env-step by kernel group (the kernels that write those outputs).  Dense path:
  forward (mjw_kernel, the convex pre-pass) and dense (factor / solve / Euler, the sensor kernel).  Sparse
  path: forward (the four stage kernels + the mesh pre-pass; they also write qLD and qacc_smooth), solve
  (transposed index + CG: qacc, qfrc_constraint, efc_Ma, solver scalars, efc force / state) and euler."""
  fwd, dense = b_alg_parts(words, nefc_mean, ncon_mean, row_words)
  if not sparse:
    # step: the fused whole-step kernel (mjw_step.hip step_kernel) writes both groups' outputs
    return {"forward": fwd, "dense": dense, "step": fwd + dense}
  solve = 4.0 * (3 * mjm.nv + 5 + 2.0 * nefc_mean)
  euler = 4.0 * (mjm.nq + 2 * mjm.nv + 1)
  return {"forward": fwd + dense - solve - euler, "solve": solve, "euler": euler}


def kernel_group(name, sparse):
  """Kernel group of a traced launch (see b_alg_groups); 'other' = the pool-counter reset."""
  if "reset_counters" in name or "ctrl_noise" in name:
    return "other"
  if sparse:
    if "solve_kernel" in name:
      return "solve"
    if "euler_kernel" in name:
      return "euler"
    return "forward"
  if "dense_kernel" in name or "sensor_acc" in name or "sensor_coll" in name:
    return "dense"
  if "step_kernel" in name:
    return "step"
  return "forward"


def parse():
  p = argparse.ArgumentParser()
  p.add_argument("--gpus", type=int, default=None, help="GPUs (ranks); default: WORLD_SIZE when launched by torchrun, else 1")
  p.add_argument("--steps", type=int, default=None, help="timed steps (default: the config's, 1000 unless stated)")
  p.add_argument("--warmup", type=int, default=20)
  p.add_argument("--model", default="humanoid", choices=sorted(MODELS), help="benchmark config (default: the headline C2)")
  p.add_argument("--nworld", type=int, default=None, help="worlds per GPU (default: the config's)")
  p.add_argument("--solver", default=None, choices=["CG", "NEWTON"], help="override opt.solver (default: the config's)")
  p.add_argument("--nconmax", type=int, default=None)
  p.add_argument("--njmax", type=int, default=None)
  p.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on rank 0 (0 = skip)")
  p.add_argument("--cpu-worlds", type=int, default=None, help="CPU baseline sample worlds (default: the config's, 1024)")
  p.add_argument("--cpu-steps", type=int, default=None, help="CPU baseline sample steps (default: the config's, 1000)")
  p.add_argument("--pmc", default=None, help="PMC traffic summary (default: the newest profiles/pmc_<model>_rNN.json)")
  p.add_argument("--graph", type=int, default=1, help="capture mjw.step once as a hipGraph and replay it every step "
                 "(benchmark.py:123-155: ctrl noise is launched outside the graph); 0 = launch the step eagerly")
  p.add_argument("--trace-steps", type=int, default=0,
                 help="after the timed region the Data state saved before it is restored and the first --trace-steps "
                 "of the same timed steps (0 = all of them) run again eagerly with a HIP event after each kernel "
                 "launch (mjw_step_trace): the per-kernel durations of `roofline`; every timed step is a graph replay")
  p.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                 help="weak: --nworld worlds per rank; strong: --nworld worlds in total, split over the ranks")
  p.add_argument("--streams", type=int, default=1,
                 help="independent world shards per rank, each with its own Data and HIP stream (measured slower "
                 "than one batch on the humanoid: 12.2 vs 13.9 M env-steps/s)")
  p.add_argument("--dump-qpos", default=None, help="directory: each rank writes its final qpos + world offset (tests)")
  a = p.parse_args()
  if a.gpus is None:  # torchrun without --gpus: one rank per process of the launch
    a.gpus = int(os.environ.get("WORLD_SIZE", "1"))
  cfg = MODELS[a.model]
  for k in ("nworld", "nconmax", "njmax", "solver"):
    if getattr(a, k) is None:
      setattr(a, k, cfg[k])
  if a.pmc is None:  # the committed summaries for this model (pmc_<model>[_<solver>]_rNN.json), newest first;
    import glob    # main() takes the first one that matches the workload and the current kernel sources

    found = glob.glob(os.path.join(ROOT, "profiles", f"pmc_{a.model}_r[0-9]*.json"))
    found += glob.glob(os.path.join(ROOT, "profiles", f"pmc_{a.model}_[a-z]*_r[0-9]*.json"))
    a.pmc = sorted(set(found), key=lambda f: (os.path.basename(f).rsplit("_r", 1)[-1], os.path.getmtime(f)), reverse=True)
  else:
    a.pmc = [a.pmc]
  for k, dflt in (("steps", 1000), ("cpu_worlds", 1024), ("cpu_steps", 1000)):
    if getattr(a, k) is None:
      setattr(a, k, cfg.get(k, dflt))
  return a


def _host_cpu():
  """(logical CPUs of the host, CPUs this process may run on, model name) for the cpu_baseline record."""
  model = None
  try:
    with open("/proc/cpuinfo") as f:
      for line in f:
        if line.startswith("model name"):
          model = line.split(":", 1)[1].strip()
          break
  except OSError:
    pass
  try:
    allowed = len(os.sched_getaffinity(0))
  except AttributeError:
    allowed = os.cpu_count() or 1
  return os.cpu_count() or 1, allowed, model


def cpu_baseline(mjm, nworld, nsteps, key, njmax, nconmax, model):
  """C oracle (restatement of the reference step), OpenMP over worlds on every CPU this process may use;
  rank 0 only.  fp64 is the parity oracle and the reported value; the fp32 build (the path's arithmetic
  type) is timed on the same sample next to it."""
  from oracle import orc

  nproc, allowed, cpu_model = _host_cpu()
  # the GPU box grants a 1-GPU job its CPU share through OMP_NUM_THREADS (16) while the affinity mask shows
  # the whole host; the baseline uses that share, all of it (MJW_CPU_BASELINE_THREADS overrides)
  nthread = int(os.environ.get("MJW_CPU_BASELINE_THREADS", "0")) or int(os.environ.get("OMP_NUM_THREADS", "0")) or allowed
  nthread = max(1, min(nthread, allowed))
  rates = {}
  for bits in (64, 32):
    om = orc.OracleModel(mjm, real_bits=bits)
    od = orc.OracleData(om, nworld, njmax, nconmax)
    center = None
    if key is not None:
      od.qpos[:] = mjm.key_qpos[key]
      od.ctrl[:] = mjm.key_ctrl[key]
      center = mjm.key_ctrl[key]
    t0 = time.perf_counter()
    for i in range(nsteps):
      od.ctrl_noise(i, center=center)
      od.step(nthread=nthread)
    rates[bits] = (nworld * nsteps / (time.perf_counter() - t0), time.perf_counter() - t0)
  return dict(
    value=rates[64][0],
    unit="env-steps/s",
    cores=nthread,
    kind="port",
    value_fp32=rates[32][0],
    value_per_thread=rates[64][0] / nthread,
    # worlds are independent, so the OpenMP loop scales with threads up to the memory bandwidth; this is
    # the linear extrapolation to every CPU the affinity mask shows, not a measurement
    value_all_cpus_linear_estimate=rates[64][0] / nthread * allowed,
    host_nproc=nproc,
    host_cpus_allowed=allowed,
    cpu_model=cpu_model,
    sample=f"C oracle (oracle/oracle.c), {model}, {nworld} worlds x {nsteps} steps with ctrl noise, {nthread} OpenMP "
    f"threads = the box's CPU share for one GPU (host: {nproc} logical CPUs, {allowed} in the affinity mask), "
    f"fp64 {rates[64][1]:.1f} s (value), fp32 "
    f"{rates[32][1]:.1f} s (value_fp32); the reference's Warp-CPU path is not runnable here (no warp/mujoco)",
  )


def pmc_traffic(path, model, nworld, solver_name):
  """Per-kernel HBM bytes from a committed rocprofv3 PMC summary (tools/pmc_traffic.py): {kernel name:
  {bytes_per_launch, bytes_per_step, launches_per_step}}, only when that summary was taken on the same
  workload (`nworld` = worlds per launch) AND on a kernel build from the current sources (its `csrc_sha`
  equals build.sources_hash()); else (None, reason)."""
  from mujoco_warp_amd import build as _build

  if not path or not os.path.exists(path):
    return None, "no PMC summary"
  with open(path) as f:
    pmc = json.load(f)
  if pmc.get("solver", "CG") != solver_name or pmc.get("nworld") != nworld or pmc.get("model", "humanoid") != model:
    return None, f"PMC summary {os.path.basename(path)} is for another workload"
  if pmc.get("csrc_sha") != _build.sources_hash():
    return None, f"PMC summary {os.path.basename(path)} predates the current kernel sources"
  out = {}
  for k, v in pmc.get("kernels", {}).items():
    if v.get("hbm_bytes_per_launch") is None:
      continue
    out[k] = {"bytes_per_launch": v["hbm_bytes_per_launch"], "bytes_per_step": v.get("hbm_bytes_per_step"),
              "launches_per_step": v.get("launches_per_step")}
  # the counted window's nefc / ncon (tools/pmc_traffic.py records the PMC passes' own bench lines)
  win = (pmc.get("window") or {}).get("fetch")
  if win is not None:
    out["_window"] = {"nefc_mean": float(win["nefc_mean"]), "ncon_mean": float(win["ncon_mean"])}
  return out, os.path.basename(path)


def kernel_table(durations, sparse):
  """Per kernel: mean time and launches per step over the traced steps (mjw_step_trace durations)."""
  tab = {}
  nstep = max(1, len(durations))
  for launches in durations:
    for name, ms in launches:
      e = tab.setdefault(name, {"ms_per_step": 0.0, "launches_per_step": 0.0, "group": kernel_group(name, sparse)})
      e["ms_per_step"] += ms / nstep
      e["launches_per_step"] += 1.0 / nstep
  return tab


def roofline_record(tab, groups_alg, nworld, pmc, pmc_src, groups_alg_at=None):
  """`roofline` of the dominant kernel group (most time per step) and the per-group / per-kernel figures.
  `groups_alg_at(nefc, ncon)` prices the algorithmic bytes at the PMC window's sizes for traffic_over_alg
  (the counters were taken on other steps than the trace pass; without a recorded window the trace pass's
  bytes are used and the record says so)."""
  win = (pmc or {}).get("_window")
  alg_pmc = groups_alg_at(win["nefc_mean"], win["ncon_mean"]) if (win and groups_alg_at) else groups_alg
  groups = {}
  for name, e in tab.items():
    g = groups.setdefault(e["group"], {"kernels": [], "ms_per_step": 0.0, "traffic_per_step": 0.0, "traffic_known": True})
    g["kernels"].append(name)
    g["ms_per_step"] += e["ms_per_step"]
    t = (pmc or {}).get(name)
    e["alg_group"] = e["group"]
    if t is not None:
      e["traffic_per_launch"] = t["bytes_per_launch"]
      e["traffic_per_step"] = t["bytes_per_launch"] * e["launches_per_step"]
      g["traffic_per_step"] += e["traffic_per_step"]
    else:
      e["traffic_per_launch"] = None
      g["traffic_known"] = False
  rec = {}
  for gname, g in groups.items():
    alg = groups_alg.get(gname)
    ach = alg * nworld / (g["ms_per_step"] * 1e-3) / 1e9 if alg and g["ms_per_step"] > 0 else None
    rec[gname] = {
      "kernels": sorted(g["kernels"]), "ms_per_step": g["ms_per_step"],
      "alg_bytes_per_env_step": alg, "alg_bytes_per_step": alg * nworld if alg else None,
      "achieved_GBs": ach, "frac": ach / HBM_PEAK_GBS if ach else None,
      "traffic_per_step": g["traffic_per_step"] if g["traffic_known"] else None,
      "traffic_over_alg": (g["traffic_per_step"] / (alg_pmc[gname] * nworld)) if g["traffic_known"] and alg_pmc.get(gname) else None,
    }
  cand = {k: v for k, v in rec.items() if v["alg_bytes_per_env_step"]}
  dom = max(cand, key=lambda k: cand[k]["ms_per_step"])
  d = rec[dom]
  return {
    "bound": "hbm",
    "achieved": d["achieved_GBs"],
    "peak": HBM_PEAK_GBS,
    "unit": "GB/s",
    "frac": d["frac"],
    "traffic": d["traffic_per_step"],
    "traffic_source": pmc_src,
    "traffic_note": "HBM bytes per step of the group's launches ((2 FETCH_SIZE + WRITE_SIZE) KB, rocprofv3 PMC); "
                    "= per launch when the group is one kernel launched once per step; traffic_over_alg divides by the "
                    + (f"algorithmic bytes at the PMC window's own nefc {win['nefc_mean']:.2f} / ncon {win['ncon_mean']:.2f}"
                       if win else "trace pass's algorithmic bytes (the PMC summary records no window)"),
    "kernel": " + ".join(d["kernels"]),
    "group": dom,
    "kernel_ms": d["ms_per_step"],
    "worlds_per_launch": nworld,
    "alg_bytes_per_env_step": d["alg_bytes_per_env_step"],
    "groups": rec,
    "kernels": tab,
    "step_alg_bytes_per_env_step": sum(v for v in (x["alg_bytes_per_env_step"] for x in rec.values()) if v),
  }


def _tensors(obj, prefix=""):
  """(name, tensor) of every torch tensor reachable from a Data container (Contact / Constraint nested)."""
  import torch

  for k, v in vars(obj).items():
    if isinstance(v, torch.Tensor):
      yield prefix + k, v
    elif hasattr(v, "__dict__") and type(v).__name__ in ("Contact", "Constraint"):
      yield from _tensors(v, prefix + k + ".")


def snapshot(d):
  """Copy of every Data tensor (state, pools, solver warmstart, the world-order histogram ...)."""
  return {k: v.clone() for k, v in _tensors(d)}


def restore(d, saved):
  """Write a snapshot back in place (the captured graph keeps its pointers)."""
  for k, v in _tensors(d):
    v.copy_(saved[k])


def _free_port():
  import socket

  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  port = s.getsockname()[1]
  s.close()
  return port


def launch_ranks(nranks):
  """`bench.py --gpus N` run directly: this parent never touches HIP; it starts N ranks through
  torch.distributed.run (one process per GPU) as a child and exits with its status."""
  import subprocess

  env = dict(os.environ)
  env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
  cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
         "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
  return subprocess.call(cmd, env=env)


def main():
  args = parse()
  if "WORLD_SIZE" not in os.environ and args.gpus > 1:
    sys.exit(launch_ranks(args.gpus))

  import torch
  import torch.distributed as dist

  import mujoco_warp_amd as mjw
  from mujoco_warp_amd import mjcf
  from mujoco_warp_amd.shard import strong_shard, weak_shard

  rank = int(os.environ.get("RANK", "0"))
  world = int(os.environ.get("WORLD_SIZE", "1"))
  local = int(os.environ.get("LOCAL_RANK", "0"))
  if world != args.gpus:
    raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
  if world > 1:
    # the barrier and the max/sum of scalars go over gloo (host); the data path has no collective
    dist.init_process_group("gloo")
  # one rank per GPU; more ranks than devices (a rehearsal on a 1-GPU box) share them round-robin
  ndev = torch.cuda.device_count()
  if ndev == 0:
    raise SystemExit("bench.py needs a ROCm device")
  dev = torch.device("cuda", local % ndev)
  torch.cuda.set_device(dev)

  if args.scaling == "weak":
    offset, nworld = weak_shard(args.nworld, rank)
  else:
    offset, nworld = strong_shard(args.nworld, rank, world)

  cfg = MODELS[args.model]
  mjm = mjcf.load_model(os.path.join(ROOT, cfg["path"]))
  if args.solver is not None:
    mjw.override_model(mjm, [f"opt.solver={args.solver}"])
  solver_name = {1: "CG", 2: "NEWTON"}[int(mjm.opt.solver)]
  mjd = mjcf.MjData(mjm)
  center = None
  if cfg["key"] is not None:  # testspeed: keyframe state, ctrl noise around the keyframe ctrl
    mjcf.reset_data_keyframe(mjm, mjd, cfg["key"])
    center = torch.as_tensor(np.asarray(mjm.key_ctrl[cfg["key"]], dtype=np.float32), device=dev)
  m = mjw.put_model(mjm, device=dev)
  # the rank's worlds run as `--streams` independent shards (own Data, own HIP stream, world ids
  # offset like ranks), so one shard's launch tail overlaps the other's next kernels; nothing
  # synchronises the shards inside the timed region
  nshard = max(1, min(args.streams, nworld))
  shards = []
  for k in range(nshard):
    soff, scnt = strong_shard(nworld, k, nshard)
    dk = mjw.put_data(mjm, mjd, nworld=scnt, nconmax=args.nconmax, njmax=args.njmax, device=dev, m=m)
    dk.world_offset = offset + soff
    shards.append(dk)
  # one batch runs on the current stream; shards each get a stream of their own (not the legacy
  # default stream, which would synchronise with the others)
  streams = [torch.cuda.current_stream(dev)] if nshard == 1 else [torch.cuda.Stream(device=dev) for _ in range(nshard)]

  from mujoco_warp_amd.forward import StepTracer

  graphs = None
  tracer = StepTracer()

  def one_step(i, traced=False):
    for k, (dk, st) in enumerate(zip(shards, streams)):
      with torch.cuda.stream(st):
        mjw.ctrl_noise(m, dk, i, center=center)
        if traced and k == 0:
          tracer.step(m, dk)  # shard 0's kernels are the timed launches
        elif graphs is not None:
          graphs[k].replay()
        else:
          mjw.step(m, dk)

  graph_error = None

  def capture():
    # benchmark.py:123-155 captures fn(m, d) once and replays it every step; should the capture fail,
    # the steps run eagerly and the record says why.  Capture does not execute: the state is unchanged.
    nonlocal graphs, graph_error
    try:
      graphs = []
      for dk in shards:
        cs = torch.cuda.Stream(device=dev)
        cs.wait_stream(torch.cuda.current_stream(dev))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cs):
          mjw.step(m, dk)
        graphs.append(g)
    except RuntimeError as e:
      graphs, graph_error = None, str(e)[:200]
    torch.cuda.synchronize()

  # warmup: the first step eagerly (loads the kernels), then the graph is captured and the remaining
  # warmup steps already replay it, so the timed region starts on a warm graph
  for i in range(args.warmup):
    if i == 1 and args.graph:
      capture()
    one_step(i)
  torch.cuda.synchronize()
  if args.graph and graphs is None and graph_error is None:
    capture()

  def sizes():
    nefc = sum(float(dk.nefc.float().sum()) for dk in shards) / nworld
    ncon = sum(float(dk.nacon[0]) for dk in shards) / nworld
    return nefc, ncon

  # the timed region: K graph replays (or K eager steps when capture failed), nothing else
  nefc_t0, ncon_t0 = sizes()
  saved = [snapshot(dk) for dk in shards]  # the state the timed window starts from (restored for the trace)
  torch.cuda.synchronize()
  if world > 1:
    dist.barrier()
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for i in range(args.steps):
    one_step(args.warmup + i)
  torch.cuda.synchronize()
  if world > 1:
    dist.barrier()
  elapsed = time.perf_counter() - t0
  nefc_t1, ncon_t1 = sizes()
  qpos_all = torch.cat([dk.qpos for dk in shards])
  qpos_timed = qpos_all.clone()
  # per-kernel durations over the timed window itself: restore the saved state and run the first `ntrace`
  # timed steps again eagerly with one HIP event after every kernel launch (mjw_step_trace); every world is
  # computed by one wave from its own data, so these are the timed steps' kernels, with the same nefc /
  # ncon, which the algorithmic bytes of `roofline` are priced at (mean over the traced steps)
  ntrace = args.steps if args.trace_steps <= 0 else min(args.trace_steps, args.steps)
  for dk, sv in zip(shards, saved):
    restore(dk, sv)
  del saved
  acc = torch.zeros(2, dtype=torch.float64, device=dev)
  for i in range(ntrace):
    one_step(args.warmup + i, traced=True)
    acc[0] += shards[0].nefc.sum()
    acc[1] += shards[0].nacon[0]
  torch.cuda.synchronize()
  tab = kernel_table(tracer.durations(), bool(m.is_sparse))
  nefc_mean, ncon_mean = (float(x) / (ntrace * shards[0].nworld) for x in acc.cpu())
  trace_sum = sum(e["ms_per_step"] for e in tab.values())
  # a full re-run of the window ends in the timed run's state, bitwise (the replay of the same work)
  replay_bitwise = bool(torch.equal(shards[0].qpos, qpos_timed[: shards[0].nworld])) if ntrace == args.steps else None
  converged = int((~torch.isnan(qpos_all).any(dim=1)).sum())
  solver_niter_mean = float(torch.cat([dk.solver_niter for dk in shards]).float().mean())
  solver_niter_max = int(torch.cat([dk.solver_niter for dk in shards]).max())
  if args.dump_qpos:
    os.makedirs(args.dump_qpos, exist_ok=True)
    np.savez(os.path.join(args.dump_qpos, f"qpos_rank{rank}.npz"), qpos=qpos_all.cpu().numpy(), offset=offset)
  d = shards[0]

  total_worlds = nworld
  if world > 1:
    names = sorted(tab)
    t = torch.tensor([elapsed] + [tab[k]["ms_per_step"] for k in names], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0])
    for k, v in zip(names, t[1:]):
      tab[k]["ms_per_step"] = float(v)
    c = torch.tensor([converged, nworld], dtype=torch.int64)
    dist.all_reduce(c)
    converged, total_worlds = int(c[0]), int(c[1])

  value = total_worlds * args.steps / elapsed
  if rank == 0:
    words = step_words(mjm, m.nv_pad, bool(m.is_sparse))
    # a sparse efc row carries njrow values + njrow column indices instead of an nv_pad dense row
    groups_alg = b_alg_groups(mjm, words, nefc_mean, ncon_mean, 2 * m.njrow if m.is_sparse else m.nv_pad, bool(m.is_sparse))
    # worlds per timed launch: shard 0's
    nlaunch = d.nworld
    pmc, pmc_src = None, "no PMC summary"
    for path in args.pmc:
      pmc, pmc_src = pmc_traffic(path, args.model, nlaunch, solver_name)
      if pmc is not None:
        break
    row_w = 2 * m.njrow if m.is_sparse else m.nv_pad
    roof = roofline_record(tab, groups_alg, nlaunch, pmc, pmc_src,
                           lambda ne, nc: b_alg_groups(mjm, words, ne, nc, row_w, bool(m.is_sparse)))
    if args.scaling == "weak":
      parallelism = f"{args.nworld} worlds per rank on {world} GPU(s) (weak), no collective"
    else:
      parallelism = f"{args.nworld} worlds split over {world} GPU(s) (strong), no collective"
    parallelism += f"; {nshard} stream shard(s) per rank"
    out = {
      "metric": METRIC if args.model == "humanoid" else f"env-steps/sec (whole node), {args.model} nworld={args.nworld} per GPU",
      "value": value,
      "unit": "env-steps/s",
      "n_gpus": world,
      "steps": args.steps,
      "warmup": args.warmup,
      "ms_per_step": elapsed / args.steps * 1e3,
      "higher_is_better": True,
      "scaling": args.scaling,
      "vs_baseline": None,
      "dtype": "fp32",
      "data": "synthetic (keyframe state + OU/Halton ctrl noise of benchmark.py, no dataset)",
      "config": {
        "workload": f"{os.path.basename(cfg['path'])} ({args.model}) nworld={args.nworld} "
        f"{'per GPU' if args.scaling == 'weak' else 'total'} fp32, "
        f"{['Euler', 'RK4', 'implicit', 'implicitfast'][int(mjm.opt.integrator)]}+{solver_name}, 1xMI355X per rank",
        "nworld_per_gpu": nworld,
        "nworld_total": total_worlds,
        "nconmax": args.nconmax,
        "njmax": args.njmax,
        "solver": solver_name,
        "parallelism": parallelism,
        "graph": graphs is not None,
        **({"graph_error": graph_error} if graph_error else {}),
        "timed_region": "graph replays only" if graphs is not None else "eager steps (no graph)",
        "trace_steps": ntrace,
        "trace_window": "the timed steps themselves: state restored to the timed region's start, steps "
                        f"{args.warmup}..{args.warmup + ntrace - 1} re-run eagerly with HIP events per launch",
        "trace_kernel_sum_ms_per_step": trace_sum,
        "trace_over_timed": trace_sum / (elapsed / args.steps * 1e3),
        "trace_consistent": trace_sum <= 1.03 * (elapsed / args.steps * 1e3),
        "trace_replay_bitwise": replay_bitwise,
        "converged_worlds": converged,
        "nefc_mean": nefc_mean,
        "ncon_mean": ncon_mean,
        "nefc_ncon_window": "mean over the traced (= timed) steps; timed region start / end: "
                            f"nefc {nefc_t0:.2f} / {nefc_t1:.2f}, ncon {ncon_t0:.2f} / {ncon_t1:.2f}",
        "solver_niter_mean": solver_niter_mean,
        "solver_niter_max": solver_niter_max,
        "streams": nshard,
      },
      "roofline": roof,
      "cpu_baseline": None,
    }
    if world == 1 and args.cpu_baseline:
      out["cpu_baseline"] = cpu_baseline(mjm, args.cpu_worlds, args.cpu_steps, cfg["key"], args.njmax, args.nconmax, args.model)
    print(json.dumps(out), flush=True)
  if world > 1:
    dist.destroy_process_group()


if __name__ == "__main__":
  main()
