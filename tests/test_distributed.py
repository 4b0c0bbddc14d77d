"""Multi-process (gloo, world_size=2) checks of the sharding used by bench.py --gpus N."""

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from mujoco_warp_amd.shard import strong_shard, weak_shard


def test_shard_ranges_cover_exactly():
  for total in (1, 7, 8192, 8193):
    for n in (1, 2, 3, 8):
      seen = []
      for r in range(n):
        off, cnt = strong_shard(total, r, n)
        seen += list(range(off, off + cnt))
      assert seen == list(range(total))
  assert weak_shard(8192, 3) == (3 * 8192, 8192)


def _free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _worker(rank, nranks, port, q):
  import torch

  from oracle import orc
  from tests.common import humanoid_model

  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  dist.init_process_group("gloo", rank=rank, world_size=nranks)
  mjm = humanoid_model()
  nper = 3
  off, cnt = weak_shard(nper, rank)
  om = orc.OracleModel(mjm)
  od = orc.OracleData(om, cnt, 64, 24)
  od.qpos[:] = mjm.key_qpos[0]
  for i in range(4):
    od.ctrl_noise(i, center=np.zeros(mjm.nu), world_offset=off)
    od.step()
  local = torch.tensor(np.concatenate([od.ctrl.reshape(-1), od.qpos.reshape(-1)]))
  gathered = [torch.zeros_like(local) for _ in range(nranks)]
  dist.all_gather(gathered, local)
  t = torch.tensor([float(rank + 1)])
  dist.all_reduce(t, op=dist.ReduceOp.MAX)
  if rank == 0:
    q.put((torch.stack(gathered).numpy(), float(t[0])))
  dist.destroy_process_group()


def test_sharded_rollout_equals_single_process():
  from oracle import orc
  from tests.common import humanoid_model

  nranks, nper = 2, 3
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_worker, args=(r, nranks, port, q)) for r in range(nranks)]
  for p in procs:
    p.start()
  gathered, tmax = q.get(timeout=300)
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  assert tmax == 2.0
  # single process over all 6 worlds with global ids
  mjm = humanoid_model()
  om = orc.OracleModel(mjm)
  od = orc.OracleData(om, nranks * nper, 64, 24)
  od.qpos[:] = mjm.key_qpos[0]
  for i in range(4):
    od.ctrl_noise(i, center=np.zeros(mjm.nu))
    od.step()
  for r in range(nranks):
    n = nper * mjm.nu
    ctrl = gathered[r][:n].reshape(nper, mjm.nu)
    qpos = gathered[r][n:].reshape(nper, mjm.nq)
    np.testing.assert_array_equal(ctrl, od.ctrl[r * nper:(r + 1) * nper])
    np.testing.assert_array_equal(qpos, od.qpos[r * nper:(r + 1) * nper])
