"""world_size-2 gloo run of the env-sharded path (host build of the kernel body): the union of the
ranks' envs gives exactly the single-process result (envs are independent; no data-path collective)."""
import importlib
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from tests import hostsim

HP = dict(gamma=1.0, epsilon=0.5, epsilon_decay_rate=0.9997, lr=0.1, lr_decay_rate=1.0, default_q=0.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    par = importlib.import_module("network-distributed-q-learning_amd.parallel")
    mapgen = importlib.import_module("network-distributed-q-learning_amd.mapgen")
    comp = importlib.import_module("network-distributed-q-learning_amd.compiler")
    runtime = importlib.import_module("network-distributed-q-learning_amd.runtime")
    dist = par.init("gloo")
    cm = comp.compile_scenario(mapgen.make_config("c2"))
    b = runtime.Batch(cm, HP, par.shard_seeds(450565, 3, rank), lib=hostsim.lib(), ntab=4096)
    b.learn_begin()
    b.apply_qinit()
    n, _ = b.step(120)
    dt, total = par.reduce_timing(dist, 1.0 + rank, n)
    q = [b.q_raw(e)[0].sum() for e in range(3)]
    allq = par.gather_env_stats(dist, np.array(q))
    if rank == 0:
        qout.put((dt, total, allq.tolist()))
    dist.barrier()
    dist.destroy_process_group()


qout = None


def test_two_rank_sharding_matches_single_process():
    global qout
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    dt, total, allq = res
    assert dt == 2.0 and total == 2 * 3 * 120
    mapgen = importlib.import_module("network-distributed-q-learning_amd.mapgen")
    comp = importlib.import_module("network-distributed-q-learning_amd.compiler")
    runtime = importlib.import_module("network-distributed-q-learning_amd.runtime")
    cm = comp.compile_scenario(mapgen.make_config("c2"))
    b = runtime.Batch(cm, HP, [450565 + i for i in range(6)], lib=hostsim.lib(), ntab=4096)
    b.learn_begin()
    b.apply_qinit()
    b.step(120)
    assert allq == [b.q_raw(e)[0].sum() for e in range(6)]


def _run(rank, world, port, q):
    global qout
    qout = q
    _worker(rank, world, port, q)
