"""bench.py --gpus N runs N ranks or refuses (the driver's SCALE runs time exactly what they report).

* Without torch.distributed.run, ``bench.py --gpus 2`` launches ``torch.distributed.run --nproc-per-node 2``
  as a child process; here the ranks run the host build of the kernel body over gloo
  (``--rehearse-on-host``), end to end: sharding, timing max / decision sum, parity reduction, rank-0 line.
* Under a launcher whose WORLD_SIZE differs from --gpus, every rank refuses.
* With fewer visible GPUs than --gpus (none here), the launcher refuses before starting anything.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "SFL_DIST_BACKEND", "SFL_DEVICE")}
    env.update(kw)
    return env


def _bench(args, env, timeout=300):
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_2_launches_two_ranks_end_to_end():
    r = _bench(["--gpus", "2", "--rehearse-on-host", "--config", "c2", "--envs", "4", "--decisions", "32",
                "--steps", "2", "--warmup", "1", "--verify-envs", "2"], _env(OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "launching" in r.stderr and "--nproc-per-node=2" in r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    # stdout is the JSON line and nothing else (gloo's / RCCL's own prints go to stderr, bench.json_stdout)
    assert r.stdout.strip().splitlines() == lines, r.stdout[:2000]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["world_size"] == 2 and res["backend"] == "gloo"
    assert res["devices"] == [-1, -1]
    assert res["config"]["parallelism"] == "env-batch dp2"
    assert res["parity"] == "ok" and res["parity_envs_checked"] == 4, res
    assert "rehearsal" in res and res["roofline"] is None
    assert res["partition_leg"]["parity"] == "ok" and res["partition_leg"]["world_size"] == 2
    # every rank's decisions are in the job's total: 2 ranks x 4 envs x 32 decisions x 2 timed steps
    assert abs(res["value"] * res["ms_per_step"] * 1e-3 * res["steps"] - 2 * 4 * 32 * 2) < 1e-6 * res["value"] + 1


def test_gpus_4_host_rehearsal_runs_the_partitioned_leg():
    """The driver's SCALE runs (--gpus N > 1) carry configs[4]'s partitioned leg on the same ranks.  Rehearsed
    here on four host-build ranks over gloo end to end: the env-sharded line plus the leg, whose owned Q rows and
    env states are checked against a fused host run (parity ok), with one message exchange and one reply
    exchange per round."""
    env = _env()
    env.pop("OMP_NUM_THREADS", None)  # (the ranks bound their host-build threads themselves)
    r = _bench(["--gpus", "4", "--rehearse-on-host", "--config", "c2", "--envs", "4", "--decisions", "32",
                "--steps", "2", "--warmup", "1", "--verify-envs", "2"], env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["world_size"] == 4 and res["parity"] == "ok"
    # the host-build parity check of each rank runs on its share of the granted cores, not one thread per core
    cores, quota = len(os.sched_getaffinity(0)), None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else int(q) / int(per)
    except OSError:
        pass
    granted = max(1, min(cores, int(quota)) if quota else cores)
    assert res["parity_threads_per_rank"] == max(1, granted // 4), res["parity_reference"]
    leg = res["partition_leg"]
    assert "error" not in leg, leg
    assert leg["world_size"] == 4 and leg["backend"] == "gloo" and leg["parity"] == "ok", leg
    assert leg["parity_envs_checked"] >= 8 and leg["collectives_per_round"] == 2 and "rehearsal" in leg
    assert leg["rounds_per_step"] >= 25  # (the host build's local step sends every row: decisions + 1 rounds)


def test_gpus_2_host_rehearsal_partition_with_cohorts():
    """bench.py --partition --cohorts 2 on two host-build ranks over gloo: each rank's envs as two cohort jobs
    (a process group each), owned rows and env states of the sampled envs checked against a fused host run."""
    r = _bench(["--gpus", "2", "--rehearse-on-host", "--partition", "--cohorts", "2", "--config", "c5", "--envs", "4",
                "--decisions", "24", "--steps", "1", "--warmup", "1", "--verify-envs", "4"], _env(OMP_NUM_THREADS="2"),
               timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["world_size"] == 2 and res["config"]["cohorts"] == 2, res
    # (each rank checks its owned rows of the job's sampled envs: parity.spread(8, 4) = 3 envs, on 2 ranks)
    assert res["parity"] == "ok" and res["parity_envs_checked"] == 6, res
    assert res["config"]["rounds_per_step"] == 25  # (the host build sends every row: decisions + 1 rounds)


def test_world_size_other_than_gpus_is_refused():
    r = _bench(["--gpus", "3", "--steps", "1"], _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), timeout=60)
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 3" in r.stderr
    assert not r.stdout.strip()


def test_too_few_gpus_is_refused_before_launch():
    r = _bench(["--gpus", "2", "--steps", "1"], _env(HIP_VISIBLE_DEVICES=""), timeout=60)
    assert r.returncode == 2
    assert "needs 2 visible GPUs, found 0" in r.stderr
    assert "launching" not in r.stderr and not r.stdout.strip()


def test_ranks_refuse_without_devices():
    # under torch.distributed.run with RCCL: a node with fewer GPUs than ranks refuses on every rank
    r = _bench(["--gpus", "2", "--steps", "1"],
               _env(WORLD_SIZE="2", LOCAL_WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", HIP_VISIBLE_DEVICES=""),
               timeout=60)
    assert r.returncode == 2
    assert "2 ranks on this node need 2 visible GPUs, found 0" in r.stderr
