"""Benchmark: agent-env-steps/sec of the SwitchFL + network-distributed-Q hot path on MI355X.

Workload (BASELINE.json configs[2]): the 64-switch / 32-train map, 65,536 lock-step envs per GPU,
learning mode (epsilon-greedy, Q updates) with the hyper-parameters of test_model.py:56-63 and
malfunctions at rate 0.01 (5-15 ticks, test_model.py:14-18).  A *step* = every env advances by
``--decisions`` agent-env-steps (one iteration of distr_q.py:302-362 each, with every Flatland
tick in between and episodes restarting as they end).  N GPUs: one process per GPU, each with its
own 65,536 envs (weak scaling, no collective on the data path; the reference's parallelism is an
embarrassingly parallel seed sweep, hyperparam_tuning.py:85-91).

Usage: python bench.py [--gpus N --steps K --warmup W].  N > 1 runs one rank per GPU: under
torch.distributed.run (the driver's launch) every rank checks WORLD_SIZE == N and that N devices are
visible; started without it, bench.py launches ``torch.distributed.run --nproc-per-node N`` itself as a
child process (before any HIP call) and exits with its return code.
"""
from __future__ import annotations

import argparse
import glob
import importlib
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = "network-distributed-q-learning_amd"

HP = dict(gamma=1.0, epsilon=0.5, epsilon_decay_rate=0.9997, lr=0.1, lr_decay_rate=1.0, default_q=0.0)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "agent-env-steps/sec (whole node), 64-switch map, 1/2/4/8 MI355X vs CPU"


def host_cores():
    """(affinity core count, cgroup CPU quota in cores or None) of this process."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except Exception:
        pass
    return n, quota


def _cxx_rate(cm, lib, threads: int, seconds: float):
    """agent-env-steps/s of the host build on `threads` OpenMP threads, 8 envs per thread."""
    import ctypes
    runtime = importlib.import_module(PKG + ".runtime")
    threads = lib.dll.sflh_set_threads(ctypes.c_int(threads))
    E = 8 * threads
    b = runtime.Batch(cm, HP, [450565 + i for i in range(E)], lib=lib)
    b.learn_begin()
    b.apply_qinit()
    b.step(64)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        n += b.step(64)[0]
    dt = time.perf_counter() - t0
    b.close()
    return n / dt, threads, E, n, dt


def cpu_baseline(cm, seconds: float, config: str = "c3"):
    """BASELINE.md / SURVEY.md §8(d): the build's C++ CPU backend -- the same kernel body compiled for
    the host (libsfl_hostsim.so, OpenMP, one env per thread at a time) -- on ALL host cores of this
    box (os.sched_getaffinity), 8 envs per core, same map, seeds and hyper-parameters, learning mode.
    When a cgroup CPU quota grants fewer cores than the affinity mask lists (the GPU box: 16 of the
    machine's cores), one thread per granted core is timed too and the faster of the two is reported,
    both in `sample`.  The reference loop itself cannot run here (flatland-rl is absent): a "port"."""
    import ctypes
    build = importlib.import_module(PKG + ".build")
    _lib = importlib.import_module(PKG + "._lib")
    cores, quota = host_cores()
    lib = _lib.Lib(build.build_hostsim())
    lib.check_fresh()
    lib.dll.sflh_set_threads.restype = ctypes.c_int
    runs = []
    if quota and int(quota + 0.999) < cores:
        runs.append(_cxx_rate(cm, lib, int(quota + 0.999), seconds * 2 / 3))
        runs.append(_cxx_rate(cm, lib, cores, seconds / 3))
    else:
        runs.append(_cxx_rate(cm, lib, cores, seconds))
    best = max(runs)
    desc = "; ".join(f"{t} threads: {v / 1e6:.3f} M/s ({n} decisions over {E} envs in {dt:.1f} s)"
                     for v, t, E, n, dt in runs)
    q = f", cgroup CPU quota {quota:g} cores" if quota else ""
    return dict(value=best[0], unit="agent-env-steps/sec", cores=best[1], kind="port",
                sample=f"libsfl_hostsim.so (the kernel body built for the host, OpenMP, 8 envs per thread) on the "
                       f"{config} map, seeds 450565+i, os.sched_getaffinity = {cores} cores{q}; {desc}; "
                       f"after one untimed 64-decision step")


def _oracle_worker(job):
    """One host core of the oracle baseline: the oracle's learn loop on one env (seed) for about `seconds`,
    in chunks of 100 decisions.  Runs in a process started before this job touched the GPU."""
    config, seed, seconds, want_q = job
    sys.path.insert(0, REPO)
    from oracle import sfl_oracle as so
    mapgen = importlib.import_module(PKG + ".mapgen")
    sc = mapgen.make_config(config)
    env, model = so.build(sc, seed, HP, trace=False)
    state = None
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        n += 100
        state = so.run_decisions(model, n, state)
    dt = time.perf_counter() - t0
    return n, dt, (dict(model.q) if want_q else None)


def oracle_cores() -> int:
    """Host cores the oracle baseline runs on: the cgroup CPU quota (the GPU box grants 16) or the affinity set."""
    cores, quota = host_cores()
    return max(1, min(cores, int(quota)) if quota else cores)


def _oracle_loop(jobs, results):
    """A fixed oracle worker: one job from `jobs`, its result (or the error) to `results`, then exit."""
    job = jobs.get()
    if job is None:
        return
    try:
        results.put(("ok", job[1], _oracle_worker(job)))
    except BaseException as ex:  # noqa: BLE001 -- reported on the line
        results.put(("error", job[1], repr(ex)))


class OraclePool:
    """The oracle baseline's worker processes: a FIXED set, started BEFORE any HIP call of this process (a process
    that has initialised the GPU must not start programs: spawn = fork + exec).  Nothing ever replaces a worker --
    unlike multiprocessing.Pool, whose handler thread respawns a dead worker (a fork + exec from a GPU-initialised
    process) and whose map() waits forever for a lost task.  A worker that dies makes `map` raise."""

    def __init__(self, n: int):
        import multiprocessing as mp
        ctx = mp.get_context("spawn")
        self.jobs, self.results = ctx.Queue(), ctx.Queue()
        self.procs = [ctx.Process(target=_oracle_loop, args=(self.jobs, self.results), daemon=True) for _ in range(n)]
        for p in self.procs:
            p.start()
        self._processes = n
        self.used = False

    def map(self, jobs, timeout: float):
        import queue
        assert not self.used and len(jobs) <= len(self.procs)
        self.used = True
        for j in jobs:
            self.jobs.put(j)
        for _ in range(len(self.procs) - len(jobs)):
            self.jobs.put(None)
        out, deadline = {}, time.monotonic() + timeout
        while len(out) < len(jobs):
            try:
                kind, seed, r = self.results.get(timeout=1.0)
            except queue.Empty:
                if time.monotonic() > deadline:
                    raise RuntimeError(f"oracle baseline: no result from {len(jobs) - len(out)} worker(s) in {timeout:.0f} s")
                if any(p.exitcode not in (None, 0) for p in self.procs):
                    raise RuntimeError("oracle baseline: a worker process died without a result "
                                       f"(exit codes {[p.exitcode for p in self.procs]})")
                continue
            if kind != "ok":
                raise RuntimeError(f"oracle baseline: worker for seed {seed} failed: {r}")
            out[seed] = r
        return [out[j[1]] for j in jobs]

    def close(self):
        if not self.used:
            for _ in self.procs:
                self.jobs.put(None)
            self.used = True
        deadline = time.monotonic() + 30.0  # (one budget for all: a worker may be stuck behind a dead one's queue lock)
        for p in self.procs:
            p.join(timeout=max(0.0, deadline - time.monotonic()))
        for p in self.procs:
            if p.exitcode is None:
                p.kill()  # (this pool's own child, by its handle)
                p.join(timeout=5)

    def join(self):
        pass


def start_oracle_pool(n: int):
    return OraclePool(n)


def cpu_oracle_baseline(config: str, seconds: float, pool=None, check=None):
    """The reference-speed CPU baseline: the CPU oracle (pure-Python restatement of the reference loop,
    the reference's own speed class) as one process per granted host core, one env each -- the analogue of
    the reference's scale-out, one process per seed (hyperparam_tuning.py:85-91).  value = decisions of all
    processes / the longest process time.  check = (cm, device, group_lanes): afterwards the product kernel runs
    process 0's env (seed, map, hyper-parameters) for the same decisions at the bench's group size, and its
    Q-table must equal the oracle's (the reference's q_table dict) -- the bench line's own oracle parity on
    exactly the sample it timed."""
    jobs = [(config, 450565 + i, seconds, i == 0) for i in range(pool._processes if pool is not None else 1)]
    res = pool.map(jobs, timeout=4 * seconds + 120) if pool is not None else [_oracle_worker(jobs[0])]
    n_all = sum(r[0] for r in res)
    dt_max = max(r[1] for r in res)
    n0, dt0, q0 = res[0]
    out = dict(value=n_all / dt_max, unit="agent-env-steps/sec", cores=len(res), kind="port",
               sample=f"oracle/sfl_oracle.py learn loop, {len(res)} process(es) (one per granted host core), one env "
                      f"each (seeds 450565+i) of the {config} map, {n_all} decisions in {dt_max:.1f} s (from episode "
                      f"start, incl. the Q-table init); 1 core: {n0 / dt0:.4g} agent-env-steps/s ({n0} decisions in "
                      f"{dt0:.1f} s)",
               one_core_value=n0 / dt0)
    if check is not None:
        cm, device, g = check
        runtime = importlib.import_module(PKG + ".runtime")
        old = os.environ.get("SFL_WAVE_G")
        os.environ["SFL_WAVE_G"] = str(g)  # (the bench kernel's shape, not the one-env batch's default)
        try:
            b = runtime.Batch(cm, HP, [450565], device=device)
        finally:
            if old is None:
                os.environ.pop("SFL_WAVE_G", None)
            else:
                os.environ["SFL_WAVE_G"] = old
        try:
            b.learn_begin()
            b.apply_qinit()
            b.step(n0)
            c = b.counters()
            same = b.q_dict(0) == q0
            out["oracle_parity"] = {
                "result": "ok" if same else "FAIL",
                "what": f"the product kernel (k_wave variant {c['kernel_variant']}, {c['group_lanes']} lanes per env) on "
                        f"process 0's env for the same {n0} decisions: Q-table (the reference's q_table dict) equal "
                        "to the oracle's" + ("" if same else " -- it is not")}
        finally:
            b.close()
    return out


JSON_OUT = [sys.stdout]


def json_stdout():
    """Keep stdout for the one JSON line: from here on everything else written to file descriptor 1 -- RCCL's version
    banner at communicator set-up, gloo's connection lines, library or Python prints -- goes to stderr, and the
    line is written to a duplicate of the original stdout (JSON_OUT)."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    JSON_OUT[0] = os.fdopen(fd, "w", buffering=1)


def visible_gpus() -> int:
    """GPUs this process may use, counted without any HIP call: the KFD topology's GPU nodes (gpu_id != 0),
    restricted by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set."""
    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
        try:
            n += int(open(f).read().strip() or "0") != 0
        except (OSError, ValueError):
            pass
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def rehearsal() -> bool:
    """SFL_DIST_BACKEND=gloo: the multi-rank path rehearsed with several ranks sharing one device (or the host
    build): the launcher, sharding and reductions, not the RCCL transport."""
    return os.environ.get("SFL_DIST_BACKEND", "nccl") != "nccl"


def launch_or_check(args, argv) -> int | None:
    """The contract's --gpus N (the reference's scale-out is N independent processes,
    hyperparam_tuning.py:85-91).  Outside torch.distributed.run with N > 1: launch N ranks as a child
    ``torch.distributed.run`` (never exec: this process has not touched the GPU, and the child is a new
    process) and return its exit code.  Inside it: return 2 unless WORLD_SIZE == N and, for RCCL, N devices
    are visible.  None: go on in this process."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        if args.gpus <= 1:
            return None
        if not rehearsal() and not args.rehearse_on_host and visible_gpus() < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {visible_gpus()}; refusing to "
                  f"time fewer (SFL_DIST_BACKEND=gloo rehearses several ranks on one device)", file=sys.stderr)
            return 2
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
        print("bench.py: launching " + " ".join(cmd[1:]), file=sys.stderr, flush=True)
        return subprocess.run(cmd).returncode
    if int(ws) != args.gpus:
        print(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}: the job would report a different GPU count than "
              f"it runs on; refusing", file=sys.stderr)
        return 2
    if not rehearsal() and not args.rehearse_on_host:
        local_ws = int(os.environ.get("LOCAL_WORLD_SIZE", ws))
        if visible_gpus() < local_ws:
            print(f"bench.py: {local_ws} ranks on this node need {local_ws} visible GPUs, found {visible_gpus()}; "
                  f"refusing", file=sys.stderr)
            return 2
    return None


def dist_setup(par, local: int, host: bool = False):
    """torch.distributed for the bench: RCCL ("nccl") over the GPUs of the node, one per rank.
    SFL_DIST_BACKEND=gloo and SFL_DEVICE=<index> rehearse the multi-rank path with several ranks
    on one GPU (the launcher, sharding and reductions; not the RCCL transport).  ``host``: the
    --rehearse-on-host run (gloo, no device)."""
    backend = "gloo" if host else os.environ.get("SFL_DIST_BACKEND", "nccl")
    dev = int(os.environ.get("SFL_DEVICE", local))
    dist = par.init(backend)
    return dist, dev, ("cuda" if backend == "nccl" else "cpu")


def rank_devices(dist, dev: int, device=None):
    """The device index of every rank, in rank order."""
    if dist is None:
        return [dev]
    import torch
    t = torch.tensor([dev], dtype=torch.int64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [int(p.item()) for p in parts]


def pmc_profile(lib, workload: str):
    """The committed rocprofv3 PMC summary (profiles/*_pmc.json, scripts/pmc_summary.py) of exactly this
    library build (build id: sources + defines + flags) and workload, as (dict, path), or (None, None).
    An experiment build never matches a product profile."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("build_id", d.get("source_sha1")) == lib.build_id and d.get("workload") == workload:
            return d, os.path.relpath(f, REPO)
    return None, None


def library_info(lib):
    return {"file": os.path.relpath(lib.path, REPO), "build_id": lib.build_id, "defines": lib.defines,
            "flags": lib.flags,
            "experimental": bool(lib.experimental)}


def issue_bound(prof):
    """The binding bound of the env kernel from its PMC profile: the fraction of SIMD issue capacity its
    vector instructions use (SQ_ACTIVE_INST_VALU quad-cycles over the SIMDs' wave-cycle budget), the
    fraction of wave time spent waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES) and the VALU lane utilisation."""
    if not prof:
        return None
    med = prof.get("per_launch_median", {})
    out = {}
    if "SQ_WAVE_CYCLES" in med and "SQ_WAIT_ANY" in med:
        out["wait_frac"] = med["SQ_WAIT_ANY"] / med["SQ_WAVE_CYCLES"]
    if "SQ_WAVE_CYCLES" in med and "SQ_ACTIVE_INST_ANY" in med:
        out["active_frac"] = med["SQ_ACTIVE_INST_ANY"] / med["SQ_WAVE_CYCLES"]
    if "SQ_THREAD_CYCLES_VALU" in med and "SQ_ACTIVE_INST_VALU" in med:
        out["valu_lane_util"] = med["SQ_THREAD_CYCLES_VALU"] / (64.0 * med["SQ_ACTIVE_INST_VALU"])
    for k in ("valu_issue_frac", "occupancy_waves_per_simd"):
        if k in prof:
            out[k] = prof[k]
    return out or None


def verify_threads() -> int:
    """OpenMP threads of this rank's host-build parity check: the granted cores (cgroup quota, else the affinity
    set) shared by the ranks of this node.  Without it libgomp starts one thread per affinity core -- 256 on the
    GPU box, whose quota is 16 cores -- in every rank."""
    cores, quota = host_cores()
    granted = max(1, min(cores, int(quota)) if quota else cores)
    return max(1, granted // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1"))))


def host_verifier():
    """The host build of the kernel body, with verify_threads() OpenMP threads: (Lib, threads)."""
    import ctypes
    build = importlib.import_module(PKG + ".build")
    _lib = importlib.import_module(PKG + "._lib")
    host = _lib.Lib(build.build_hostsim())
    host.check_fresh()
    host.dll.sflh_set_threads.restype = ctypes.c_int
    return host, int(host.dll.sflh_set_threads(ctypes.c_int(verify_threads())))


def verify_fused(b, cm, seeds, schedule, n_envs: int):
    """Parity of a spread sample of this rank's envs vs the host build of the kernel body (after timing):
    (envs checked, mismatches, OpenMP threads used)."""
    parity = importlib.import_module(PKG + ".parity")
    host, threads = host_verifier()
    pick = parity.spread(len(seeds), n_envs)
    bad = parity.check_batch(b, HP, pick, schedule, host)
    return len(pick), bad, threads


def parity_field(dist, n_checked: int, bad, device=None, threads: int = 0):
    """Job-wide parity verdict: envs checked and mismatches summed over ranks."""
    par = importlib.import_module(PKG + ".parallel")
    _, n_all = par.reduce_timing(dist, 0.0, float(n_checked), device=device)
    _, nbad = par.reduce_timing(dist, 0.0, float(len(bad)), device=device)
    verdict = ("ok" if nbad == 0 else f"FAIL ({int(nbad)} mismatches)") if n_all > 0 else "not verified"
    return {"parity": verdict,
            "parity_envs_checked": int(n_all),
            "parity_reference": "libsfl_hostsim.so (the kernel body built for the host, pinned to the oracle and "
                                "the reference's golden traces by tests/), same seeds and step schedule, "
                                f"Q-table + key set + env state bit-exact; {threads} OpenMP thread(s) per rank "
                                "(the granted host cores / the ranks of the node)",
            "parity_threads_per_rank": threads,
            "parity_first_mismatches": list(bad[:4])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--decisions", type=int, default=1024, help="agent-env-steps per env per step (one launch)")
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--sustain-seconds", type=float, default=8.0,
                    help="after the parity check, repeat the step for about this long and report the rate as "
                         "'sustained' (0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--verify-envs", type=int, default=32,
                    help="envs per rank re-run on the host build after timing and compared bit-exactly (0: none)")
    ap.add_argument("--experimental", action="store_true",
                    help="accept a tuning / experiment build as SFL_LIB (its defines are reported; SFL_X_* / SFL_AB_* "
                         "builds compute wrong results)")
    ap.add_argument("--remote-rows", action="store_true",
                    help="with --partition: every row operation travels as a message, also those on the rank's own "
                         "switches (the message path measured on one rank)")
    ap.add_argument("--virtual-ranks", type=int, default=0,
                    help="with --partition on one rank: only the switches of block 0 of a V-rank partition are "
                         "decided on in place, the rest travel as messages (a V-rank job's per-GPU traffic, without "
                         "the transfers)")
    ap.add_argument("--cohorts", type=int, default=None,
                    help="--partition: the rank's envs as this many independent partitioned jobs whose rounds are "
                         "issued alternately (partition.CohortPipeline), so one cohort's exchange and owner step "
                         "overlap another's local step (default: %d on one GPU; 1 on the host build and with RCCL at N > 1)"
                         % PARTITION_COHORTS)
    ap.add_argument("--partition", action="store_true",
                    help="graph-partitioned mode (BASELINE configs[4]): switch agents owned by ranks, RCCL all-to-all "
                         "of row lookups and updates; defaults to --config c5 --envs 16384 (238 GB of owned Q rows per GPU)")
    ap.add_argument("--rccl-one-rank", action="store_true",
                    help="--partition on one GPU: the segments still travel as RCCL all-to-alls (a process group of "
                         "one) -- RCCL's cost inside the round, which a single-rank job otherwise skips")
    ap.add_argument("--rehearse-on-host", action="store_true",
                    help="TEST ONLY: run the ranks on the host build of the kernel body (libsfl_hostsim.so, gloo) to "
                         "rehearse the launcher without a GPU; the line says so and is no measurement")
    args = ap.parse_args()
    rc = launch_or_check(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    json_stdout()
    if args.experimental:
        os.environ["SFL_EXPERIMENTAL"] = "1"
    if args.partition:
        return bench_partition(args)

    import torch
    host = args.rehearse_on_host
    par = importlib.import_module(PKG + ".parallel")
    world, rank, local = par.world()
    pool = None
    if world == 1 and not args.no_cpu and not host and not any(k.startswith("ROCPROF") for k in os.environ):
        # (before the first HIP call; never under rocprofv3, whose preload initialises the GPU at start)
        pool = start_oracle_pool(oracle_cores())
    dist, dev, red_dev = dist_setup(par, local, host)
    if not host:
        torch.cuda.set_device(dev)
    devices = rank_devices(dist, -1 if host else dev, device=red_dev)

    mapgen = importlib.import_module(PKG + ".mapgen")
    comp = importlib.import_module(PKG + ".compiler")
    runtime = importlib.import_module(PKG + ".runtime")
    build = importlib.import_module(PKG + ".build")
    if rank == 0:  # (re)build if the library is not from these sources; the other ranks wait for it
        build.build_hostsim() if host else build.build_hip()
    if dist is not None:
        dist.barrier()
    sc = mapgen.make_config(args.config)
    cm = comp.compile_scenario(sc)
    E = args.envs
    seeds = par.shard_seeds(450565, E, rank)
    lib = None
    if host:
        lib, _ = host_verifier()  # (its OpenMP threads bounded like the parity check's)
    b = runtime.Batch(cm, HP, seeds, device=dev, lib=lib)
    b.learn_begin()
    b.apply_qinit()
    for _ in range(args.warmup):
        b.step(args.decisions)

    def barrier():
        if dist is not None:
            dist.barrier()
        if not host:
            torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    total = 0
    kms = 0.0
    abytes = 0
    dec_l = ticks_l = 0
    cnt0 = b.counters()
    kname = (f"k_wave<{cnt0['kernel_variant']}> ({64 // cnt0['group_lanes']} env(s) per wavefront)" if cnt0["kernel_variant"] > 0
             else "k_run (one env per lane)")
    for _ in range(args.steps):
        n, ms = b.step(args.decisions)
        total += n
        kms += ms
        cl = b.counters()
        abytes += cl["last_launch_alg_bytes"]
        dec_l += cl["last_launch_decisions"]
        ticks_l += cl["last_launch_ticks"]
    barrier()
    dt = time.perf_counter() - t0
    dt, total_all = par.reduce_timing(dist, dt, float(total), device=red_dev)
    # after the timed region: a spread sample of every rank's envs re-run on the host build, bit-exact
    checked, bad, vthreads = 0, ["not verified (--verify-envs 0)"], 0
    if args.verify_envs > 0:
        checked, bad, vthreads = verify_fused(b, cm, seeds, [args.decisions] * (args.warmup + args.steps),
                                              args.verify_envs)
    pfield = parity_field(dist, checked, bad, device=red_dev, threads=vthreads)
    # after the parity check: the same step repeated for about --sustain-seconds, timed the same way (barrier +
    # synchronize on both sides, max over ranks) -- the rate over a longer window than the K timed steps, so that
    # a sampler of the GPU's activity around the run sees the kernel running
    sustained = None
    if args.sustain_seconds > 0 and not host and args.steps > 0:
        n_sus = max(1, int(math.ceil(args.sustain_seconds / max(1e-6, dt / args.steps))))
        barrier()
        t1 = time.perf_counter()
        tot_s = 0
        for _ in range(n_sus):
            tot_s += b.step(args.decisions)[0]
        barrier()
        dt_s, tot_s_all = par.reduce_timing(dist, time.perf_counter() - t1, float(tot_s), device=red_dev)
        sustained = {"value": tot_s_all / dt_s, "steps": n_sus, "seconds": dt_s,
                     "what": "the same step repeated after the parity check (not the timed K steps): the rate over a "
                             "longer window"}
    res = None
    if rank == 0:
        avg_ms = kms / max(1, args.steps)
        bytes_per_launch = abytes / max(1, args.steps)
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        workload = (f"{args.config}: {cm.S} switches / {cm.T} trains, {E} envs per GPU, learning "
                    f"(eps-greedy + Q update), {args.decisions} agent-env-steps per env per step")
        prof, prof_src = pmc_profile(b.lib, workload)
        traffic = prof["traffic_bytes_per_launch"] if prof else None
        res = {
            "metric": METRIC,
            "value": total_all / dt,
            "unit": "agent-env-steps/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic {cm.S}-switch/{cm.T}-train Flatland-format map (mapgen {args.config}, seed 450565), "
                    "Q-tables at default_q + the optimistic init",
            "config": {"workload": workload,
                       "envs_per_gpu": E, "decisions_per_env_per_step": args.decisions,
                       "parallelism": f"env-batch dp{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": prof_src,
                         "kernel": kname, "avg_kernel_ms": avg_ms,
                         "alg_bytes_per_launch": bytes_per_launch,
                         "ticks_per_decision": ticks_l / max(1, dec_l),
                         "issue": issue_bound(prof)},
            "library": library_info(b.lib),
            "world_size": world,
            "backend": (dist.get_backend() if dist is not None else None),
            "devices": devices,
            **pfield,
            "sustained": sustained,
        }
        if host:
            res["rehearsal"] = ("--rehearse-on-host: every rank ran the host build of the kernel body; a launcher "
                                "rehearsal, not a GPU measurement")
            res["roofline"] = None
        if world == 1 and not args.no_cpu and not host:
            res["cpu_baseline"] = cpu_baseline(cm, args.cpu_seconds, args.config)
            try:
                res["cpu_oracle_baseline"] = cpu_oracle_baseline(args.config, args.cpu_seconds / 2, pool=pool,
                                                                 check=(cm, dev, cnt0["group_lanes"]))
            except RuntimeError as ex:  # a lost worker: the baseline failed, never replaced or retried
                res["cpu_oracle_baseline"] = {"error": str(ex)}
    if pool is not None:
        pool.close()
    b.close()
    printed = []

    def emit(r):
        if not printed:
            printed.append(1)
            print(json.dumps(r), file=JSON_OUT[0], flush=True)
    if world > 1 and os.environ.get("SFL_NO_PARTITION_LEG") != "1":
        leg = partition_leg(par, dist, world, rank, dev, red_dev, devices, res, emit, host=host)
        if rank == 0:
            res["partition_leg"] = leg
    if rank == 0:
        emit(res)
    if dist is not None:
        dist.destroy_process_group()


def bench_partition(args):
    """configs[4]: the 256-switch map with its switch agents graph-partitioned over the ranks; each rank
    simulates its own envs and owns the Q rows of its switches for every env (weak scaling: envs and owned
    Q bytes per GPU fixed).  A step = every env makes --decisions decisions = decisions + 1 message rounds."""
    import torch
    par = importlib.import_module(PKG + ".parallel")
    world, rank, local = par.world()
    host = args.rehearse_on_host
    dist, dev, red_dev = dist_setup(par, local, host)
    if not host:
        torch.cuda.set_device(dev)
    if getattr(args, "rccl_one_rank", False) and world == 1 and not host:
        # one rank whose segments still travel as RCCL collectives (partition.PartitionedBatch exchange_collective):
        # RCCL's launch and stream costs inside the round, measured on one GPU
        import torch.distributed as tdist
        s_ = socket.socket()
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
        s_.close()
        tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", world_size=1, rank=0)
        dist, red_dev = tdist, "cuda"
    devices = rank_devices(dist, -1 if host else dev, device=red_dev)
    if rank == 0:
        build = importlib.import_module(PKG + ".build")
        build.build_hostsim() if host else build.build_hip()
    if dist is not None:
        dist.barrier()
    res = partition_run(args, par, dist, world, rank, dev, red_dev, devices, host=host)
    if rank == 0:
        print(json.dumps(res), file=JSON_OUT[0], flush=True)
    if dist is not None:
        dist.destroy_process_group()


# --partition's default cohorts on the GPU (round 5, profiles/r05m_part_cohorts.txt: 1 / 2 / 3 / 4 cohorts
# 98.6 / 101.1 / 103.1-105.3 / 73.4 M per GPU on the 8-rank rehearsal; with more cohorts, or more hardware
# queues than the default 4, the cohorts' local steps run fully side by side and every round finishes later)
PARTITION_COHORTS = 3


def partition_run(args, par, dist, world, rank, dev, red_dev, devices, host: bool = False):
    """The partitioned bench on the ranks of `dist` (collective); the bench line's dict on rank 0, else None.
    host: the --rehearse-on-host run (the host build of the kernel body, CPU buffers, gloo)."""
    import torch
    part = importlib.import_module(PKG + ".partition")
    mapgen = importlib.import_module(PKG + ".mapgen")
    comp = importlib.import_module(PKG + ".compiler")
    cfg = args.config if args.config != "c3" else "c5"
    E = args.envs if args.envs != 65536 else 16384
    cm = comp.compile_scenario(mapgen.make_config(cfg))
    seeds = par.shard_seeds(450565, E, rank)
    local = not args.remote_rows
    if args.virtual_ranks > 1 and world == 1 and local:
        local = (part.partition_switches(cm, args.virtual_ranks) == 0).astype(np.uint8)
    lib = None
    if host:
        lib, _ = host_verifier()
    cohorts = getattr(args, "cohorts", None)
    # default: one cohort on the host build and on an RCCL job of several ranks (each cohort has its own
    # communicator, and concurrent communicators on one device have not been run on RCCL yet); --cohorts N asks
    # for the pipeline anyway
    rccl_multi = ((world > 1 or getattr(args, "rccl_one_rank", False)) and dist is not None
                  and dist.get_backend() == "nccl")
    cohorts = min(E, cohorts if cohorts else (1 if (host or rccl_multi) else PARTITION_COHORTS))
    # the break-even comparison: the same envs run env-sharded on the fused kernel -- every rank its
    # own envs with all their Q rows, no exchange -- timed the same way, before the partitioned job allocates
    fused = None
    if getattr(args, "compare_fused", True):
        runtime = importlib.import_module(PKG + ".runtime")
        fb = runtime.Batch(cm, HP, seeds, device=dev, lib=lib)
        fb.learn_begin()
        fb.apply_qinit()
        for _ in range(args.warmup):
            fb.step(args.decisions)
        if dist is not None:
            dist.barrier()
        if not host:
            torch.cuda.synchronize()
        tf = time.perf_counter()
        nf = 0
        for _ in range(args.steps):
            nf += fb.step(args.decisions)[0]
        if dist is not None:
            dist.barrier()
        if not host:
            torch.cuda.synchronize()
        dtf, nf_all = par.reduce_timing(dist, time.perf_counter() - tf, float(nf), device=red_dev)
        fused = nf_all / dtf
        fb.close()
    kw = dict(rank=rank, world=world, dist=dist, device=dev, lib=lib, buffer_device="cpu" if host else "cuda",
              local_rows=local)
    if getattr(args, "rccl_one_rank", False) and world == 1 and dist is not None:
        kw["exchange_collective"] = True
    pb = (part.CohortPipeline(cm, HP, seeds, rank * E, world * E, cohorts=cohorts, **kw) if cohorts > 1
          else part.PartitionedBatch(cm, HP, seeds, rank * E, world * E, **kw))
    pb.learn_begin()
    pb.apply_qinit()
    for _ in range(args.warmup):
        pb.step(args.decisions)

    def barrier():
        if dist is not None:
            dist.barrier()
        if not host:
            torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    rounds = 0
    ck0, d0, (w0, r0) = pb.checkpoints, pb.deferrals, pb.sync_count()
    for _ in range(args.steps):
        rounds += pb.step(args.decisions)
    barrier()
    (w1, r1) = pb.sync_count()
    dt = time.perf_counter() - t0
    total = float(E * args.decisions * args.steps)
    dt, total_all = par.reduce_timing(dist, dt, total, device=red_dev)
    # after the timed region: a spread sample of the job's envs, this rank's owned rows of them and the
    # state of those it simulates, vs a fused single-process host run of their seeds
    checked, bad, vthreads = 0, ["not verified (--verify-envs 0)"], 0
    if args.verify_envs > 0:
        parity = importlib.import_module(PKG + ".parity")
        hlib, vthreads = host_verifier()
        pick = parity.spread(world * E, args.verify_envs)
        bad = parity.check_partition(pb, HP, pick, lambda g: 450565 + g, [args.decisions] * (args.warmup + args.steps),
                                     hlib)
        checked = len(pick)
    pfield = parity_field(dist, checked, bad, device=red_dev, threads=vthreads)
    res = None
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": total_all / dt,
            "unit": "agent-env-steps/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic {cm.S}-switch/{cm.T}-train Flatland-format map (mapgen {cfg}, seed 450565)",
            "config": {"workload": f"{cfg}: {cm.S} switches / {cm.T} trains, switch agents graph-partitioned over "
                                   f"{world} rank(s) (BFS blocks, cut {part.cut_fraction(cm, pb.owner):.2f}), {E} envs "
                                   f"per GPU, {args.decisions} agent-env-steps per env per step, "
                                   + ("every row operation as a message" if args.remote_rows else
                                      f"rows of block 0 of a {args.virtual_ranks}-rank partition in place, the rest "
                                      "as messages" if (args.virtual_ranks > 1 and world == 1) else
                                      "own rows in place, other ranks' rows as messages"),
                       "local_switches": int(pb.local_mask.sum()),
                       "envs_per_gpu": E, "decisions_per_env_per_step": args.decisions,
                       "rounds_per_step": rounds / max(1, args.steps),
                       # the host's part in the rounds: count reads / device waits of the library (at the
                       # checkpoints only), the fixed segment sizes the ranks agreed on, envs deferred
                       "checkpoints_per_step": (pb.checkpoints - ck0) / max(1, args.steps),
                       "host_waits_per_step": (w1 - w0) / max(1, args.steps),
                       "count_reads_per_step": (r1 - r0) / max(1, args.steps),
                       "segment_records": pb.k_msg, "segment_capacity": pb.cap_msg,
                       "collectives_per_round": 2 if (world > 1 or kw.get("exchange_collective")) else 0,
                       "exchange": ("RCCL all_to_all_single" if (dist is not None and dist.get_backend() == "nccl"
                                                                 and (world > 1 or kw.get("exchange_collective")))
                                    else "gloo all_to_all_single" if world > 1 else "identity (one rank)"),
                       "cohorts": cohorts,
                       "deferrals": pb.deferrals - d0,
                       "parallelism": f"env-batch dp{world} x switch-agent partition {world}"},
            "library": library_info(pb.lib),
            "world_size": world,
            "backend": (dist.get_backend() if dist is not None else None),
            "devices": devices,
            **pfield,
        }
        if fused is not None:
            # > 1 only if the partition beats running the same envs env-sharded (each GPU all Q rows of its own
            # envs); it cannot while one env's rows fit a GPU (break-even)
            res["env_sharded_fused"] = {"value": fused, "unit": "agent-env-steps/sec",
                                        "what": f"the same {E} envs per GPU on the fused kernel, env-sharded over "
                                                f"{world} rank(s) (no exchange), {args.steps} x {args.decisions} "
                                                "decisions per env, timed the same way"}
            res["vs_env_sharded_fused"] = res["value"] / fused if fused > 0 else None
        if host:
            res["rehearsal"] = "host build of the kernel body over gloo: a rehearsal, not a GPU measurement"
    pb.close()
    return res


# configs[4] inside every N > 1 run of the default bench: the driver launches bench.py itself under
# torch.distributed.run, so this is where the partitioned exchange meets RCCL on a multi-GPU node.  A short run
# (c5, 2,048 envs per GPU, 4 timed steps of 256 decisions after 2 warm-up steps, 8 envs of the job re-run on
# the host build), after the env-sharded measurement, parity-checked like
# --partition.  A failure of the leg must not cost the bench line, and must not look like success either: rank 0
# prints the line with the leg's error and every rank exits with PARTITION_LEG_FAILED -- on an exception at once
# (rank 0) or after the watchdog (the other ranks wait for it, so that the launcher does not stop rank 0 before it
# has printed), on a hang by the watchdog (rank 0 first).  SFL_NO_PARTITION_LEG=1 skips it.  --rehearse-on-host
# runs it on the host build (PARTITION_LEG_HOST).
# (one cohort: the leg is the first contact of the exchange with RCCL, so it runs the single-job path with one
# communicator; --partition --cohorts N measures the cohort pipeline)
PARTITION_LEG = dict(config="c5", envs=2048, decisions=256, steps=4, warmup=2, verify_envs=8, remote_rows=False,
                     virtual_ranks=0, cohorts=1)
PARTITION_LEG_HOST = dict(PARTITION_LEG, envs=4, decisions=24, steps=1)
PARTITION_LEG_TIMEOUT_S = 300.0
PARTITION_LEG_FAILED = 3


def _hold_then_exit(seconds: float):
    """A rank other than 0 whose leg failed: wait (for rank 0's line), then end with the failure code."""
    time.sleep(seconds)
    os._exit(PARTITION_LEG_FAILED)


def partition_leg(par, dist, world, rank, dev, red_dev, devices, res, emit, host: bool = False):
    """Run PARTITION_LEG on every rank; on rank 0 return its summary for the bench line."""
    import threading
    timeout = PARTITION_LEG_TIMEOUT_S + (0.0 if rank == 0 else 30.0)  # (rank 0's fires first)

    def fail(error):
        if rank == 0:
            res["partition_leg"] = {"error": error}
            emit(res)
        os._exit(PARTITION_LEG_FAILED)
    timer = threading.Timer(timeout, fail, args=(f"no result within {PARTITION_LEG_TIMEOUT_S:.0f} s; the bench "
                                                 "line was printed by the watchdog",))
    timer.daemon = True
    timer.start()
    t0 = time.perf_counter()
    spec = PARTITION_LEG_HOST if host else PARTITION_LEG
    try:
        leg = partition_run(argparse.Namespace(**spec), par, dist, world, rank, dev, red_dev, devices, host=host)
    except Exception as ex:  # noqa: BLE001 -- reported on the line and in the exit code
        print(f"bench.py: rank {rank}: the partitioned leg failed: {ex!r}", file=sys.stderr, flush=True)
        if rank == 0:
            timer.cancel()
            fail(f"rank 0: {ex!r}")
            return None  # (only when os._exit is replaced, in tests)
        return _hold_then_exit(max(0.0, timeout - (time.perf_counter() - t0)))
    timer.cancel()
    if rank != 0:
        return None
    cfgd = leg["config"]
    out = {"what": "configs[4] at this N: " + cfgd["workload"] + f", {spec['steps']} timed step(s)",
           "value": leg["value"], "unit": leg["unit"], "backend": leg["backend"], "world_size": leg["world_size"],
           "rounds_per_step": cfgd["rounds_per_step"], "checkpoints_per_step": cfgd["checkpoints_per_step"],
           "count_reads_per_step": cfgd["count_reads_per_step"], "segment_records": cfgd["segment_records"],
           "collectives_per_round": cfgd.get("collectives_per_round"), "cohorts": cfgd.get("cohorts"),
           "deferrals": cfgd["deferrals"], "parity": leg.get("parity"),
           "vs_env_sharded_fused": leg.get("vs_env_sharded_fused"),
           "parity_envs_checked": leg.get("parity_envs_checked"), "wall_s": time.perf_counter() - t0}
    if host:
        out["rehearsal"] = leg.get("rehearsal")
    return out


if __name__ == "__main__":
    main()
