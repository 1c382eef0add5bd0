"""GPU parity tests (MI355X): the HIP library through the C-ABI against the reference's golden
vectors, the CPU oracle, and the host build of the same kernel body."""
import importlib

import numpy as np
import pytest

from tests import _golden, _trace
from oracle import sfl_oracle as so

pytestmark = pytest.mark.gpu

mapgen = importlib.import_module("network-distributed-q-learning_amd.mapgen")
comp = importlib.import_module("network-distributed-q-learning_amd.compiler")
runtime = importlib.import_module("network-distributed-q-learning_amd.runtime")
_lib = importlib.import_module("network-distributed-q-learning_amd._lib")
build = importlib.import_module("network-distributed-q-learning_amd.build")
parity = importlib.import_module("network-distributed-q-learning_amd.parity")
HP = dict(gamma=1.0, epsilon=0.5, epsilon_decay_rate=0.9997, lr=0.1, lr_decay_rate=1.0, default_q=0.0)
CASES = _golden.cases()


@pytest.fixture(scope="module")
def lib():
    build.build_hip()
    return _lib.load_product()


def _select_kernel(request, monkeypatch):
    monkeypatch.delenv("SFL_KERNEL", raising=False)
    monkeypatch.delenv("SFL_WAVE_G", raising=False)
    if request.param == "scalar":
        monkeypatch.setenv("SFL_KERNEL", "scalar")
    elif request.param == "wave":
        monkeypatch.setenv("SFL_WAVE_G", "16")
    elif request.param == "wave8":
        monkeypatch.setenv("SFL_WAVE_G", "8")
    else:
        monkeypatch.setenv("SFL_WAVE_G", "32")
    return request.param


@pytest.fixture(params=["wave", "wave32", "wave8", "scalar"])
def kernel(request, monkeypatch):
    """Which device kernel a Batch created inside the test runs (chosen at sfl_create):
    'wave' = k_wave at the default group size (four envs per wavefront for maps with <= 32 trains: the
    bench kernel), 'wave32' = two envs per wavefront (what a batch too small to fill the device gets,
    sfl_engine.h choose_variant), 'wave8' = eight envs per wavefront, one train per lane (the default for
    maps with <= 8 trains and batches that fill the device; maps with more trains fall back to one env per
    wavefront), 'scalar' = k_run."""
    return _select_kernel(request, monkeypatch)


@pytest.fixture(params=["wave", "scalar"])
def part_kernel(request, monkeypatch):
    """The partitioned local step's kernels: k_wave (one env per wavefront, whatever the fused group size --
    so the fused kernel's 'wave32' / 'wave8' group sizes are not separate cases here) or k_run."""
    return _select_kernel(request, monkeypatch)


def _check_kernel(b, kernel):
    c = b.counters()
    assert (c["kernel_variant"] > 0) == (kernel != "scalar"), c


def _q(items):
    return {tuple(k): v for k, v in items}


@pytest.mark.parametrize("name", CASES)
def test_golden_env0_and_trace(lib, kernel, name):
    g = _golden.load(name)
    hp = g["hparams"]
    cm = comp.compile_scenario(g["scenario_obj"])
    seed1 = g["seed"] + 7
    b = runtime.Batch(cm, hp, [g["seed"], seed1, seed1 + 1], lib=lib, max_steps=hp.get("max_steps", 100_000),
                      ntab=1 << 16)
    b.trace_env = 1
    _check_kernel(b, kernel)
    out = b.learn(g["n_episodes"], exploit_freq=g["exploit_freq"])
    ref = g["learn"]["outputs"]
    assert out["cum_reward"][:, 0].tolist() == ref["cum_reward"]
    assert out["arrived"][:, 0].tolist() == ref["arrived_trains"]
    assert out["num_malfunctions"][:, 0].tolist() == ref["num_malfunctions"]
    assert out["delays"][:, :, 0].astype(float).tolist() == ref["delays"]
    assert b.q_dict(0) == _q(g["learn"]["q_final"])
    mine = _trace.decode_kernel_trace(b.last_trace)
    env, model = so.build(g["scenario_obj"], seed1, hp, max_steps=hp.get("max_steps", 100_000), trace=False)
    recs = []
    model.on_step = _trace.oracle_recorder(cm, recs)
    model.learn(g["n_episodes"], exploit_freq=g["exploit_freq"])
    assert mine == recs
    b.trace_env = None
    t = b.test(1)
    assert float(t["cum_reward"][0, 0]) == g["test"]["cum_reward"]
    assert int(t["arrived"][0, 0]) == g["test"]["arrived"]
    assert b.q_dict(0) == _q(g["test"]["q_final"])


def test_c2_batch_gpu_equals_host_build_and_oracle(lib, kernel):
    """512 envs stepped in chunks: every env's Q-table bit-equal to the host build, sampled envs to the oracle."""
    from tests import hostsim
    sc = mapgen.make_config("c2")
    cm = comp.compile_scenario(sc)
    seeds = [1000 + i for i in range(512)]
    chunks = [37, 91, 250]
    bg = runtime.Batch(cm, HP, seeds, lib=lib, ntab=1 << 14)
    _check_kernel(bg, kernel)
    bh = runtime.Batch(cm, HP, seeds, lib=hostsim.lib(), ntab=1 << 14)
    for b in (bg, bh):
        b.learn_begin()
        b.apply_qinit()
        for n in chunks:
            got, _ = b.step(n)
            assert got == n * len(seeds)
    for e in range(len(seeds)):
        qg, tg = bg.q_raw(e)
        qh, th = bh.q_raw(e)
        assert np.array_equal(qg, qh) and np.array_equal(tg, th), f"env {e}"
    for e in (0, 255, 511):
        env, model = so.build(sc, seeds[e], HP, trace=False)
        so.run_decisions(model, sum(chunks))
        assert bg.q_dict(e) == model.q


@pytest.mark.parametrize("cfg,E", [("c2", 256), ("c3", 1024), ("c5", 8)])
def test_flatland_malfunction_stream_gpu(lib, kernel, cfg, E):
    """§8(f)4: the Flatland-compatible malfunction table (mfstream.py) read by the device kernels:
    every env bit-equal to the host build, env 1 to the oracle drawing live from numpy's RandomState."""
    from tests import hostsim
    sc = mapgen.make_config(cfg, malfunction=(0.02, 5, 15))
    cm = comp.compile_scenario(sc)
    seeds = [777 + i for i in range(E)]
    bg = runtime.Batch(cm, HP, seeds, lib=lib, ntab=1 << 14, malfunction_stream="flatland")
    _check_kernel(bg, kernel)
    bh = runtime.Batch(cm, HP, seeds, lib=hostsim.lib(), ntab=1 << 14, malfunction_stream="flatland")
    og, oh = bg.learn(3), bh.learn(3)
    for k in ("num_malfunctions", "cum_reward", "arrived", "decisions", "delays"):
        assert np.array_equal(og[k], oh[k]), k
    assert og["num_malfunctions"].sum() > 0
    for e in range(E):
        qg, tg = bg.q_raw(e)
        qh, th = bh.q_raw(e)
        assert np.array_equal(qg, qh) and np.array_equal(tg, th), f"env {e}"
    env, model = so.build(sc, seeds[1], HP, trace=False, mf_stream="flatland")
    ref = model.learn(3)
    assert og["num_malfunctions"][:, 1].tolist() == ref["num_malfunctions"]
    assert bg.q_dict(1) == model.q


@pytest.mark.parametrize("thr", [0, 1])
def test_observer_delay_threshold_gpu(lib, kernel, thr):
    """StandardObserver(delay_threshold=thr) (observer.py:221, 228-244) on the device: every env
    bit-equal to the host build, env 3 to the oracle."""
    from tests import hostsim
    sc = mapgen.make_config("c2")
    cm = comp.compile_scenario(sc)
    seeds = [31 + i for i in range(128)]
    bg = runtime.Batch(cm, HP, seeds, lib=lib, ntab=1 << 14, delay_threshold=thr)
    _check_kernel(bg, kernel)
    bh = runtime.Batch(cm, HP, seeds, lib=hostsim.lib(), ntab=1 << 14, delay_threshold=thr)
    og, oh = bg.learn(3), bh.learn(3)
    assert np.array_equal(og["cum_reward"], oh["cum_reward"])
    for e in range(len(seeds)):
        qg, tg = bg.q_raw(e)
        qh, th = bh.q_raw(e)
        assert np.array_equal(qg, qh) and np.array_equal(tg, th), f"env {e}"
    env, model = so.build(sc, seeds[3], HP, trace=False, delay_threshold=thr)
    model.learn(3)
    assert bg.q_dict(3) == model.q


def test_c3_full_size_batch(lib):
    """BASELINE config: 64-switch / 32-train map, 65,536 envs on one GPU.  Size-independent
    checks on the whole batch + exact oracle parity on sampled envs."""
    sc = mapgen.make_config("c3")
    cm = comp.compile_scenario(sc)
    E = 65536
    seeds = [450565 + i for i in range(E)]
    b = runtime.Batch(cm, HP, seeds, lib=lib)
    assert b.counters()["kernel_variant"] > 0  # the bench kernel
    b.learn_begin()
    b.apply_qinit()
    total = 0
    for n in (16, 48):
        got, ms = b.step(n)
        assert got == n * E and ms > 0
        total += n
    c = b.counters()
    assert c["decisions"] == total * E
    for e in (0, 12345, E - 1):
        env, model = so.build(sc, seeds[e], HP, trace=False)
        so.run_decisions(model, total)
        assert b.q_dict(e) == model.q, f"env {e}"
    b.close()


def test_c5_small_batch(lib, kernel):
    """256-switch / 128-train map (max trains per env, two train slots per lane in k_wave), a few
    envs against the oracle, on both kernels."""
    sc = mapgen.make_config("c5")
    cm = comp.compile_scenario(sc)
    seeds = [5, 6, 7, 8]
    b = runtime.Batch(cm, HP, seeds, lib=lib, ntab=1 << 14)
    _check_kernel(b, kernel)
    b.learn_begin()
    b.apply_qinit()
    b.step(150)
    env, model = so.build(sc, seeds[2], HP, trace=False)
    so.run_decisions(model, 150)
    assert b.q_dict(2) == model.q


@pytest.mark.parametrize("local_rows", [False, True, "block0of4"])
@pytest.mark.parametrize("cfg,E", [("c2", 256), ("c5", 64), ("golden:city6_s5", 128)])
def test_partitioned_rounds_gpu_equal_fused(lib, cfg, E, part_kernel, local_rows):
    """Graph-partitioned mode (BASELINE configs[4]) on the GPU, one rank: the owner-side Q rows,
    the request / reply / update round trips through device buffers, bit-equal to the fused kernel.
    kernel: the local step on k_wave (observe / apply passes, PART) or on the lane-per-env body;
    local_rows: k_wave decides on this rank's own rows in place (one round per step), sends every
    row operation as a message (decisions + 1 rounds), or keeps only block 0 of a 4-rank partition
    in place (a 4-rank job's message traffic on one rank)."""
    import torch
    kernel = part_kernel
    part = importlib.import_module("network-distributed-q-learning_amd.partition")
    sc = _golden.load(cfg[7:])["scenario_obj"] if cfg.startswith("golden:") else mapgen.make_config(cfg)
    cm = comp.compile_scenario(sc)
    seeds = [2000 + i for i in range(E)]
    ref = runtime.Batch(cm, HP, seeds, lib=lib, ntab=1 << 14)
    ref.learn_begin()
    ref.apply_qinit()
    loc = (part.partition_switches(cm, 4) == 0).astype(np.uint8) if local_rows == "block0of4" else local_rows
    pb = part.PartitionedBatch(cm, HP, seeds, 0, E, lib=lib, ntab=1 << 14, buffer_device="cuda", local_rows=loc)
    pb.learn_begin()
    pb.apply_qinit()
    _check_kernel(pb.batch, kernel)
    for n in (40, 75, 600):  # (600: one launch of local decisions runs past the 8-bit stage field)
        ref.step(n)
        r = pb.step(n)
        if kernel == "scalar" or local_rows is False:
            assert r == n + 1
        elif local_rows is True:
            assert r == 1
        else:
            assert 1 < r <= n + 1
    torch.cuda.synchronize()
    mk = pb.owned_mask()
    assert mk.all()
    for e in range(E):
        q, t = pb.owned_q(e)
        qr, tr = ref.q_raw(e)
        assert np.array_equal(q, qr) and np.array_equal(t, tr), f"env {e}"
    pb.close()
    ref.close()


@pytest.mark.parametrize("cohorts", [2, 3])
def test_cohort_pipeline_gpu_equal_fused(lib, cohorts):
    """partition.CohortPipeline on the GPU, one rank: the envs as independent partitioned jobs on their own
    streams, their rounds issued alternately (kernels of different cohorts run concurrently), block 0 of a
    4-rank partition in place; every env's rows bit-equal to the fused kernel."""
    import torch
    part = importlib.import_module("network-distributed-q-learning_amd.partition")
    cm = comp.compile_scenario(mapgen.make_config("c5"))
    E = 200
    seeds = [2000 + i for i in range(E)]
    ref = runtime.Batch(cm, HP, seeds, lib=lib, ntab=1 << 14)
    ref.learn_begin()
    ref.apply_qinit()
    loc = (part.partition_switches(cm, 4) == 0).astype(np.uint8)
    pb = part.CohortPipeline(cm, HP, seeds, 0, E, cohorts=cohorts, lib=lib, ntab=1 << 14, buffer_device="cuda",
                             local_rows=loc)
    assert len({p.stream.cuda_stream for p in pb.parts}) == cohorts
    pb.learn_begin()
    pb.apply_qinit()
    for n in (40, 300):
        ref.step(n)
        assert 1 < pb.step(n) <= n + 1
    torch.cuda.synchronize()
    for e in range(E):
        q, t = pb.owned_q(e)
        qr, tr = ref.q_raw(e)
        assert np.array_equal(q, qr) and np.array_equal(t, tr), f"env {e}"
        b, le = pb.sim_env(e)
        for x, y in zip(parity.env_state(b, le), parity.env_state(ref, e)):
            assert np.array_equal(np.asarray(x), np.asarray(y)), f"env {e} state"
    pb.close()
    ref.close()


def test_partition_staging_overflow_reported_in_its_step(lib):
    """More update records in one env's round than its staging slots hold (upd_per_env 2, every row a
    message): the wave kernel's run raises E_MSG_OVF (flag 16) in the step where it happened -- the same step
    as the same GPU kernel reading its counts after every round (which pins the round that set it), at the
    first checkpoint round at or after that round.  (The host build is not the comparison here: the lane body
    stages one key-set insert where k_wave's owner inserts while answering, so they overflow at different
    steps; tests/test_partition.py checks the same property on the host build.)"""
    from tests import test_partition
    part = importlib.import_module("network-distributed-q-learning_amd.partition")
    cm = comp.compile_scenario(mapgen.make_config("c2"))
    seeds = [3000 + i for i in range(64)]
    kw = dict(lib=lib, buffer_device="cuda", ntab=1 << 14, local_rows=False, upd_per_env=2)
    every = part.PartitionedBatch(cm, HP, seeds, 0, len(seeds), checkpoint_every_round=True, **kw)
    dflt = part.PartitionedBatch(cm, HP, seeds, 0, len(seeds), **kw)
    assert dflt.cap_upd == 128 and dflt.batch.counters()["kernel_variant"] > 0
    (i_e, r_e), (i_d, r_d) = test_partition._first_failing_step(every), test_partition._first_failing_step(dflt)
    every.close()
    dflt.close()
    assert i_e is not None and i_d == i_e, (i_e, i_d)
    assert r_d == min(r for r in range(r_e, 4 * 4 + 65) if dflt._checkpoint(r, 4)), (r_e, r_d)


@pytest.mark.parametrize("cfg,world", [("c2", 2), ("c5", 2), ("c5", 3)])
def test_two_rank_partition_wave_gpu(lib, cfg, world):
    """Two ranks (processes) on GPU 0 over gloo: k_wave's PART local step with the row requests,
    replies and update records crossing ranks; each rank's owned Q rows, key set and env states
    bit-equal to the fused run of all envs (host build)."""
    from tests import test_partition
    test_partition.two_rank_run(cfg, gpu=True, world=world)


def test_two_rank_cohorts_gpu(lib):
    """Two ranks on GPU 0 over gloo, two cohorts per rank (a process group and a stream each), the
    cohorts' rounds alternating; bit-equal to the fused run (segments starting at 2 records)."""
    from tests import test_partition
    test_partition.two_rank_run("c5", gpu=True, world=2, steps=(90, 60), k_init=2, cohorts=2)


def test_two_rank_partition_gpu_rounds_queue_between_checkpoints(lib):
    """Two ranks on GPU 0 over gloo, one 1,024-decision step: between checkpoint rounds the library neither
    waits for the device nor reads a count (tests/test_partition.py _check_round_log), bit-equal to the
    fused run.  (gloo itself stages each device segment through host memory; RCCL moves it device to
    device on the same stream.)"""
    from tests import test_partition
    for st in test_partition.two_rank_run("c5", gpu=True, world=2, steps=(1024,), log_rounds=True):
        s = st[1024]
        # (k_wave decides on each rank's own rows in place, so a step takes fewer rounds than decisions + 1)
        assert s["reads"] == s["checkpoints"] <= 8 + s["rounds"] // 32


def test_partition_rccl_one_rank_stream_ordering(lib):
    """RCCL itself on the partitioned exchange: one rank over backend "nccl" whose segments still travel as
    all_to_all_single collectives between separate device buffers, queued on the job's stream between the wave
    kernel's local step and the owner kernel -- the stream ordering of a multi-GPU job (RCCL refuses two ranks on
    one GPU).  A missing dependency would let the owner read stale messages; owned rows and env states equal the
    fused host run."""
    from tests import test_partition
    rounds = test_partition.one_rank_collective_run("nccl")
    assert all(r > 1 for r in rounds)


def test_two_rank_partition_gpu_deferred_envs_bit_equal(lib):
    """k_part_compact's deferral on the device: segments of 2 message records per destination to start with,
    envs deferred whole and skipped by the wave kernel's local step until they fit."""
    from tests import test_partition
    stats = test_partition.two_rank_run("c5", gpu=True, world=2, steps=(90, 60), k_init=2)
    assert sum(st["deferrals"] for st in stats) > 0


@pytest.mark.parametrize("S,T,variant", [(64, 48, 3), (100, 48, 4), (120, 64, 4), (100, 100, 5), (200, 40, 5),
                                         (256, 128, 5)])
def test_wave_kernel_shapes(lib, S, T, variant):
    """Every k_wave shape (sfl::kVariants: more trains per env, more ports / switches per lane)
    bit-equal to the host build of the lane kernel, and sampled envs to the oracle."""
    from tests import hostsim
    sc = mapgen.generate(S, T, 8, seed=4242, malfunction=(0.01, 5, 15), name="shape")
    cm = comp.compile_scenario(sc)
    seeds = [300 + i for i in range(64)]
    bg = runtime.Batch(cm, HP, seeds, lib=lib, ntab=1 << 14)
    assert bg.counters()["kernel_variant"] == variant
    bh = runtime.Batch(cm, HP, seeds, lib=hostsim.lib(), ntab=1 << 14)
    for b in (bg, bh):
        b.learn_begin()
        b.apply_qinit()
        for n in (50, 130):
            b.step(n)
    for e in range(len(seeds)):
        qg, tg = bg.q_raw(e)
        qh, th = bh.q_raw(e)
        assert np.array_equal(qg, qh) and np.array_equal(tg, th), f"env {e}"
    env, model = so.build(sc, seeds[5], HP, trace=False)
    so.run_decisions(model, 180)
    assert bg.q_dict(5) == model.q
    bg.close()
    bh.close()


# ---- the bench horizon and the reference's API on the product library ---------------------------

def _spread(E, n=64, stride=1021):
    """n env indices spread over the batch (different blocks, CUs and XCDs)."""
    return sorted({(k * stride) % E for k in range(n)} | {0, E - 1})


def _env_state(b, env):
    import ctypes as C
    cm = b.cm
    el, ph = C.c_int32(), C.c_int32()
    sem = np.zeros(4 * cm.S, np.uint64)
    pos = np.zeros(cm.T, np.int32)
    bits = np.zeros(cm.T, np.uint32)
    P = C.POINTER
    b.lib.check(b.lib.dll.sfl_get_env_state(b.h, env, C.byref(el), C.byref(ph), sem.ctypes.data_as(P(C.c_uint64)),
                                            pos.ctypes.data_as(P(C.c_int32)), bits.ctypes.data_as(P(C.c_uint32))),
                "sfl_get_env_state")
    return el.value, ph.value, sem, pos, bits


def test_c3_full_size_bench_horizon(lib):
    """BASELINE configs[2] at the bench's size AND horizon: 65,536 envs, 2,560 decisions each in
    bench-sized launches (every env crosses >= 2 episode ends: resets, arrival bonuses, truncation
    and the (switch, train) slot epochs).  66 envs spread over the grid bit-equal to the host build
    (Q-table, key set, semaphores, trains), 3 of them to the oracle."""
    from tests import hostsim
    sc = mapgen.make_config("c3")
    cm = comp.compile_scenario(sc)
    E = 65536
    seeds = [450565 + i for i in range(E)]
    chunks = (1024, 512, 1024)
    b = runtime.Batch(cm, HP, seeds, lib=lib)
    assert b.counters()["kernel_variant"] > 0
    b.learn_begin()
    b.apply_qinit()
    for n in chunks:
        got, ms = b.step(n)
        assert got == n * E and ms > 0
    assert b.counters()["decisions"] == sum(chunks) * E
    pick = _spread(E)
    bh = runtime.Batch(cm, HP, [seeds[e] for e in pick], lib=hostsim.lib())
    bh.learn_begin()
    bh.apply_qinit()
    for n in chunks:
        bh.step(n)
    for i, e in enumerate(pick):
        qg, tg = b.q_raw(e)
        qh, th = bh.q_raw(i)
        assert np.array_equal(qg, qh) and np.array_equal(tg, th), f"env {e}"
        sg, sh = _env_state(b, e), _env_state(bh, i)
        assert sg[0] == sh[0] and sg[1] == sh[1], f"env {e}"
        for x, y in zip(sg[2:], sh[2:]):
            assert np.array_equal(x, y), f"env {e}"
    for e in (0, pick[len(pick) // 2], E - 1):
        env, model = so.build(sc, seeds[e], HP, trace=False)
        st = so.run_decisions(model, sum(chunks))
        assert st["t"] >= 2, "the horizon must cross episode ends"
        assert b.q_dict(e) == model.q, f"env {e}"
    bh.close()
    b.close()


def test_c2_stated_batch_4096(lib):
    """BASELINE configs[1] at its stated size: 16-switch / 8-train map, 4,096 envs, every env
    bit-equal to the host build after 1,200 decisions (many episodes)."""
    from tests import hostsim
    sc = mapgen.make_config("c2")
    cm = comp.compile_scenario(sc)
    E = 4096
    seeds = [450565 + i for i in range(E)]
    bg = runtime.Batch(cm, HP, seeds, lib=lib)
    assert bg.counters()["kernel_variant"] > 0
    bh = runtime.Batch(cm, HP, seeds, lib=hostsim.lib())
    for b in (bg, bh):
        b.learn_begin()
        b.apply_qinit()
        for n in (200, 1000):
            assert b.step(n)[0] == n * E
    for e in range(E):
        qg, tg = bg.q_raw(e)
        qh, th = bh.q_raw(e)
        assert np.array_equal(qg, qh) and np.array_equal(tg, th), f"env {e}"
    env, model = so.build(sc, seeds[4095], HP, trace=False)
    so.run_decisions(model, 1200)
    assert bg.q_dict(4095) == model.q
    bg.close()
    bh.close()


@pytest.mark.parametrize("lds_map", ["1", "0"])
def test_c2_stated_batch_lds_map_variant(lib, monkeypatch, lds_map):
    """configs[1]'s batch runs variant 11 (variant 8 with the move table and distance map in LDS, sfl_engine.h); with
    SFL_LDS_MAP=0 variant 8 reads them from global memory.  Both bit-equal to the host build on 512 of its envs (the
    same 2,048-wavefront launch shape: the other envs run too)."""
    from tests import hostsim
    monkeypatch.setenv("SFL_LDS_MAP", lds_map)
    monkeypatch.delenv("SFL_WAVE_G", raising=False)
    cm = comp.compile_scenario(mapgen.make_config("c2"))
    seeds = [777 + i for i in range(4096)]
    bg = runtime.Batch(cm, HP, seeds, lib=lib)
    assert bg.counters()["kernel_variant"] == (11 if lds_map == "1" else 8)
    pick = list(range(0, 4096, 8))
    bh = runtime.Batch(cm, HP, [seeds[e] for e in pick], lib=hostsim.lib())
    for b in (bg, bh):
        b.learn_begin()
        b.apply_qinit()
        for n in (300, 700):
            b.step(n)
    for i, e in enumerate(pick):
        qg, tg = bg.q_raw(e)
        qh, th = bh.q_raw(i)
        assert np.array_equal(qg, qh) and np.array_equal(tg, th), f"env {e}"
    bg.close()
    bh.close()


def test_device_pow_beyond_tables(lib, kernel):
    """ntab = 16: epsilon beyond the host table comes from the device's pow (pow_ool); checked
    against the oracle's Python ``**`` (distr_q.py:59-68) bit-exactly.  (eps only decides
    ``random() < eps``: an ulp of pow moves that decision by ~1e-17 in probability.)"""
    hp = dict(gamma=0.95, epsilon=0.3, epsilon_decay_rate=0.99, lr=0.2, lr_decay_rate=1.0, default_q=-5.0)
    sc = mapgen.make_config("c2")
    cm = comp.compile_scenario(sc)
    seeds = [77 + i for i in range(128)]
    b = runtime.Batch(cm, hp, seeds, lib=lib, ntab=16)
    _check_kernel(b, kernel)
    b.learn_begin()
    b.apply_qinit()
    b.step(900)
    for e in (0, 64, 127):
        env, model = so.build(sc, seeds[e], hp, trace=False)
        st = so.run_decisions(model, 900)
        assert max(st["counts"].values()) > 16  # the pow path ran
        assert b.q_dict(e) == model.q, f"env {e}"
    b.close()


def test_decayed_lr_beyond_table_fails_loudly(lib, kernel):
    """A decaying lr (distr_q.py:70-79) enters the Q values, and the device pow differs from the
    host libm's by an ulp (measured: round 2, test_device_pow_beyond_tables with lr_decay 0.999 at
    ntab 16): past the table the run stops with E_LR_TABLE instead of silently losing bit-exactness."""
    hp = dict(gamma=0.95, epsilon=0.3, epsilon_decay_rate=0.99, lr=0.2, lr_decay_rate=0.999, default_q=-5.0)
    cm = comp.compile_scenario(mapgen.make_config("c2"))
    b = runtime.Batch(cm, hp, [77, 78], lib=lib, ntab=16)
    _check_kernel(b, kernel)
    b.learn_begin()
    b.apply_qinit()
    with pytest.raises(_lib.SflError, match="ntab"):
        b.step(900)
    b.close()


@pytest.mark.parametrize("name", ["c1_s7", "c2_mf"])
def test_distr_q_learn_outputs_gpu(lib, tmp_path, name):
    """DistrQLearning.learn / save / load / test through libsfl.so: the reference's .npz set and
    .pkl dict equal the golden vectors recorded from the reference."""
    from tests import test_api_hostsim as api
    api.test_learn_outputs_match_reference_files(tmp_path, name, lib=lib)


@pytest.mark.parametrize("name", ["c2_s3", "city6_s5"])
def test_distr_q_checkpoint_exploit_gpu(lib, tmp_path, name):
    from tests import test_api_hostsim as api
    api.test_checkpoint_after_coinciding_exploit_round(tmp_path, name, lib=lib)


@pytest.mark.parametrize("exploit", [None, 1])
def test_distr_q_checkpoint_every_episode_gpu(lib, tmp_path, exploit):
    from tests import test_api_hostsim as api
    api.test_checkpoint_every_episode(tmp_path, exploit, lib=lib)


def test_distr_q_load_reference_pickle_gpu(lib, tmp_path):
    from tests import test_api_hostsim as api
    api.test_load_reference_pickle_format(tmp_path, lib=lib)


def test_long_horizon_city_map_stays_on_wave(lib):
    """A city map whose timetable horizon (t_hi = 1,110 ticks) overflowed round 1's 11-bit record
    time field now runs k_wave (14-bit start tick, 9-bit span), bit-equal to the host build."""
    from tests import hostsim
    sc = mapgen.generate_cities(6, 24, seed=3, spacing=70, malfunction=(0.01, 5, 15), name="long")
    assert sc.max_episode_steps > 900
    cm = comp.compile_scenario(sc)
    seeds = [900 + i for i in range(64)]
    bg = runtime.Batch(cm, HP, seeds, lib=lib, ntab=1 << 14)
    assert bg.counters()["kernel_variant"] > 0 and bg.kernel_note == ""
    bh = runtime.Batch(cm, HP, seeds, lib=hostsim.lib(), ntab=1 << 14)
    for b in (bg, bh):
        b.learn_begin()
        b.apply_qinit()
        for n in (300, 900):
            b.step(n)
    for e in range(len(seeds)):
        qg, tg = bg.q_raw(e)
        qh, th = bh.q_raw(e)
        assert np.array_equal(qg, qh) and np.array_equal(tg, th), f"env {e}"
        sg, sh = _env_state(bg, e), _env_state(bh, e)
        assert sg[0] == sh[0] and all(np.array_equal(x, y) for x, y in zip(sg[2:], sh[2:])), f"env {e}"
    env, model = so.build(sc, seeds[7], HP, trace=False)
    so.run_decisions(model, 1200)
    assert bg.q_dict(7) == model.q
    bg.close()
    bh.close()


def test_fallback_kernel_is_reported(lib, monkeypatch):
    """A map k_wave cannot hold (more than 256 switches) runs the lane-per-env body with a
    warning, or is refused under SFL_REQUIRE_WAVE=1."""
    sc = mapgen.generate(300, 40, 8, seed=5, name="big")
    cm = comp.compile_scenario(sc)
    with pytest.warns(RuntimeWarning, match="256 switches"):
        b = runtime.Batch(cm, HP, [1, 2], lib=lib)
    assert b.counters()["kernel_variant"] == 0
    b.close()
    monkeypatch.setenv("SFL_REQUIRE_WAVE", "1")
    with pytest.raises(_lib.SflError, match="256 switches"):
        runtime.Batch(cm, HP, [1, 2], lib=lib)


# ---- round 3: the entry scripts on the GPU, the external-action (AEC) mode ---------------------------
def _script(*args, timeout=600):
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, *args], cwd=repo, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (args, r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


@pytest.mark.parametrize("name", ["c1_s7", "city6_s5"])
def test_main_and_eval_scripts_gpu(lib, tmp_path, name):
    """``python main.py -c config.ini`` then ``python eval.py EXP`` through libsfl.so (main.py:13-78,
    eval.py:34-99): the .npz / .pkl outputs equal the golden vectors recorded from the reference."""
    from tests import test_entrypoints as te
    g, exp = te.prepare_golden_experiment(tmp_path, name)
    out = _script("main.py", "-c", str(exp / "config.ini"))
    assert "DONE!" in out
    te.check_main_outputs(g, exp)
    _script("eval.py", str(exp))
    te.check_eval_outputs(g, exp)


def test_main_script_flatland_stream_gpu(lib, tmp_path):
    """``[ENV] malfunction_stream = flatland`` through main.py on libsfl.so equals the oracle."""
    from tests import test_entrypoints as te
    sc, hp, exp = te.prepare_flatland_stream_experiment(tmp_path)
    _script("main.py", "-c", str(exp / "config.ini"))
    te.check_flatland_stream_outputs(sc, hp, exp)


@pytest.mark.parametrize("name", CASES)
def test_aec_replay_golden_gpu(lib, name):
    """The external-action mode on the GPU: the reference's recorded actions replayed through
    ASyncSwitchEnv.reset / agent_iter / last / step reproduce every golden decision and step event
    (observation, reward, mask, successor, arrivals, time, semaphore-table digest)."""
    from tests import aec_replay
    g = _golden.load(name)
    n_dec = sum(1 for e in g["learn"]["events"] if e[0] == "D")
    # (each step is a launch plus host reads of the env's state; the > 4,000-decision runs -- c5_mf's 256 switches /
    # 128 trains, grid100x48_s3 -- replay a 3,000-decision prefix of learn() and of test() with the semaphore digest
    # every 4th step; the host build replays every event of them, tests/test_aec.py)
    cap, every = (3000, 4) if n_dec > 4000 else (None, 1)
    n = aec_replay.replay(g, g["learn"]["events"], lib, digest_every=every, max_decisions=cap)
    assert n == (n_dec if cap is None else min(cap, n_dec))
    aec_replay.replay(g, g["test"]["events"], lib, digest_every=every, max_decisions=cap)


@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_aec_batch_gpu_equals_host_build(lib, cfg):
    """512 c2 and c3 envs stepped by a fixed policy through sfl_env_step: every output of every call equals
    the host build's (bit-exact), c2 across episode ends."""
    from tests import hostsim
    aec = importlib.import_module("network-distributed-q-learning_amd.aec")
    cm = comp.compile_scenario(mapgen.make_config(cfg))
    seeds = [450565 + i for i in range(512)]
    bg, bh = aec.AECBatch(cm, seeds, lib=lib), aec.AECBatch(cm, seeds, lib=hostsim.lib())
    og, oh = bg.step(None), bh.step(None)
    ends = 0
    for k in range(400):
        for key in og:
            assert np.array_equal(og[key], oh[key]), (k, key)
        acts = []
        for e in range(len(seeds)):
            s = int(og["agent"][e])
            if s < 0:
                acts.append(-1)
                ends += 1
                continue
            m, n = int(og["mask"][e]), int(cm.n_actions[s])
            allowed = [a for a in range(n) if (m >> a) & 1]
            acts.append(allowed[(k + e) % len(allowed)])
        og, oh = bg.step(acts), bh.step(acts)
    assert ends > 0 or cfg != "c2"
    bg.close()
    bh.close()


def test_phase_timers_fill_the_reference_accumulators(lib, tmp_path):
    """learn() runs the TIMED kernel: the seven accumulators of the reference's scripts
    (switch_env.py:67-73, printed at test_model.py:73-82) are filled from the device's phase cycles, their
    parts add up to the learn launches' kernel time, and the Q-tables equal an untimed run's (the trace
    instantiation carries no timers): the timers only observe."""
    env_mod = importlib.import_module("network-distributed-q-learning_amd.env")
    dq = importlib.import_module("network-distributed-q-learning_amd.distr_q")
    models = []
    for traced in (False, True):
        env = env_mod.ASyncSwitchEnv(mapgen.make_config("c3"), max_steps=100_000, n_envs=256)
        model = dq.DistrQLearning(env=env, gamma=1.0, epsilon=0.5, epsilon_decay_rate=0.9997, lr=0.1,
                                  lr_decay_rate=1.0, default_q=0.0, seed=450565, lib=lib)
        assert model.batch.counters()["kernel_variant"] > 0
        if traced:
            model.batch.trace_env = 7
        model.learn(num_episodes=2, out_dir=str(tmp_path), checkpoint_freq=10_000)
        models.append((env, model))
    env, model = models[0]
    for k in ("flatland_step_time", "step_time", "last_time", "action_selection_time", "update_time",
              "reset_time", "reset_total_time"):
        assert getattr(env, k) > 0.0, k
    ph = model.batch.phase_seconds()
    assert abs(sum(ph.values()) - model.batch.timed_kernel_ms * 1e-3) <= 1e-6 * sum(ph.values())
    assert sum(models[1][1].batch.phase_seconds().values()) == 0.0  # the traced run was untimed
    for e in (0, 100, 255):
        q0, t0 = model.batch.q_raw(e)
        q1, t1 = models[1][1].batch.q_raw(e)
        assert np.array_equal(q0, q1) and np.array_equal(t0, t1), e
