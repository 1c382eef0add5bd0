"""bench.py's partitioned leg of N > 1 runs (configs[4] on the ranks' process group, bench.partition_leg): its
summary on the bench line, and what a failure of the leg does -- rank 0 prints the line with the leg's error and
every rank exits with bench.PARTITION_LEG_FAILED (never 0), whether the leg raised or hung.  Here partition_run
is replaced, so only the bench-side logic is exercised; tests/test_bench_launcher.py runs the real leg on four
host-build ranks."""
import time

import bench


def _fake_leg():
    return {"value": 1.5e8, "unit": "agent-env-steps/sec", "backend": "nccl", "world_size": 8,
            "parity": "ok", "parity_envs_checked": 2,
            "config": {"workload": "c5: 256 switches / 128 trains, ...", "rounds_per_step": 61.0,
                       "checkpoints_per_step": 7.0, "count_reads_per_step": 7.0, "segment_records": 4096,
                       "collectives_per_round": 2, "deferrals": 12}}


def test_leg_summary_on_rank0(monkeypatch):
    monkeypatch.setattr(bench, "partition_run", lambda *a, **k: _fake_leg())
    printed = []
    leg = bench.partition_leg(None, None, 8, 0, 0, "cuda", [0] * 8, {}, printed.append)
    assert not printed  # the caller prints the line
    assert leg["value"] == 1.5e8 and leg["backend"] == "nccl" and leg["parity"] == "ok"
    assert leg["segment_records"] == 4096 and leg["deferrals"] == 12 and leg["what"].startswith("configs[4]")
    assert leg["collectives_per_round"] == 2
    monkeypatch.setattr(bench, "partition_run", lambda *a, **k: None)
    assert bench.partition_leg(None, None, 8, 3, 0, "cuda", [0] * 8, None, printed.append) is None


def test_watchdog_prints_the_line_and_exits_nonzero(monkeypatch):
    exits = []
    monkeypatch.setattr(bench, "PARTITION_LEG_TIMEOUT_S", 0.2)
    monkeypatch.setattr(bench.os, "_exit", lambda code: exits.append(code))

    def hang(*a, **k):
        time.sleep(0.6)
        return _fake_leg()
    monkeypatch.setattr(bench, "partition_run", hang)
    printed, res = [], {"metric": "m", "value": 1.0}
    bench.partition_leg(None, None, 2, 0, 0, "cuda", [0, 0], res, printed.append)
    assert exits == [bench.PARTITION_LEG_FAILED] and bench.PARTITION_LEG_FAILED != 0
    assert len(printed) == 1 and "no result within" in printed[0]["partition_leg"]["error"]


def test_exception_on_rank0_prints_the_line_and_exits_nonzero(monkeypatch):
    exits = []
    monkeypatch.setattr(bench.os, "_exit", lambda code: exits.append(code))

    def boom(*a, **k):
        raise RuntimeError("rank 1: sfl_part_local: kernel fault")
    monkeypatch.setattr(bench, "partition_run", boom)
    printed, res = [], {"metric": "m", "value": 1.0}
    assert bench.partition_leg(None, None, 2, 0, 0, "cuda", [0, 0], res, printed.append) is None
    assert exits == [bench.PARTITION_LEG_FAILED]
    assert len(printed) == 1 and "kernel fault" in printed[0]["partition_leg"]["error"]
    assert printed[0]["value"] == 1.0  # the env-sharded measurement is still on the line


def test_exception_on_another_rank_waits_for_rank0_then_exits_nonzero(monkeypatch):
    held = []
    monkeypatch.setattr(bench, "_hold_then_exit", lambda s: held.append(s))

    def boom(*a, **k):
        raise RuntimeError("RCCL error")
    monkeypatch.setattr(bench, "partition_run", boom)
    printed = []
    bench.partition_leg(None, None, 2, 1, 0, "cuda", [0, 0], None, printed.append)
    assert not printed  # (rank 0 prints)
    # it waits past rank 0's watchdog before it ends, so the launcher does not stop rank 0 first
    assert len(held) == 1 and held[0] > bench.PARTITION_LEG_TIMEOUT_S
