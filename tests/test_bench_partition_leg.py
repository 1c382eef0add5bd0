"""bench.py's partitioned leg of N > 1 runs (configs[4] on the ranks' process group, bench.partition_leg): its
summary on the bench line, and the watchdog that prints the line and ends the rank when the leg hangs.  The leg
itself runs on GPUs (the --gpus 2 rehearsal on one GPU over gloo: profiles/r04k_gpus2_gloo_rehearsal.json); here
partition_run is replaced, so only the bench-side logic is exercised."""
import time

import bench


def _fake_leg():
    return {"value": 1.5e8, "unit": "agent-env-steps/sec", "backend": "nccl", "world_size": 8,
            "parity": "ok", "parity_envs_checked": 2,
            "config": {"workload": "c5: 256 switches / 128 trains, ...", "rounds_per_step": 61.0,
                       "checkpoints_per_step": 7.0, "count_reads_per_step": 7.0, "segment_records": [2048, 4096],
                       "deferrals": 12}}


def test_leg_summary_on_rank0(monkeypatch):
    monkeypatch.setattr(bench, "partition_run", lambda *a, **k: _fake_leg())
    printed = []
    leg = bench.partition_leg(None, None, 8, 0, 0, "cuda", [0] * 8, {}, printed.append)
    assert not printed  # the caller prints the line
    assert leg["value"] == 1.5e8 and leg["backend"] == "nccl" and leg["parity"] == "ok"
    assert leg["segment_records"] == [2048, 4096] and leg["deferrals"] == 12 and leg["what"].startswith("configs[4]")
    monkeypatch.setattr(bench, "partition_run", lambda *a, **k: None)
    assert bench.partition_leg(None, None, 8, 3, 0, "cuda", [0] * 8, None, printed.append) is None


def test_watchdog_prints_the_line_and_exits(monkeypatch):
    exits = []
    monkeypatch.setattr(bench, "PARTITION_LEG_TIMEOUT_S", 0.2)
    monkeypatch.setattr(bench.os, "_exit", lambda code: exits.append(code))

    def hang(*a, **k):
        time.sleep(0.6)
        return _fake_leg()
    monkeypatch.setattr(bench, "partition_run", hang)
    printed, res = [], {"metric": "m", "value": 1.0}
    bench.partition_leg(None, None, 2, 0, 0, "cuda", [0, 0], res, printed.append)
    assert exits == [0]
    assert len(printed) == 1 and "error" in printed[0]["partition_leg"]
