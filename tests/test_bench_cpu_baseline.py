"""bench.py's reference-speed CPU baseline (cpu_oracle_baseline): the oracle's learn loop as one process per
granted host core, one env each (the reference's one-process-per-seed scale-out, hyperparam_tuning.py:85-91),
with the 1-core figure kept -- run here with two processes for a second each."""
import bench


def test_oracle_baseline_one_process_per_core():
    pool = bench.start_oracle_pool(2)
    try:
        out = bench.cpu_oracle_baseline("c1", 1.0, pool=pool)
    finally:
        pool.close()
        pool.join()
    assert out["cores"] == 2 and out["kind"] == "port" and out["unit"] == "agent-env-steps/sec"
    assert out["value"] > out["one_core_value"] > 0
    assert "2 process(es)" in out["sample"] and "1 core:" in out["sample"]
    assert bench.oracle_cores() >= 1


def test_oracle_pool_lost_worker_fails_without_respawn():
    """a worker that dies is never replaced (a respawn is a fork + exec, which a GPU-initialised process
    must not do) and the baseline fails instead of waiting forever."""
    import os
    import signal

    import pytest
    pool = bench.start_oracle_pool(2)
    pids = [p.pid for p in pool.procs]
    os.kill(pids[1], signal.SIGKILL)
    pool.procs[1].join(timeout=30)
    try:
        with pytest.raises(RuntimeError, match="died without a result"):
            bench.cpu_oracle_baseline("c1", 5.0, pool=pool)
        assert [p.pid for p in pool.procs] == pids  # nothing was started in its place
    finally:
        pool.close()
