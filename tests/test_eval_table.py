"""scripts/eval_table.py: plot.ipynb cell 15's train-arrival rule, and the script end to end on the host build
(main.py -c -> eval.py -> the rule on the files eval.py wrote)."""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))
import eval_table  # noqa: E402


def test_cell15_rule_literal():
    # trains 0, 2, 3 arrived; delays in train_to_last_node order (the rule pairs mask[h] with delays[h])
    assert eval_table.classify([-1.0, 5.0, 0.0, 2.0], [0, 2, 3], 4) == [2, 1, 1]
    assert eval_table.classify([3.0, 3.0], [], 2) == [0, 0, 2]
    # fewer delays than trains: cell 15's mask & delays cannot broadcast
    assert eval_table.classify([1.0], [0], 2) is None


def test_eval_table_end_to_end_host(tmp_path):
    out = tmp_path / "t.json"
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "eval_table.py"), str(out), "--host",
                        "--episodes", "30", "--seeds", "64", "--checkpoint-freq", "10", "--exploit-freq", "10",
                        "--work", str(tmp_path / "w")], cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.load(open(out))
    s = d["seeds"]["64"]
    assert s["evals"] == 10  # malfunctions on: eval.py's 10 evaluations
    rows = [x for x in s["table_per_eval"] if x is not None]
    assert rows and all(sum(x) == 15 for x in rows)
    # every evaluation resets with the learner's seed: the same episode each time
    assert len({tuple(x) for x in rows}) == 1 and len(set(s["eval_cum_reward"])) == 1
    t = d["table"]
    assert abs(t["early"] + t["late"] + t["not_arrived"] - 15) < 1e-9
    # the files eval.py wrote are the reference's
    ev = tmp_path / "w" / "seed_0" / "eval_0"
    assert np.load(ev / "delays.npz")["x"].shape == (15,)
    assert (ev / "trains_at_dest.npz").exists() and (ev / "cum_reward.npz").exists()
