"""The reference's published evaluation table, reproduced through the entry points.

plot.ipynb cell 15 (`barplot`) classifies every train of every greedy evaluation run from the run's
``eval_<i>/delays.npz`` and ``eval_<i>/trains_at_dest.npz`` (written by DistrQLearning.test, distr_q.py:229-239):

    mask[trains_at_dest] = True
    early = sum(mask & (delays <= 0));  late = sum(mask & (delays > 0));  not_arrived = sum(~mask)

and cells 21-23 report the mean over 3 seeds x 10 evaluations of the 15-train sweep config with malfunctions
("15_agents_hp_malf_easy"): 10.9 early / 1.6 late / 2.5 not arrived.  Cells 16-20 do the same for the
100-train challenge: 26.4 / 2.4 / 71.2.

What runs here, per seed: the sweep's config.ini as hyperparam_tuning.py:49-82 writes it (80 x 80,
max_num_cities 25, max_rails_between_cities 2, max_rail_pairs_in_city 2, 15 trains, epsilon 0.5, decay 0.9997,
lr 0.1, gamma 1, default_q 0, 10,000 episodes, checkpoint every 1,000, exploit every 100) with malfunctions
(default: test_model.py:14-18's rate 0.01, 5-15 ticks -- the "easy" sweep's own parameters are not in the
reference), then ``main.launch_experiment`` (main.py -c) and ``eval.evaluate`` (eval.py: 10 greedy evaluations
when malfunctions are on, eval.py:85-97), all through libsfl.so, then cell 15's rule on the files eval.py wrote.

Notes on the rule, applied literally: ``delays`` is ``train_to_last_node``'s values in insertion order (the order
in which trains first decided, distr_q.py:230), not handle order, so cell 15 pairs ``mask[h]`` with another train's
delay whenever those orders differ; the table reports the literal rule, as the published numbers came from it.
A run in which a train never decides has fewer delays than trains, and cell 15 would fail on it (reported as such).
Every evaluation resets with the learner's seed (distr_q.py:195), so the 10 evaluations of one model are the same
episode unless the malfunction stream differs between resets (it does not, here or in Flatland reseeded by
``reset(random_seed)``).

Usage: python scripts/eval_table.py OUT.json [--episodes N] [--seeds 64,65,66] [--mf 0.01,5,15] [--host]
                                   [--work DIR] [--compare REF.json] [--trains 15] [--size 80] [--cities 25]
"""
import argparse
import configparser
import hashlib
import importlib
import json
import os
import pickle
import sys
import tempfile
import time
import warnings

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# plot.ipynb cells 21-23 / 16-20 (bar labels): mean trains per evaluation, early / late / not arrived
PUBLISHED = {15: dict(early=10.9, late=1.6, not_arrived=2.5, what="plot.ipynb cell 23, 15 trains with malfunctions, "
                                                                   "3 seeds x 10 evaluations"),
             100: dict(early=26.4, late=2.4, not_arrived=71.2, what="plot.ipynb cells 16-20, the 100-train challenge, "
                                                                     "5 seeds x 1 evaluation")}


HP_SWEEP = dict(gamma=1.0, epsilon=0.5, epsilon_decay_rate=0.9997, lr=0.1, lr_decay_rate=1.0, default_q=0.0)


def classify(delays, trains_at_dest, n_trains):
    """plot.ipynb cell 15, literally: (early, late, not_arrived), or None when cell 15 would fail (fewer delays than
    trains: its mask & delays cannot broadcast)."""
    delays = np.asarray(delays, dtype=float)
    mask = np.zeros(n_trains).astype(bool)
    mask[np.asarray(trains_at_dest, dtype=np.int64)] = True
    if delays.shape != mask.shape:
        return None
    return [int(np.sum(mask & (delays <= 0))), int(np.sum(mask & (delays > 0))), int(np.sum(~mask))]


def write_config(path, exp_dir, seed, args):
    """hyperparam_tuning.py:49-82's config.ini (its keys and values; the sweep's malfunction keys set)."""
    c = configparser.ConfigParser()
    c["MISC"] = {"random_seed": seed, "out_dir": exp_dir, "checkpoint_freq": args.checkpoint_freq,
                 "exploit_freq": args.exploit_freq}
    c["ENV"] = {"width": args.size, "height": args.size, "max_num_cities": args.cities,
                "max_rails_between_cities": 2, "max_rail_pairs_in_city": 2, "number_of_agents": args.trains,
                "malfunction_rate": args.mf[0], "min_duration": int(args.mf[1]), "max_duration": int(args.mf[2])}
    c["MODEL"] = {"gamma": 1.0, "epsilon": 0.5, "epsilon_decay_rate": 0.9997, "lr": 0.1, "lr_decay_rate": 1.0,
                  "default_q": 0.0, "num_episodes": args.episodes}
    with open(path, "w") as f:
        c.write(f)


def q_digest(model_path):
    """SHA-1 of the saved Q-table (the reference's pickle format: {tuple(obs): [q...]}), keys sorted."""
    with open(model_path, "rb") as f:
        q = pickle.load(f)  # (a file this script's own run just wrote)
    h = hashlib.sha1()
    for k in sorted(q):
        h.update(np.asarray(k, np.int64).tobytes() + np.asarray(q[k], np.float64).tobytes())
    return h.hexdigest(), len(q)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--episodes", type=int, default=10_000)
    ap.add_argument("--seeds", default="64,65,66", help="hyperparam_tuning.py:10's first three (cell 21: seed_0..2)")
    ap.add_argument("--mf", default="0.01,5,15", help="malfunction rate, min, max duration")
    ap.add_argument("--trains", type=int, default=15)
    ap.add_argument("--size", type=int, default=80)
    ap.add_argument("--cities", type=int, default=25)
    ap.add_argument("--checkpoint-freq", type=int, default=1000)
    ap.add_argument("--exploit-freq", type=int, default=100)
    ap.add_argument("--host", action="store_true", help="the host build of the kernel body (tests / the reference run)")
    ap.add_argument("--work", default=None, help="experiment directories (default: a temporary directory)")
    ap.add_argument("--compare", default=None, help="another run's OUT.json: per-seed Q digests and tables must match")
    args = ap.parse_args()
    a = args.mf.split(",")
    args.mf = (float(a[0]), int(a[1]), int(a[2]))
    lib = None
    if args.host:
        from tests import hostsim
        lib = hostsim.lib()
    import main as entry_main
    import eval as entry_eval

    work = args.work or tempfile.mkdtemp(prefix="sfl_eval_")
    # a progress line every 30 s (a learn() call of many episodes prints nothing until its first checkpoint)
    import threading
    t_start = time.time()

    def heartbeat():
        while True:
            time.sleep(30)
            print(f"... {time.time() - t_start:.0f} s", flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    res = {"config": f"hyperparam_tuning.py:17-35 keys: {args.size} x {args.size}, max_num_cities {args.cities}, "
                     f"max_rails_between_cities 2, max_rail_pairs_in_city 2, {args.trains} trains, malfunctions "
                     f"{args.mf}, {args.episodes} episodes, checkpoint {args.checkpoint_freq}, exploit {args.exploit_freq}",
           "library": "libsfl_hostsim.so (host build)" if args.host else "libsfl.so (HIP, gfx950)",
           "rule": "plot.ipynb cell 15: mask[trains_at_dest] = True; early = mask & (delays <= 0), late = mask & "
                   "(delays > 0), not arrived = ~mask",
           "seeds": {}}
    t_all = time.time()
    rows = []
    for i, seed in enumerate(int(s) for s in args.seeds.split(",")):
        exp_dir = os.path.join(work, f"seed_{i}")
        os.makedirs(exp_dir, exist_ok=True)
        cfg = os.path.join(exp_dir, "config.ini")
        write_config(cfg, exp_dir, seed, args)
        t0 = time.time()
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            entry_main.launch_experiment(cfg, lib=lib)
            t_learn = time.time() - t0
            runs = entry_eval.evaluate([exp_dir], lib=lib)[exp_dir]
        n_ev = len(runs)
        per = []
        for k in range(n_ev):
            d = os.path.join(exp_dir, f"eval_{k}")
            delays = np.load(os.path.join(d, "delays.npz"))["x"]
            at = np.load(os.path.join(d, "trains_at_dest.npz"))["x"]
            row = classify(delays, at, args.trains)
            per.append(row)
            if row is not None:
                rows.append(row)
        arrived_learn = np.load(os.path.join(exp_dir, "arrived_trains.npz"))["x"]
        qd, nkeys = q_digest(os.path.join(exp_dir, "distr_q_model.pkl"))
        kern = None
        if not args.host:  # the device kernel this map runs on (k_wave variant, lanes per env)
            import configparser as _cp
            runtime = importlib.import_module("network-distributed-q-learning_amd.runtime")
            comp = importlib.import_module("network-distributed-q-learning_amd.compiler")
            c = _cp.ConfigParser()
            c.read(cfg)
            kb = runtime.Batch(comp.compile_scenario(entry_main.build_scenario(c)), HP_SWEEP, [seed])
            cn = kb.counters()
            kern = {"kernel_variant": cn["kernel_variant"], "group_lanes": cn["group_lanes"]}
            kb.close()
        cr, arr, dl = runs[0]
        res["seeds"][str(seed)] = dict(
            evals=n_ev, table_per_eval=per, eval_cum_reward=[float(r[0]) for r in runs],
            eval_arrived=[int(r[1]) for r in runs], eval_delays_first=[float(x) for x in dl],
            learn_mean_arrived_last_500=float(np.mean(arrived_learn[-500:])), q_sha1=qd, q_keys=nkeys, kernel=kern,
            learn_seconds=t_learn, seconds=time.time() - t0)
        print(f"seed {seed}: learn {t_learn:.1f} s, last-500 mean arrived {np.mean(arrived_learn[-500:]):.2f} / "
              f"{args.trains}; eval {per[0]} x {n_ev}, Q {qd[:12]} ({nkeys} keys)", flush=True)
    H = np.array(rows, dtype=float) if rows else np.zeros((0, 3))
    res["table"] = {"early": float(H[:, 0].mean()) if len(H) else None,
                    "late": float(H[:, 1].mean()) if len(H) else None,
                    "not_arrived": float(H[:, 2].mean()) if len(H) else None,
                    "sem": (H.std(axis=0) / np.sqrt(max(1, len(H)))).tolist() if len(H) else None,
                    "rows": len(H), "rows_cell15_would_fail": sum(v is None for s in res["seeds"].values()
                                                                 for v in s["table_per_eval"])}
    res["published"] = PUBLISHED.get(args.trains)
    res["wall_s"] = time.time() - t_all
    if args.compare:
        ref = json.load(open(args.compare))
        cmp = {}
        for k, v in res["seeds"].items():
            r = ref["seeds"].get(k)
            cmp[k] = ("missing" if r is None else
                      "equal" if (v["q_sha1"] == r["q_sha1"] and v["table_per_eval"] == r["table_per_eval"]
                                  and v["eval_cum_reward"] == r["eval_cum_reward"]) else "DIFFERENT")
        res["compare"] = {"reference": os.path.basename(args.compare), "seeds": cmp,
                          "all_equal": all(x == "equal" for x in cmp.values())}
        print(json.dumps(res["compare"]), flush=True)
    json.dump(res, open(args.out, "w"), indent=1)
    print(json.dumps({"table": res["table"], "published": res["published"], "wall_s": res["wall_s"]}), flush=True)


if __name__ == "__main__":
    main()
