"""Learning curve of the reference's hyper-parameter sweep config on the device.

hyperparam_tuning.py:10-35: 80 x 80 grid, max_num_cities 25, 15 trains, no malfunctions, 10,000 episodes,
exploit round every 100 episodes, seeds 64, 65, 66, 67, 69; epsilon 0.5, decay 0.9997, lr 0.1, lr decay
1.0, gamma 1, default_q 0.  Each seed is its own run (map and learner seeded by it, main.py:13-60), here
one device batch per seed (mapgen's stand-in for Flatland's sparse_rail_generator, which is absent).
Writes the per-episode arrived trains / cumulative reward of every seed and a summary to compare with
plot.ipynb cells 11 and 13 (mean arrived ~6 -> ~14.7 of 15 by ~6k episodes).

Each seed's final Q-table (compact Q block + key-set bitmap) is recorded as a SHA-1, and --compare REF.json
checks a run against another (e.g. the GPU against the host build): every episode's arrived trains, cumulative
reward and decisions, and the final Q-table digests, equal.

Usage: python scripts/learning_curve.py OUT.json [--episodes N] [--seeds 64,65,...] [--host] [--compare REF.json]
"""
import argparse
import gzip
import hashlib
import importlib
import json
import os
import sys
import time
import warnings

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "network-distributed-q-learning_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--episodes", type=int, default=10_000)
    ap.add_argument("--seeds", default="64,65,66,67,69")
    ap.add_argument("--exploit-freq", type=int, default=100)
    ap.add_argument("--chunk", type=int, default=500, help="episodes per learn call (progress lines)")
    ap.add_argument("--host", action="store_true", help="run the host build (tests only)")
    ap.add_argument("--rows", type=int, default=0, help="with --layout citygrid: city rows (0: what fits)")
    ap.add_argument("--cols", type=int, default=0, help="with --layout citygrid: city columns (0: what fits)")
    ap.add_argument("--layout", default="cities", choices=["cities", "grid", "citygrid"],
                    help="cities: main.py's [ENV] keys (mapgen.from_flatland_params, city stand-in); grid: a line-grid "
                         "stand-in with the same trains (mapgen.generate, 60 switches, 8 stations)")
    ap.add_argument("--rails", type=int, default=2, help="max_rails_between_cities (the sweep: 2)")
    ap.add_argument("--pairs", type=int, default=2, help="max_rail_pairs_in_city (the sweep: 2)")
    ap.add_argument("--compare", default=None, help="a previous run's OUT.json(.gz): per-episode results and final "
                                                    "Q-table digests must be equal")
    args = ap.parse_args()
    mapgen = importlib.import_module(PKG + ".mapgen")
    comp = importlib.import_module(PKG + ".compiler")
    runtime = importlib.import_module(PKG + ".runtime")
    lib = None
    if args.host:
        from tests import hostsim
        lib = hostsim.lib()
    hp = dict(gamma=1.0, epsilon=0.5, epsilon_decay_rate=0.9997, lr=0.1, lr_decay_rate=1.0, default_q=0.0)
    res = {"config": "hyperparam_tuning.py:10-35 (80x80, max_num_cities 25, max_rails_between_cities "
                     f"{args.rails}, max_rail_pairs_in_city {args.pairs}, 15 trains, no malfunctions)",
           "layout": args.layout,
           "episodes": args.episodes, "exploit_freq": args.exploit_freq, "hparams": hp, "seeds": {}}
    t_all = time.time()
    for seed in [int(s) for s in args.seeds.split(",")]:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            if args.layout == "cities":
                # the sweep's [ENV] keys (hyperparam_tuning.py:17-25), as main.py passes them
                sc = mapgen.from_flatland_params(80, 80, 25, 15, seed, malfunction=(0.0, 0, 0),
                                                 max_rails_between_cities=args.rails, max_rail_pairs_in_city=args.pairs)
            elif args.layout == "citygrid":
                sc = mapgen.generate_city_grid(args.rows or 4, args.cols or 2, 15, seed, rails=args.rails,
                                               track_choices=[2 * k for k in range(1, args.pairs + 1)], size=80)
            else:
                sc = mapgen.generate(60, 15, 8, seed=seed)
        cm = comp.compile_scenario(sc)
        b = runtime.Batch(cm, hp, [seed], lib=lib)
        t0 = time.time()
        arrived, cum, arr_x, cum_x, dec = [], [], [], [], []
        # one learn() call over all episodes, in chunks: the device keeps the learner's state (Q, epsilon
        # counters, RNG) across sfl_learn calls exactly as DistrQLearning.learn's loop does
        b.learn_begin()
        b.apply_qinit()
        done = 0
        while done < args.episodes:
            n = min(args.chunk, args.episodes - done)
            out = b._run(b.lib.dll.sfl_learn, n, args.exploit_freq)
            arrived += out["arrived"][:, 0].tolist()
            cum += out["cum_reward"][:, 0].tolist()
            dec += out["decisions"][:, 0].tolist()
            sel = (np.arange(done, done + n) + 1) % args.exploit_freq == 0
            arr_x += out["arrived_trains_exploit"][sel, 0].tolist()
            cum_x += out["cum_reward_exploit"][sel, 0].tolist()
            done += n
            print(f"seed {seed}: {done} episodes, mean arrived (last {n}) {np.mean(out['arrived'][:, 0]):.2f} / "
                  f"{cm.T}, {time.time() - t0:.1f} s", flush=True)
        q, t = b.q_raw(0)
        qsha = hashlib.sha1(np.ascontiguousarray(q).tobytes() + np.ascontiguousarray(t).tobytes()).hexdigest()
        kern = b.counters()
        b.close()
        res["seeds"][str(seed)] = dict(map=f"{sc.width}x{sc.height}, {cm.S} switches, {cm.T} trains, {cm.K} stations",
                                       arrived=arrived, cum_reward=cum, decisions=dec, arrived_exploit=arr_x,
                                       cum_reward_exploit=cum_x, seconds=time.time() - t0, q_sha1=qsha,
                                       library=os.path.basename(b.lib.path), kernel_variant=kern["kernel_variant"])
    A = np.array([v["arrived"] for v in res["seeds"].values()], dtype=float)
    w = max(1, args.episodes // 20)
    res["summary"] = {
        "mean_arrived_first_100": float(A[:, :100].mean()),
        "mean_arrived_by_window": [[int(i), float(A[:, i:i + w].mean())] for i in range(0, args.episodes, w)],
        "mean_arrived_last_500": float(A[:, -500:].mean()),
        "exploit_mean_arrived_last_5": float(np.mean([v["arrived_exploit"][-5:] for v in res["seeds"].values()])),
        "trains": 15, "wall_s": time.time() - t_all,
        "decisions_total": int(sum(sum(v["decisions"]) for v in res["seeds"].values())),
    }
    if args.compare:
        op = gzip.open if args.compare.endswith(".gz") else open
        ref = json.load(op(args.compare, "rt"))
        cmp = {}
        for k, v in res["seeds"].items():
            r = ref["seeds"].get(k)
            if r is None:
                cmp[k] = "missing in the reference run"
                continue
            same = {f: v[f] == r[f] for f in ("arrived", "cum_reward", "decisions", "arrived_exploit", "cum_reward_exploit")}
            same["q_sha1"] = v["q_sha1"] == r.get("q_sha1")
            cmp[k] = "equal" if all(same.values()) else "DIFFERENT: " + ", ".join(f for f, ok in same.items() if not ok)
        res["compare"] = {"reference": os.path.basename(args.compare), "seeds": cmp,
                          "all_equal": all(x == "equal" for x in cmp.values())}
        print(json.dumps(res["compare"]), flush=True)
    json.dump(res, open(args.out, "w"))
    print(json.dumps(res["summary"]), flush=True)


if __name__ == "__main__":
    main()
