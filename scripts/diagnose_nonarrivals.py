"""Attribute every non-arrival of the greedy policy on the reference's sweep config.

Learns ``--episodes`` episodes of the sweep config (hyperparam_tuning.py:10-35: 80 x 80, max_num_cities 25,
15 trains, no malfunctions) for each seed on the host build of the kernel body (bit-equal to the GPU), loads
the learned Q-table into the oracle (oracle/sfl_oracle.py, the CPU restatement) and replays one greedy
episode (the exploit round, distr_q.py:184-241) tick by tick, recording every train's state.  Each train that
does not arrive is classified:

  never_departed   still WAITING / READY_TO_DEPART at the end (never entered the map)
  deadlock         on the map, not moving over the last ``--stall`` ticks, and its next cell is held by another
                   stalled train (a head-on pair or a cycle of blocked trains)
  stop_loop        on the map, stalled, next cell free: the policy keeps choosing STOP at its switch
  moving_late      still moving at the end (the episode's tick horizon max_episode_steps ran out)
  truncated        the episode was cut by max_steps decisions (switch_env.py:652-657)

Usage: python scripts/diagnose_nonarrivals.py OUT.json [--seeds 64,66] [--episodes 10000] [--layout cities]
"""
import argparse
import importlib
import json
import os
import sys
import time
import warnings
from collections import Counter

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "network-distributed-q-learning_amd"
HP = dict(gamma=1.0, epsilon=0.5, epsilon_decay_rate=0.9997, lr=0.1, lr_decay_rate=1.0, default_q=0.0)


def scenario(mapgen, layout, seed, **kw):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        if layout == "cities":
            return mapgen.from_flatland_params(80, 80, 25, 15, seed, malfunction=(0.0, 0, 0), **kw)
        if layout.startswith("citygrid"):  # citygrid[RxC]
            rc = layout[8:] or "4x2"
            r, c = (int(x) for x in rc.split("x"))
            return mapgen.generate_city_grid(r, c, 15, seed, rails=kw.get("max_rails_between_cities", 2),
                                             track_choices=[2 * k for k in range(1, kw.get("max_rail_pairs_in_city", 2) + 1)],
                                             size=80)
        return mapgen.generate(60, 15, 8, seed=seed)


def learn_host(cm, seed, episodes, exploit_freq, lib):
    runtime = importlib.import_module(PKG + ".runtime")
    b = runtime.Batch(cm, HP, [seed], lib=lib)
    b.learn_begin()
    b.apply_qinit()
    arrived = []
    done = 0
    while done < episodes:
        n = min(2000, episodes - done)
        out = b._run(b.lib.dll.sfl_learn, n, exploit_freq)
        arrived += out["arrived"][:, 0].tolist()
        done += n
    q = b.q_dict(0)
    b.close()
    return q, arrived


def greedy_episode(sc, seed, q, stall):
    from oracle import flatland_lite as fl
    from oracle import sfl_oracle as so
    env, model = so.build(sc, seed, HP, trace=False)
    model.q = {tuple(k): list(v) for k, v in q.items()}
    ticks = []  # per tick: [(state, position)] per train
    orig = env.rail_env.step

    def step(actions):
        r = orig(actions)
        ticks.append([(a.state, a.position, a.direction) for a in env.rail_env.agents])
        return r
    env.rail_env.step = step
    cum, arrived, delays = model.test()
    rail = env.rail_env
    T = len(rail.agents)
    end_tick = rail._elapsed_steps
    horizon = rail._max_episode_steps
    out = {"arrived": arrived, "ticks": end_tick, "max_episode_steps": horizon, "truncated": bool(env.truncated),
           "cum_reward": cum, "trains": {}}
    last = ticks[-1] if ticks else []
    held = {}
    for h, (st, pos, d) in enumerate(last):
        if pos is not None:
            held[tuple(pos)] = h
    stalled = set()
    for h in range(T):
        st, pos, d = last[h]
        if pos is None:
            continue
        window = [tk[h][1] for tk in ticks[-stall:]]
        if all(p == pos for p in window):
            stalled.add(h)
    for h in range(T):
        st, pos, d = last[h]
        if st == fl.TrainState.DONE:
            continue
        if env.truncated:
            cls = "truncated"
        elif pos is None:
            cls = "never_departed"
        elif h not in stalled:
            cls = "moving_late"
        else:
            # the cell this train would enter next along its current heading / plan
            nxt = None
            for act in (fl.RailEnvActions.MOVE_FORWARD, fl.RailEnvActions.MOVE_LEFT, fl.RailEnvActions.MOVE_RIGHT):
                ok = fl.action_valid(rail.rail, act, pos, d)
                if ok:
                    _, (p2, _), _, _ = rail.rail.check_action_on_agent(act, (pos, d))
                    if tuple(p2) in held and held[tuple(p2)] in stalled:
                        nxt = held[tuple(p2)]
                        break
            cls = "deadlock" if nxt is not None else "stop_loop"
        out["trains"][h] = {"class": cls, "state": str(st), "position": list(pos) if pos else None,
                            "earliest_departure": rail.agents[h].earliest_departure,
                            "latest_arrival": rail.agents[h].latest_arrival}
    out["summary"] = dict(Counter(v["class"] for v in out["trains"].values()))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--seeds", default="64,66")
    ap.add_argument("--episodes", type=int, default=10_000)
    ap.add_argument("--exploit-freq", type=int, default=100)
    ap.add_argument("--stall", type=int, default=30)
    ap.add_argument("--layout", default="cities")
    ap.add_argument("--rails", type=int, default=None, help="max_rails_between_cities")
    ap.add_argument("--pairs", type=int, default=None, help="max_rail_pairs_in_city")
    args = ap.parse_args()
    from tests import hostsim
    mapgen = importlib.import_module(PKG + ".mapgen")
    comp = importlib.import_module(PKG + ".compiler")
    kw = {}
    if args.rails is not None:
        kw["max_rails_between_cities"] = args.rails
    if args.pairs is not None:
        kw["max_rail_pairs_in_city"] = args.pairs
    res = {"config": "hyperparam_tuning.py:10-35", "layout": args.layout, "episodes": args.episodes, "map_kw": kw,
           "seeds": {}}
    for seed in [int(s) for s in args.seeds.split(",")]:
        t0 = time.time()
        sc = scenario(mapgen, args.layout, seed, **kw)
        cm = comp.compile_scenario(sc)
        q, arrived = learn_host(cm, seed, args.episodes, args.exploit_freq, hostsim.lib())
        d = greedy_episode(sc, seed, q, args.stall)
        d["map"] = f"{sc.width}x{sc.height}, {cm.S} switches, {cm.T} trains, {cm.K} stations"
        d["learn_mean_arrived_last_500"] = float(np.mean(arrived[-500:]))
        d["learn_mean_arrived_first_500"] = float(np.mean(arrived[:500]))
        res["seeds"][str(seed)] = d
        print(f"seed {seed}: {d['map']}; greedy arrived {d['arrived']}/{cm.T}, ticks {d['ticks']}/"
              f"{d['max_episode_steps']}, non-arrivals {d['summary']}, learn last-500 mean "
              f"{d['learn_mean_arrived_last_500']:.2f} ({time.time() - t0:.0f} s)", flush=True)
    json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
