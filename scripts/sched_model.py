"""Scheduling model of run_groups' flat loop (k_wave_g, G = 16: four envs per wavefront).

Why: the round-2 verdict asked whether aligning decisions across the four lane groups of a wave would pay
(only ~2.96 of 4 groups decide per iteration).  A wavefront executes each divergent block of an iteration --
tick, prefetch, post + decide -- once for every group that takes it, so an iteration costs
    T * [some group ticks] + PF * [some group stages a batch] + D * [some group decides]
whatever the number of groups in each block.  This script replays real per-env decision streams (the
decision times of c3 learn runs on the host build of the kernel body, which the GPU matches bit-exactly:
consecutive decisions at one tick form a batch) through the loop's group state machine under a tick policy,
counts the blocks executed per decision, and prices them with T, PF, D calibrated on the v29 SFL_PROFILE
wall cycles (profiles/r02_v29_group_phases.txt: tick blocks 16 %, post + decide 84 % of wave time, the
prefetch section 23 % of decide).

Usage: python scripts/sched_model.py [n_envs] [episodes]  (writes the table to stdout)
"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
PKG = "network-distributed-q-learning_amd"
HP = dict(gamma=1.0, epsilon=0.5, epsilon_decay_rate=0.9997, lr=0.1, lr_decay_rate=1.0, default_q=0.0)  # bench.py
T_COST, D_COST, PF_COST = 50.0, 27.0, 31.0  # relative block costs (calibration in the docstring)


def streams(n_envs, episodes):
    """Per env: [(ticks since the previous batch, decisions in the batch)] of a c3 learn run."""
    mapgen = importlib.import_module(PKG + ".mapgen")
    comp = importlib.import_module(PKG + ".compiler")
    runtime = importlib.import_module(PKG + ".runtime")
    import hostsim
    cm = comp.compile_scenario(mapgen.make_config("c3"))
    out = []
    for i in range(n_envs):
        b = runtime.Batch(cm, HP, [450565 + i], lib=hostsim.lib())
        b.trace_env, b.trace_cap = 0, 1 << 20
        b.learn(episodes)
        now = (b.last_trace[:, 0] & 0xFFFF).astype(np.int64)
        b.close()
        now = np.where(now >= 0x8000, now - 0x10000, now)
        ev, prev, i0 = [], 0, 0
        while i0 < len(now):
            j = i0
            while j < len(now) and now[j] == now[i0]:
                j += 1
            t = int(now[i0])
            ev.append((t - prev if t > prev else t + 1, j - i0))  # (an episode restarts at tick 0)
            prev, i0 = t, j
        out.append(ev)
    return out


def run(S, policy, seed, ndec=4096, G=4, ring=10):
    """One wavefront of G groups on random envs / offsets: blocks executed until every group made ndec
    decisions.  Returns (iterations, tick blocks, decide blocks, prefetch blocks, decisions)."""
    rng = np.random.default_rng(seed)
    envs = rng.choice(len(S), G, replace=False)
    pos = [int(rng.integers(0, len(S[e]) // 2)) for e in envs]
    q, tleft, stage, done = [0] * G, [S[envs[g]][pos[g]][0] for g in range(G)], [0] * G, [0] * G
    it = nt = nd = npf = 0
    while min(done) < ndec:
        it += 1
        tick = policy(q)
        anyt = False
        for g in range(G):
            if tick and q[g] == 0:
                anyt = True
                tleft[g] -= 1
                if tleft[g] == 0:
                    q[g], stage[g] = S[envs[g]][pos[g]][1], 0
                    pos[g] = (pos[g] + 1) % len(S[envs[g]])
                    tleft[g] = S[envs[g]][pos[g]][0]
        anyd = anypf = False
        for g in range(G):
            if q[g] > 0:
                anyd = True
                anypf |= stage[g] % ring == 0  # staged after the tick and again when the ring is used up
                stage[g] += 1
                q[g] -= 1
                done[g] += 1
        nt, nd, npf = nt + anyt, nd + anyd, npf + anypf
    return np.array([it, nt, nd, npf, sum(done)], dtype=float)


def hold(h):  # the product rule (SFL_TICK_HOLD): waiting groups tick once fewer than h groups decide
    return lambda q: sum(x > 0 for x in q) < h


def remmin(r, h=2):  # SFL_TICK_REMMIN: ... or while every deciding group has >= r decisions left
    return lambda q: sum(x > 0 for x in q) < h or min(x for x in q if x > 0) >= r


def main():
    n_envs = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    episodes = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    S = streams(n_envs, episodes)
    ks = [k for s in S for _, k in s]
    gaps = [g for s in S for g, _ in s]
    print(f"c3 learn streams: {n_envs} envs x {episodes} episodes, {len(ks)} batches, {np.mean(ks):.2f} decisions per "
          f"batch, {sum(ks) / sum(gaps):.2f} decisions per tick")
    pols = {"hold1": hold(1), "hold2 (product)": hold(2), "hold3": hold(3), "hold5 (never hold)": hold(5)}
    pols.update({f"remmin{r}": remmin(r) for r in (3, 5, 7, 9)})
    print(f"cost = {T_COST:g} * ticks + {D_COST:g} * decide blocks + {PF_COST:g} * prefetch blocks, per decision")
    print(f"{'policy':20s} {'iter/dec':>8s} {'tick/dec':>8s} {'pf/dec':>8s} {'cost':>7s} {'vs product':>10s}")
    rows = {}
    for name, p in pols.items():
        a = sum(run(S, p, sd) for sd in range(24))
        it, nt, nd, npf, dec = a / (a[4] / 4.0)  # per group decision
        rows[name] = (it, nt, npf, T_COST * nt + D_COST * nd + PF_COST * npf)
    base = rows["hold2 (product)"][3]
    for name, (it, nt, npf, c) in rows.items():
        print(f"{name:20s} {it:8.3f} {nt:8.3f} {npf:8.3f} {c:7.2f} {base / c:10.3f}")
    print("lower bound (every block with all four groups): iter/dec 1.000, tick/dec = prefetch/dec = 1 / (decisions "
          f"per tick) -> cost {T_COST / 7.2 + D_COST + PF_COST / 7.2:.2f}")


if __name__ == "__main__":
    main()
