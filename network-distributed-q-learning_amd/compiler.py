"""Host-side map compiler: ``mapgen.Scenario`` -> flat tables for the HIP kernels.

Init-time only (the reference does the same work once per env construction:
RailNetwork(rail_env), rail_network.py:85-133).  Produces, in the reference's own
numbering:

* switches in ``pandas.groupby('switch_id')`` order (rail_network.py:38), each with
  its ports in ``get_port_nodes()`` order and its actions in ``action_outcomes``
  order.  That order is the iteration order of a networkx subgraph, which for a
  small subgraph is the iteration order of a Python ``set`` of float port tuples
  inserted in graph order.  We reproduce it by replaying the
  insertion order of rail_graph.py:13-136 and asking CPython for the set order;
* per global port id ``g = 4*switch + slot``: rail neighbour, rail-segment length
  (``len(rail_nodes)``), side (``map_direction``), the unique onward port used by
  transition_semaphore (rail_network.py:355-402);
* per train: start cell/heading, station index, ED/LA, the port + distance that
  ``_init_ports`` finds (switch_env.py:507-568), the reset delay (observer.py:38-39);
* per station: the patched-DistanceMap BFS (flatland_patch/distance_map.py:62-167)
  as int32 with ``DIST_INF``;
* the compact Q layout: per (switch, in-port slot) a block of
  ``2^P * K * 3`` rows of ``routes(slot)+1`` doubles;
* the ``__init_q_table`` patch (distr_q.py:81-181) as compact rows.
"""
from __future__ import annotations

import functools
import itertools
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from .mapgen import Scenario, transitions, DELTA

DIST_INF = 0x3FFFFFFF
NTAB = 1 << 20
N_, E_, S_, W_ = 0, 1, 2, 3
# port-name digit (rail_graph.py:92-97) for the side of the switch cell the port sits on
SIDE_DIGIT = {E_: 1, N_: 2, W_: 3, S_: 4}
DIGIT_SIDE = {v: k for k, v in SIDE_DIGIT.items()}
SUFFIX = {1: 0.1, 2: 0.2, 3: 0.3, 4: 0.4}
ACT_LEFT, ACT_FWD, ACT_RIGHT, ACT_STOP = 1, 2, 3, 4


def port_tuple(cell: Tuple[int, int], side: int) -> Tuple[float, float]:
    s = SUFFIX[SIDE_DIGIT[side]]
    return (int(cell[0]) + s, int(cell[1]) + s)


@dataclass
class CompiledMap:
    scenario: Scenario
    H: int
    W: int
    S: int
    T: int
    K: int
    switch_ids: List[Tuple[int, int]]
    ports: List[List[Tuple[float, float]]]          # per switch, get_port_nodes() order
    outcomes: List[List[Tuple[int, int]]]           # per switch: (src slot, dst slot) per route action
    n_actions: np.ndarray                           # [S] incl. STOP
    stations: List[Tuple[int, int]]
    arrays: Dict[str, np.ndarray] = field(default_factory=dict)
    q_per_env: int = 0
    rows_per_env: int = 0
    qinit_rows: Dict[Tuple[int, int, int], np.ndarray] = field(default_factory=dict)  # (switch, slot, state) -> compact row

    # ------------------------------------------------------------------
    def port_id(self, s: int, slot: int) -> int:
        return 4 * s + slot

    def obs_of_row(self, s: int, slot: int, state: int) -> Tuple[int, ...]:
        """Observation tuple (observer.py:303-306) of a compact row."""
        P = len(self.ports[s])
        lvl = state % 3
        k = (state // 3) % self.K
        bits = state // (3 * self.K)
        sem = [(bits >> j) & 1 for j in range(P)]
        tgt = [-1] * (2 * P)
        tgt[2 * slot], tgt[2 * slot + 1] = self.stations[k]
        dl = [-1] * P
        dl[slot] = lvl
        r, c = self.switch_ids[s]
        return (r, c, *sem, *tgt, *dl)


def _graph_port_orders(grid: np.ndarray):
    """Per junction cell: port tuples in rail-graph insertion order, plus the total port count."""
    H, W = grid.shape
    adj: Dict[Tuple[int, int], List[Tuple[int, int]]] = {}
    order: List[Tuple[int, int]] = []

    def node(c):
        if c not in adj:
            adj[c] = []
            order.append(c)

    # rail_graph.py:19-86: scan (row, col, heading), link the cell to every cell it can exit into
    for r in range(H):
        for c in range(W):
            w = int(grid[r, c])
            if w == 0:
                continue
            for h in range(4):
                for e, ok in enumerate(transitions(w, h)):
                    if not ok:
                        continue
                    nr, nc = r + DELTA[e][0], c + DELTA[e][1]
                    if not (0 <= nr < W and 0 <= nc < H):
                        continue
                    node((r, c))
                    node((nr, nc))
                    if (nr, nc) not in adj[(r, c)]:
                        adj[(r, c)].append((nr, nc))
                        adj[(nr, nc)].append((r, c))
    # rail_graph.py:99-135: every non-degree-2 cell, in node order, turns its neighbours into ports.
    # Entries are ("cell", (r,c)) or ("port", side-of-owner) — a processed junction Y replaces its
    # entry in an adjacent junction X's list by Y's port, appended at the end.
    lists = {c: [("cell", n) for n in adj[c]] for c in order}
    junctions = [c for c in order if len(adj[c]) != 2]
    port_orders: Dict[Tuple[int, int], List[Tuple[float, float]]] = {}
    for x in junctions:
        plist = []
        for kind, ref in lists[x]:
            other = ref if kind == "cell" else ref[0]
            side = {(-1, 0): N_, (0, 1): E_, (1, 0): S_, (0, -1): W_}[(other[0] - x[0], other[1] - x[1])]
            plist.append(port_tuple(x, side))
            if kind == "cell" and len(adj[other]) != 2:
                lst = lists[other]
                idx = next(i for i, (k2, r2) in enumerate(lst) if k2 == "cell" and r2 == x)
                del lst[idx]
                lst.append(("port", (x,)))
        port_orders[x] = plist
    total = sum(len(v) for v in port_orders.values())
    return port_orders, total


def _bfs_distance(grid: np.ndarray, target: Tuple[int, int]) -> np.ndarray:
    """Reverse BFS over (cell, heading) — the patched DistanceMap semantics."""
    from collections import deque
    H, W = grid.shape
    d = np.full((H, W, 4), DIST_INF, dtype=np.int64)
    tr, tc = target
    d[tr, tc, :] = 0
    q = deque()
    done = {(tr, tc, o) for o in range(4)}

    def expand(r, c, dist, heading):
        dirs = range(4) if heading < 0 else [(heading + 2) % 4]
        out = []
        for nd in dirs:
            pr, pc = r + DELTA[nd][0], c + DELTA[nd][1]
            if not (0 <= pr < H and 0 <= pc < W):
                continue
            move = (nd + 2) % 4
            w = int(grid[pr, pc])
            for o in range(4):
                if transitions(w, o)[move]:
                    nv = min(int(d[pr, pc, o]), dist + 1)
                    d[pr, pc, o] = nv
                    out.append((pr, pc, o, nv))
        return out

    q.extend(expand(tr, tc, 0, -1))
    while q:
        r, c, o, dist = q.popleft()
        if (r, c, o) in done:
            continue
        done.add((r, c, o))
        q.extend(expand(r, c, dist, o))
    return d


def _check_action(grid, action, cell, heading):
    """flatland-lite ``check_action_on_agent`` (the frozen Flatland spec) on the host."""
    H, W = grid.shape
    tr = transitions(int(grid[cell]), heading)
    n = sum(tr)
    nd, valid = heading, None
    if action == ACT_LEFT:
        nd = heading - 1
        if n <= 1:
            valid = False
    elif action == ACT_RIGHT:
        nd = heading + 1
        if n <= 1:
            valid = False
    nd %= 4
    if action == ACT_FWD and n == 1:
        nd = tr.index(1)
        valid = True
    ncell = (cell[0] + DELTA[nd][0], cell[1] + DELTA[nd][1])
    ok = 0 <= ncell[0] < H and 0 <= ncell[1] < W and grid[ncell] != 0
    if valid is None:
        valid = bool(tr[nd])
    return ncell, nd, bool(valid), bool(ok)


def _valid_moves(grid, cell, heading):
    """[left, forward, right] successors (get_valid_move_actions_)."""
    tr = transitions(int(grid[cell]), heading)
    n = sum(tr)
    res = []
    for i in (-1, 0, 1):
        nd = (heading + i) % 4
        if tr[nd]:
            act = ACT_FWD if (n == 1 or i == 0) else (ACT_RIGHT if i == 1 else ACT_LEFT)
            res.append((act, (cell[0] + DELTA[nd][0], cell[1] + DELTA[nd][1]), nd))
    return res


def compile_scenario(sc: Scenario) -> CompiledMap:
    grid = sc.grid_array()
    H, W = grid.shape
    if H != W:
        raise ValueError("square maps only (rail_graph.py:45-47 swaps width/height)")
    port_orders, n_ports_total = _graph_port_orders(grid)
    for x, pl in port_orders.items():
        if len(pl) < 3:
            raise ValueError(f"dead end / degenerate junction at {x}")
    switch_ids = sorted(port_orders)
    S = len(switch_ids)
    sidx = {x: i for i, x in enumerate(switch_ids)}
    if 4 * S >= 0xFFFF:
        raise ValueError("too many switches")

    ports, outcomes, turns, n_actions = [], [], [], []
    for x in switch_ids:
        pl = port_orders[x]
        order = list(set(pl)) if 2 * len(pl) < n_ports_total else list(pl)
        keys = [int(str(p[0])[-1]) for p in order]
        if len(set(keys)) != len(keys):
            raise ValueError(f"port-digit collision at switch {x}")
        ports.append(order)
        w = int(grid[x])
        sides = [DIGIT_SIDE[round((p[0] - int(p[0])) * 10)] for p in order]
        outs, trn = [], []
        for i, si in enumerate(sides):
            for j, sj in enumerate(sides):
                if i == j:
                    continue
                conn = transitions(w, (si + 2) % 4)[sj] or transitions(w, (sj + 2) % 4)[si]
                if not conn:
                    continue
                di, dj = SIDE_DIGIT[si] - 1, SIDE_DIGIT[sj] - 1
                t = {1: ACT_RIGHT, 2: ACT_FWD, 3: ACT_LEFT}.get((dj - di) % 4)
                if t is None:
                    raise ValueError("U-turn route")
                outs.append((i, j))
                trn.append(t)
        key = (len(order), len(outs))
        na = {(3, 4): 5, (4, 4): 5, (4, 6): 7, (4, 8): 9}.get(key)
        if na is None:
            raise ValueError(f"No Agent with n_gaits={key[0]} and n_rails={key[1]}")
        outcomes.append(outs)
        turns.append(trn)
        n_actions.append(na)

    NP = 4 * S
    side_of = np.zeros(NP, np.uint8)
    for s, pl in enumerate(ports):
        for j, p in enumerate(pl):
            side_of[4 * s + j] = DIGIT_SIDE[round((p[0] - int(p[0])) * 10)]
    cell_sw = -np.ones((H, W), np.int16)
    for s, x in enumerate(switch_ids):
        cell_sw[x] = s

    # rail side of every port
    port_nb = -np.ones(NP, np.int16)
    port_len = np.zeros(NP, np.int16)
    prev_cell = -np.ones(NP, np.int32)
    for s, x in enumerate(switch_ids):
        for j in range(len(ports[s])):
            g = 4 * s + j
            side = int(side_of[g])
            cell, heading = (x[0] + DELTA[side][0], x[1] + DELTA[side][1]), side
            prev_cell[g] = cell[0] * W + cell[1]
            n = 0
            while cell_sw[cell] < 0:
                ex = [e for e, ok in enumerate(transitions(int(grid[cell]), heading)) if ok]
                if len(ex) != 1:
                    raise ValueError("plain cell without a unique exit")
                n += 1
                heading = ex[0]
                cell = (cell[0] + DELTA[heading][0], cell[1] + DELTA[heading][1])
            s2 = int(cell_sw[cell])
            if s2 == s:
                raise ValueError("rail loop from a switch back to itself")
            entry = (heading + 2) % 4
            j2 = [k for k in range(len(ports[s2])) if side_of[4 * s2 + k] == entry][0]
            port_nb[g] = 4 * s2 + j2
            port_len[g] = n
    # intra-switch adjacency; the unique onward port of a port seen as a transition target
    port_unique = -np.ones(NP, np.int16)
    for s in range(S):
        for j in range(len(ports[s])):
            intra = sorted({b for a, b in outcomes[s] if a == j} | {a for a, b in outcomes[s] if b == j})
            if len(intra) == 1:
                port_unique[4 * s + j] = 4 * s + intra[0]

    # stations / trains
    stations: List[Tuple[int, int]] = []
    for t in sc.trains:
        if tuple(t.target) not in stations:
            stations.append(tuple(t.target))
    K = len(stations)
    T = len(sc.trains)
    if T > 128:
        raise ValueError("at most 128 trains per env")
    dist_k = np.stack([_bfs_distance(grid, st) for st in stations]).astype(np.int64)
    tr_k = np.array([stations.index(tuple(t.target)) for t in sc.trains], np.int32)

    init_port = np.zeros(T, np.int16)
    init_dist = np.zeros(T, np.int32)
    init_delay = np.zeros(T, np.int32)
    for h, t in enumerate(sc.trains):
        cell, heading = tuple(t.initial_position), int(t.initial_direction)
        last, n = None, 0
        while cell_sw[cell] < 0:
            last = cell
            act = _valid_moves(grid, cell, heading)[0][0]
            cell, heading, _, _ = _check_action(grid, act, cell, heading)
            n += 1
        s = int(cell_sw[cell])
        cand = [j for j in range(len(ports[s])) if last is not None and prev_cell[4 * s + j] == last[0] * W + last[1]]
        if not cand:
            raise ValueError("train starts on a switch cell")
        init_port[h] = 4 * s + cand[0]
        init_dist[h] = n
        dv = dist_k[tr_k[h], t.initial_position[0], t.initial_position[1], t.initial_direction]
        if dv >= DIST_INF:
            raise ValueError("train cannot reach its target")
        init_delay[h] = t.earliest_departure - t.latest_arrival + dv
    max_span = int(port_len.max(initial=0)) * 2 + 8 + int(init_dist.max(initial=0))
    if sc.max_episode_steps + max_span + max(t.earliest_departure for t in sc.trains) > 32000:
        raise ValueError("episode too long for 16-bit semaphore times")

    # compact Q layout
    act_src = np.zeros((S, 8), np.uint8)
    act_dst = np.zeros((S, 8), np.uint8)
    act_turn = np.zeros((S, 8), np.uint8)
    act_j = np.zeros((S, 8), np.uint8)
    slot_nroutes = np.zeros(NP, np.uint8)
    slot_route_act = np.full((NP, 4), 0xFF, np.uint8)
    first_other = np.zeros(NP, np.uint8)
    q_off = np.zeros(NP, np.uint64)
    row_base = np.zeros(NP, np.uint32)
    q_w = np.zeros(NP, np.uint8)
    off = 0
    rows = 0
    for s in range(S):
        P = len(ports[s])
        for a, ((i, j), t) in enumerate(zip(outcomes[s], turns[s])):
            act_src[s, a], act_dst[s, a], act_turn[s, a] = i, j, t
        for i in range(P):
            g = 4 * s + i
            mine = [a for a, (src, _) in enumerate(outcomes[s]) if src == i]
            if len(mine) > 3:
                raise ValueError("more than 3 routes from one port")
            slot_nroutes[g] = len(mine)
            for jj, a in enumerate(mine):
                slot_route_act[g, jj] = a
                act_j[s, a] = jj
            first_other[g] = min(a for a, (src, _) in enumerate(outcomes[s]) if src != i)
            nrows = (1 << P) * K * 3
            q_w[g] = len(mine) + 1
            q_off[g] = off
            row_base[g] = rows
            off += nrows * (len(mine) + 1)
            rows += nrows
    cm = CompiledMap(scenario=sc, H=H, W=W, S=S, T=T, K=K, switch_ids=switch_ids, ports=ports,
                     outcomes=outcomes, n_actions=np.array(n_actions, np.uint8), stations=stations)
    cm.q_per_env = int(off)
    cm.rows_per_env = int(rows)
    cm.arrays = dict(
        grid=grid.astype(np.uint16).ravel(), cell_sw=cell_sw.ravel(),
        sw_np=np.array([len(p) for p in ports], np.uint8), sw_na=cm.n_actions,
        act_src=act_src.ravel(), act_dst=act_dst.ravel(), act_turn=act_turn.ravel(), act_j=act_j.ravel(),
        first_other=first_other, port_nb=port_nb, port_len=port_len, port_side=side_of, port_unique=port_unique,
        slot_nroutes=slot_nroutes, slot_route_act=slot_route_act.ravel(), q_off=q_off, q_w=q_w, row_base=row_base,
        dist=np.minimum(dist_k, DIST_INF).astype(np.int32).ravel(),
        tr_ed=np.array([t.earliest_departure for t in sc.trains], np.int32),
        tr_la=np.array([t.latest_arrival for t in sc.trains], np.int32),
        tr_k=tr_k,
        tr_target=np.array([t.target[0] * W + t.target[1] for t in sc.trains], np.int32),
        tr_init_cell=np.array([t.initial_position[0] * W + t.initial_position[1] for t in sc.trains], np.int32),
        tr_init_dir=np.array([t.initial_direction for t in sc.trains], np.uint8),
        tr_init_port=init_port, tr_init_dist=init_dist, tr_init_delay=init_delay,
    )
    cm.qinit_rows = _q_init_patch(cm, grid, dist_k, tr_k)
    return cm


def _q_init_patch(cm: CompiledMap, grid, dist_k, tr_k) -> Dict[Tuple[int, int, int], np.ndarray]:
    """``__init_q_table`` (distr_q.py:81-181) as compact rows, trains in handle order.

    Evaluated from the trains' start states: before the first decision every train
    is still on the rail segment leading to its first switch, and a shortest path
    from anywhere on that segment has the same switch waypoints."""
    sc, K = cm.scenario, cm.K
    W = cm.W
    A = cm.arrays
    cell_sw = A["cell_sw"].reshape(cm.H, cm.W)
    patch: Dict[Tuple[int, int, int], np.ndarray] = {}
    optimal = None  # carried over between waypoints and trains, as in the reference
    OPT, BONUS = 500.0, 1000.0
    for h, t in enumerate(sc.trains):
        dk = dist_k[tr_k[h]]
        cell, heading, target = tuple(t.initial_position), int(t.initial_direction), tuple(t.target)
        path = []
        best = math.inf
        while cell != target:
            choice = None
            for _, nc, nd in _valid_moves(grid, cell, heading):
                v = dk[nc[0], nc[1], nd]
                v = math.inf if v >= DIST_INF else v
                if v < best:
                    choice, best = (nc, nd), v
            path.append((cell, heading))
            if choice is None:
                break
            cell, heading = choice
        else:
            path.append((cell, heading))
        for wi, (wcell, wdir) in enumerate(path):
            s = int(cell_sw[wcell])
            if s < 0:
                continue
            P = len(cm.ports[s])
            entry_side = (wdir + 2) % 4
            slots = [j for j in range(P) if A["port_side"][4 * s + j] == entry_side]
            if not slots:
                raise NotImplementedError("waypoint enters a switch through no port")
            slot = slots[0]
            nxt = next(((c2, d2) for c2, d2 in path[wi + 1:] if cell_sw[c2] >= 0), None)
            best_d = math.inf
            if nxt is not None:
                want = 4 * int(cell_sw[nxt[0]]) + [j for j in range(len(cm.ports[cell_sw[nxt[0]]]))
                                                   if A["port_side"][4 * cell_sw[nxt[0]] + j] == (nxt[1] + 2) % 4][0]
                for a, (src, dst) in enumerate(cm.outcomes[s]):
                    if src == slot and A["port_nb"][4 * s + dst] == want:
                        dd = int(A["port_len"][4 * s + dst])
                        if dd < best_d:
                            optimal, best_d = a, dd
                value = OPT
            else:
                for a, (src, dst) in enumerate(cm.outcomes[s]):
                    if src != slot:
                        continue
                    # plain cells of the segment leaving through dst
                    g = 4 * s + dst
                    side = int(A["port_side"][g])
                    c2, hh = (cm.switch_ids[s][0] + DELTA[side][0], cm.switch_ids[s][1] + DELTA[side][1]), side
                    dd = 0
                    while cell_sw[c2] < 0:
                        if c2 == target:
                            if dd < best_d:
                                best_d, optimal = dd, a
                            break
                        hh = [e for e, ok in enumerate(transitions(int(grid[c2]), hh)) if ok][0]
                        c2 = (c2[0] + DELTA[hh][0], c2[1] + DELTA[hh][1])
                        dd += 1
                value = BONUS
            if optimal is None:
                raise NotImplementedError("__init_q_table would raise UnboundLocalError on this map")
            if optimal >= int(cm.n_actions[s]) or (optimal < len(cm.outcomes[s]) and cm.outcomes[s][optimal][0] != slot):
                raise NotImplementedError("stale optimal_action outside the compact row (unsupported map)")
            g = 4 * s + slot
            w = int(A["q_w"][g])
            j = w - 1 if optimal == len(cm.outcomes[s]) else int(A["act_j"][s * 8 + optimal])
            k = int(tr_k[h])
            for bits in range(1, 1 << P):
                for lvl in range(3):
                    state = (bits * K + k) * 3 + lvl
                    row = np.full(w, np.nan)   # filled with default_q by the runtime
                    row[j] = value
                    patch[(s, slot, state)] = row
    return patch


@functools.lru_cache(maxsize=8)
def _pow_table(x0: float, decay: float, n: int) -> np.ndarray:
    # Python float ``**`` (the host libm's pow, as in the reference), not numpy's vectorised power
    t = np.array([x0 * (decay ** k) for k in range(n)], dtype=np.float64)
    t.setflags(write=False)
    return t


def eps_table(eps0: float, decay: float, n: int = NTAB) -> np.ndarray:
    """``initial_epsilon * decay ** t`` with Python float arithmetic (distr_q.py:68)."""
    return _pow_table(float(eps0), float(decay), int(n))


def lr_table(lr0: float, decay: float, n: int = NTAB) -> np.ndarray:
    """``initial_lr * lr_decay ** t`` (distr_q.py:79)."""
    return _pow_table(float(lr0), float(decay), int(n))
