"""ORACLE / TEST INFRASTRUCTURE ONLY — the checker, never the thing measured or shipped.

A pure-Python CPU restatement of the reference's hot path, one env at a time:

* switch-graph compile        rail_graph.py:13-293, rail_network.py:23-133, switch_agents.py:20-78
* semaphore runtime            rail_network.py:135-436
* AEC env (reset/tick/step)    switch_env.py:93-158, 203-568, 616-675
* observer + reward            observer.py:18-151, 228-308; reward_func.py:23-78
* network-distributed Q        distr_q.py:32-181, 184-379, 419-490
* distance map / shortest path flatland_patch/distance_map.py:62-242

Train movement underneath is ``oracle/flatland_lite.py`` (the frozen Flatland
spec).  Pinned against the golden vectors that tests/golden/make_golden.py
records from the real reference (tests/test_oracle_golden.py): port orders,
distances, init ports, Q-init, every decision/update of learn() and test(),
the .npz outputs and the final Q-tables.

The restatement keeps the reference's data model (dicts keyed by float port
tuples, semaphore records ``[owner, 'in'|'out', dir, t0, t1]``, a Q dict keyed
by observation tuples) so that its semantics — including the quirks listed in
SURVEY.md §8.1 — are reproduced literally rather than re-derived.
"""
from __future__ import annotations

import itertools
import math
from typing import Dict, List, Optional, Tuple

import numpy as np

from oracle import flatland_lite as fl

ACT = fl.RailEnvActions
TS = fl.TrainState

# neighbour offset -> port-name suffix (rail_graph.py:92-97)
_SUFFIX = {(0, 1): 0.1, (-1, 0): 0.2, (0, -1): 0.3, (1, 0): 0.4}


def port_digit(p) -> int:
    return round((p[0] - int(p[0])) * 10)


def node_of(p) -> Tuple[int, int]:
    """naming.py:10-24"""
    return (int(p[0]), int(p[1]))


def side_of(p) -> int:
    """Flatland direction from the switch cell towards the port (rail_network.py:280-290)."""
    return {1: 1, 2: 0, 3: 3}.get(port_digit(p), 2)


def inverse_side(direction) -> int:
    """rail_network.py:292-301"""
    return {1: 3, 0: 4, 3: 1}.get(int(direction), 2)


def switch_name(sid) -> str:
    return f"switch_{sid[0]}-{sid[1]}"


def switch_id(name: str) -> Tuple[int, int]:
    a, b = name.split("_")[1].split("-")
    return (int(a), int(b))


# ---------------------------------------------------------------------------
# distance map + shortest paths (flatland_patch/distance_map.py)
# ---------------------------------------------------------------------------

def distance_map(rail: fl.GridTransitionMap, targets: List[Tuple[int, int]]) -> np.ndarray:
    """(n_trains, H, W, 4) float64, inf where unreachable (distance_map.py:62-167)."""
    H, W = rail.height, rail.width
    out = np.full((len(targets), H, W, 4), np.inf)
    done: Dict[Tuple[int, int], int] = {}
    for i, tgt in enumerate(targets):
        if tgt in done:
            out[i] = out[done[tgt]]
            continue
        done[tgt] = i
        d = out[i]
        d[tgt[0], tgt[1], :] = 0
        frontier = []

        def expand(cell, dist, heading):
            dirs = range(4) if heading < 0 else [(heading + 2) % 4]
            found = []
            for nd in dirs:
                nc = fl.get_new_position(cell, nd)
                if not (0 <= nc[0] < H and 0 <= nc[1] < W):
                    continue
                move = (nd + 2) % 4
                for o in range(4):
                    if rail.get_transition((nc, o), move):
                        nv = min(d[nc[0], nc[1], o], dist + 1)
                        d[nc[0], nc[1], o] = nv
                        found.append((nc, o, nv))
            return found

        from collections import deque
        q = deque(expand(tgt, 0, -1))
        seen = {(tgt, o) for o in range(4)}
        while q:
            cell, o, dist = q.popleft()
            if (cell, o) in seen:
                continue
            seen.add((cell, o))
            q.extend(expand(cell, dist, o))
    return out


def shortest_path(rail: fl.GridTransitionMap, dist_i: np.ndarray, position, direction, target):
    """Waypoints of the greedy descent on the distance map (distance_map.py:195-232)."""
    path = []
    best = math.inf
    while position != target:
        choice = None
        for na in rail.get_valid_move_actions_(direction, position):
            v = dist_i[na.next_position[0], na.next_position[1], na.next_direction]
            if v < best:
                choice, best = na, v
        path.append(fl.Waypoint(position, direction))
        if choice is None:
            return path
        position, direction = choice.next_position, choice.next_direction
    path.append(fl.Waypoint(position, direction))
    return path


# ---------------------------------------------------------------------------
# switch-graph compile
# ---------------------------------------------------------------------------

class SwitchInfo:
    def __init__(self, sid, ports, outcomes, plans, n_actions):
        self.id = sid
        self.ports = ports              # get_port_nodes() order
        self.outcomes = outcomes        # [(src_port, dst_port)] = action_outcomes
        self.plans = plans              # rail-action pair per action for the source port
        self.n_actions = n_actions      # Discrete(n) incl. STOP (switch_agents.py:194-259)


class Network:
    """Port graph of a rail grid, in the reference's port/action numbering."""

    def __init__(self, rail: fl.GridTransitionMap):
        self.rail = rail
        H, W = rail.height, rail.width
        adj: Dict[tuple, dict] = {}

        def link(u, v):
            adj.setdefault(u, {})
            adj.setdefault(v, {})
            if v not in adj[u]:
                adj[u][v] = None
                adj[v][u] = None

        # cell graph in the reference's insertion order (rail_graph.py:19-86)
        for r, c, d in itertools.product(range(H), range(W), range(4)):
            if rail.get_full_transitions(r, c) == 0:
                continue
            for e, ok in enumerate(rail.get_transitions(((r, c), d))):
                if ok:
                    nxt = fl.get_new_position((r, c), e)
                    if 0 <= nxt[0] < W and 0 <= nxt[1] < H:  # the reference's (swapped) bound check
                        link((r, c), nxt)
        # port ("proximity") nodes around every non-degree-2 cell (rail_graph.py:99-135)
        for cell in list(adj):
            if len(adj[cell]) == 2:
                continue
            for nb in list(adj[cell]):
                sfx = _SUFFIX[(int(nb[0]) - cell[0], int(nb[1]) - cell[1])]
                port = (int(cell[0]) + sfx, int(cell[1]) + sfx)
                adj.setdefault(port, {})
                link(nb, port)
                link(cell, port)
                del adj[cell][nb]
                del adj[nb][cell]
        by_switch: Dict[Tuple[int, int], list] = {}
        for n in adj:
            if isinstance(n[0], float):
                by_switch.setdefault(node_of(n), []).append(n)
        n_ports = sum(len(v) for v in by_switch.values())

        self.switch_ids = sorted(by_switch)          # pandas groupby key order (rail_network.py:38)
        self.switches: Dict[Tuple[int, int], SwitchInfo] = {}
        self.neighbor: Dict[tuple, Tuple[Tuple[int, int], tuple]] = {}
        self.seg_len: Dict[tuple, int] = {}
        self.prev_node: Dict[tuple, Tuple[int, int]] = {}
        self.intra: Dict[tuple, List[tuple]] = {}
        for sid in self.switch_ids:
            plist = by_switch[sid]
            # networkx subgraph iteration: the filter's node *set* when it is the shorter side
            order = list(set(plist)) if 2 * len(plist) < n_ports else list(plist)
            word = rail.get_full_transitions(*sid)

            def joined(a, b):
                ha, hb = (side_of(a) + 2) % 4, (side_of(b) + 2) % 4
                return bool((word >> (15 - (4 * ha + side_of(b)))) & 1) or \
                    bool((word >> (15 - (4 * hb + side_of(a)))) & 1)

            outcomes, plans = [], []
            for p in order:
                for q in order:
                    if q == p or not joined(p, q):
                        continue
                    i_in, i_out = port_digit(p) - 1, port_digit(q) - 1
                    turn = {1: ACT.MOVE_RIGHT, 2: ACT.MOVE_FORWARD, 3: ACT.MOVE_LEFT}[(i_out - i_in) % 4]
                    outcomes.append((p, q))
                    plans.append([ACT.MOVE_FORWARD, turn])
            n_act = {(3, 4): 5, (4, 4): 5, (4, 6): 7, (4, 8): 9}.get((len(order), len(outcomes)))
            if n_act is None:
                raise ValueError(f"No Agent with n_gaits={len(order)} and n_rails={len(outcomes)}")
            self.switches[sid] = SwitchInfo(sid, order, outcomes, plans, n_act)
            for p in order:
                self.intra[p] = [q for q in order if q != p and joined(p, q)]
        # rail side of every port: walk the plain track to the next switch
        for sid in self.switch_ids:
            for p in self.switches[sid].ports:
                s = side_of(p)
                cell, heading = fl.get_new_position(sid, s), s
                self.prev_node[p] = cell
                n = 0
                while cell not in self.switches:
                    exits = [e for e, ok in enumerate(rail.get_transitions(cell, heading)) if ok]
                    if len(exits) != 1:
                        raise ValueError("plain cell without a unique exit")
                    n += 1
                    heading = exits[0]
                    cell = fl.get_new_position(cell, heading)
                entry_side = (heading + 2) % 4
                q = [x for x in self.switches[cell].ports if side_of(x) == entry_side][0]
                if cell == sid:
                    raise ValueError("rail loop from a switch back to itself")
                self.neighbor[p] = (cell, q)
                self.seg_len[p] = n

    def is_switch(self, cell) -> bool:
        return cell is not None and tuple(cell) in self.switches

    def port_distance(self, a, b):
        """rail_network.py:543-558 — len(rail_nodes) of a direct edge, None if none."""
        if self.neighbor.get(a, (None, None))[1] == b:
            return self.seg_len[a]
        if b in self.intra.get(a, ()):
            return 0
        return None

    def edges_of(self, p):
        """Ports adjacent to ``p`` in the rail graph (rail edge + intra-switch edges)."""
        return [self.neighbor[p][1]] + list(self.intra[p])


# ---------------------------------------------------------------------------
# environment
# ---------------------------------------------------------------------------

class OracleEnv:
    """ASyncSwitchEnv + RailNetwork runtime + StandardObserver + StandardRewardFunction."""

    STOP_PENALTY = 1300                       # reward_func.py:21
    DELAY_THRESHOLD = 20                      # observer.py:221

    def __init__(self, rail_env: fl.RailEnv, max_steps: int = 200):
        self.rail_env = rail_env
        self.net = Network(rail_env.rail)
        self.max_steps = max_steps
        self.agents = [switch_name(s) for s in self.net.switch_ids]
        self.dist = distance_map(rail_env.rail, [a.target for a in rail_env.agents])
        T = len(rail_env.agents)
        # persistent across reset (rail_network.py:113-128 vs reset 135-149)
        self.prev_port = {h: None for h in range(T)}
        self.source_port = {h: None for h in range(T)}
        self.next_port = {h: None for h in range(T)}
        self.next_port_dist = {h: None for h in range(T)}
        self.sem: Dict[tuple, list] = {}
        self.n_ticks = 0

    # -- helpers ----------------------------------------------------------
    def now(self):
        return self.rail_env._elapsed_steps

    def train(self, h):
        return self.rail_env.agents[h]

    def n_actions(self, agent: str) -> int:
        return self.net.switches[switch_id(agent)].n_actions

    def compute_delay(self, tr, position, direction, at_departure=False):
        """observer.py:18-42"""
        v = self.dist[tr.handle, position[0], position[1], int(direction)]
        if np.isinf(v):
            raise ValueError("Infinite distance to target encountered.")
        if at_departure:
            return tr.earliest_departure - tr.latest_arrival + v
        return self.now() - tr.latest_arrival + v

    def discretize(self, tr, delay) -> int:
        """observer.py:228-244"""
        if delay <= 0:
            return 0
        if delay <= (tr.latest_arrival - tr.earliest_departure) * self.DELAY_THRESHOLD:
            return 1
        return 2

    def _live(self, rec, h):
        return rec[0] != h and rec[3] <= self.now() <= rec[4]

    def port_blocked(self, next_port, out_port, h) -> bool:
        """observer.py:44-151 — the eight guarded cases, evaluated in the reference's order."""
        agents = self.rail_env.agents

        def case(port, io, same_dir, need_malf):
            rec = self.sem[port]
            if not self._live(rec, h) or rec[1] != io:
                return False
            if (rec[2] == side_of(port)) != same_dir:
                return False
            return (not need_malf) or agents[rec[0]].state == TS.MALFUNCTION

        if next_port is not None:
            blocked = False
            if next_port in self.sem:
                for io, same, malf in (("out", True, False), ("out", False, True), ("in", False, False), ("in", True, True)):
                    if case(next_port, io, same, malf):
                        blocked = True
                        break
            if not blocked and out_port in self.sem:
                for io, same, malf in (("out", False, False), ("out", True, True), ("in", True, False), ("in", False, True)):
                    if case(out_port, io, same, malf):
                        blocked = True
                        break
            return blocked
        if out_port in self.sem:
            for io, same, malf in (("out", True, False), ("out", False, True), ("in", False, False), ("in", True, True)):
                if case(out_port, io, same, malf):
                    return True
        return False

    # -- semaphore runtime (rail_network.py) ------------------------------
    def _put(self, port, h, io, span, keep_io_on_override, override_io):
        """set-if-absent, else override when (io matches) or (t0 in the future)."""
        t = self.now()
        rec = self.sem.get(port)
        if rec is None:
            self.sem[port] = [h, io, side_of(port), t, t + span]
        elif (override_io is not None and rec[1] == override_io) or rec[3] > t:
            if keep_io_on_override:
                rec[0], rec[3], rec[4] = h, t, t + span
            else:
                self.sem[port] = [h, io, side_of(port), t, t + span]

    def transition_semaphore(self, source, out_port, target, tr, next_sid):
        """rail_network.py:303-416"""
        h = tr.handle
        if tr.state != TS.MALFUNCTION:
            for anchor in (self.next_port[h], self.prev_port[h]):
                if anchor is None:
                    continue
                for p in self.net.switches[node_of(anchor)].ports:
                    if p in self.sem and self.sem[p][0] == h:
                        del self.sem[p]
        d_ot = self.net.port_distance(out_port, target)
        self._put(out_port, h, "out", 3, True, "out")
        self._put(target, h, "in", d_ot + 1, True, "in")
        onward = [q for q in self.net.edges_of(target) if q != out_port]
        if len(onward) == 1:
            unique = onward[0]
            for p in (target, unique):
                if p not in (source, out_port, target):
                    self._put(p, h, "out", d_ot + self.net.port_distance(target, p) + 1, False, "out")
            # the reference compares the whole record with 'out' here (rail_network.py:385): never true
            self._put(unique, h, "out", d_ot + self.net.port_distance(target, unique), False, None)
            far = self.net.neighbor[unique][1]
            for p in (unique, far):
                if p not in (source, out_port, unique):
                    span = d_ot + self.net.port_distance(target, unique) + self.net.port_distance(unique, p) + 1
                    self._put(p, h, "in", span, False, "in")
        for p in (out_port, target):
            if p not in (source, out_port):
                self._put(p, h, "out", self.net.port_distance(out_port, p) + 1, False, "out")

    def transition_train(self, tr, in_port, out_port):
        """rail_network.py:246-278"""
        assert node_of(in_port) == node_of(out_port)
        next_sid, target = self.net.neighbor[out_port]
        self.transition_semaphore(in_port, out_port, target, tr, next_sid)
        self.source_port[tr.handle] = in_port
        self.next_port[tr.handle] = target
        self.prev_port[tr.handle] = out_port
        return next_sid, target

    def extend_semaphores(self):
        """rail_network.py:229-244"""
        t = self.now()
        for tr in self.rail_env.agents:
            if tr.state in (TS.STOPPED, TS.MALFUNCTION):
                for p, rec in self.sem.items():
                    if rec[0] == tr.handle:
                        span = rec[4] - rec[3]
                        rec[3] = t
                        rec[4] = t + span
            if tr.state == TS.MALFUNCTION:
                p = self.next_port[tr.handle]
                if p not in self.sem:
                    self.sem[p] = [tr.handle, "in", side_of(p), t, t + self.next_port_dist[tr.handle]]

    # -- episode ------------------------------------------------------------
    def reset(self, seed=None):
        """switch_env.py:93-158"""
        self.rail_env.reset(random_seed=seed)
        T = len(self.rail_env.agents)
        self.next_port = {h: None for h in range(T)}
        self.next_port_dist = {h: None for h in range(T)}
        self.sem = {}
        self.terminated = self.truncated = False
        self.terminations = {a: False for a in self.agents}
        self.truncations = {a: False for a in self.agents}
        self.rewards = {a: {h: 0 for h in range(T)} for a in self.agents}
        self.step_counter = 0
        self.plan = {h: [] for h in range(T)}
        self.train_done = {h: False for h in range(T)}
        self.train_info = None
        self.malfunctions = []
        self.num_malfunctions = 0
        self.active_agents: List[str] = []
        self.active_trains: List[int] = []
        self.agent_selection = None
        self.active_train = None
        self.prev_actions = {h: None for h in range(T)}
        self.last_node = {tr.handle: (None, self.compute_delay(tr, tr.initial_position, tr.initial_direction, True))
                          for tr in self.rail_env.agents}
        self._init_ports()
        self._tick_until_decision()

    def _init_ports(self):
        """switch_env.py:507-568"""
        rail = self.rail_env.rail
        for tr in self.rail_env.agents:
            pos, d = tr.position, tr.direction
            last = tr.old_position
            if pos is None or d is None:
                pos, d = tr.initial_position, tr.initial_direction
            n = 0
            while not self.net.is_switch(pos):
                last, last_d = pos, d
                act = rail.get_valid_move_actions_(last_d, last)[0].action
                _, (pos, d), _, _ = rail.check_action_on_agent(act, (pos, d))
                n += 1
            sw = self.net.switches[tuple(pos)]
            port = [p for p in sw.ports if self.net.prev_node[p] == last][0]
            self.next_port[tr.handle] = port
            self.next_port_dist[tr.handle] = n
        for tr in self.rail_env.agents:
            p = self.next_port[tr.handle]
            self.sem[p] = [tr.handle, "in", side_of(p), tr.earliest_departure - 2,
                           tr.earliest_departure + self.next_port_dist[tr.handle]]

    def _move_trains(self):
        """switch_env.py:296-401 (one Flatland tick)."""
        rail = self.rail_env.rail
        actions, predicted = {}, {}
        for tr in self.rail_env.agents:
            h = tr.handle
            if self.train_done[h]:
                continue
            if not self.plan[h]:
                actions[h] = ACT.MOVE_FORWARD
            else:
                self.prev_actions[h] = self.plan[h][0]
                actions[h] = self.plan[h].pop(0)
            if tr.position is not None:
                _, (npos, _), valid, _ = rail.check_action_on_agent(actions[h], (tr.position, tr.direction))
                predicted[h] = (npos, True) if valid else (tr.position, False)
        _, _, self.train_done, self.train_info = self.rail_env.step(actions)
        self.n_ticks += 1
        for tr in self.rail_env.agents:
            h = tr.handle
            if h in predicted:
                exp_pos, valid = predicted[h]
                if exp_pos != tr.position and valid and actions[h] != ACT.STOP_MOVING:
                    self.plan[h].insert(0, actions[h])
                    if self.net.is_switch(exp_pos):
                        self.next_port[h] = self.source_port[h]
            if self.train_done[h]:
                for p in [p for p, rec in self.sem.items() if rec[0] == h]:
                    del self.sem[p]
        t = self.now()
        for tr in self.rail_env.agents:
            if t == tr.earliest_departure - 2:
                p = self.next_port[tr.handle]
                self.sem[p] = [tr.handle, "in", side_of(p), tr.earliest_departure - 2,
                               tr.earliest_departure + self.next_port_dist[tr.handle]]
        self.extend_semaphores()
        if self.train_done["__all__"]:
            self.terminations = {a: True for a in self.terminations}
            self.terminated = True
        now_mf = list(np.nonzero([v for v in self.train_info["malfunction"].values()])[0])
        self.num_malfunctions += len(set(now_mf).difference(set(self.malfunctions)))
        self.malfunctions = now_mf

    def _check_active_switch(self):
        """switch_env.py:427-485"""
        rail = self.rail_env.rail
        for tr in self.rail_env.agents:
            if tr.position is None or tr.state == TS.WAITING:
                continue
            nxt = self.plan[tr.handle][0] if self.plan[tr.handle] else ACT.MOVE_FORWARD
            _, (npos, _), _, _ = rail.check_action_on_agent(nxt, (tr.position, tr.direction))
            if not self.net.is_switch(npos):
                continue
            if tr.state in (TS.READY_TO_DEPART, TS.MOVING):
                sid = tuple(npos)
            elif tr.state in (TS.STOPPED, TS.MALFUNCTION) and self.prev_actions[tr.handle] == ACT.STOP_MOVING:
                sid = tuple(npos)
            elif tr.state in (TS.STOPPED, TS.MALFUNCTION):
                sid = node_of(self.next_port[tr.handle])
            else:
                continue
            self.active_agents.append(switch_name(sid))
            self.active_trains.append(tr.handle)

    def _tick_until_decision(self):
        """switch_env.py:403-424"""
        while not self.active_agents and not self.terminated:
            self._move_trains()
            self._check_active_switch()
        order = np.argsort(self.active_trains)
        self.active_trains = sorted(self.active_trains)
        self.active_agents = [self.active_agents[i] for i in order]

    # -- AEC protocol -------------------------------------------------------
    def agent_iter(self):
        """switch_env.py:616-630"""
        while not (self.terminated or self.truncated):
            self.agent_selection = self.active_agents.pop(0)
            self.active_train = self.active_trains.pop(0)
            yield self.agent_selection

    def observe(self, agent):
        """observer.py:246-308"""
        sid = switch_id(agent)
        sw = self.net.switches[sid]
        h = self.active_train
        tr = self.train(h)
        sem_bits, target, delay = [], [], []
        current = None
        for p in sw.ports:
            nxt = self.net.neighbor[p][1]
            sem_bits.append(0 if self.port_blocked(nxt, p, h) else 1)
            if self.next_port[h] == p:
                current = p
                delay.append(self.discretize(tr, self.compute_delay(tr, tr.position, tr.direction)))
                target.extend(tr.target)
            else:
                delay.append(-1)
                target.extend([-1, -1])
        obs = np.concatenate([np.array(sid), np.array(sem_bits, dtype=int), np.array(target, dtype=int),
                              np.array(delay, dtype=int)]).astype(np.int64)
        return obs, {"action_mask": self.action_mask(sw, current, sem_bits), "active_train": h}

    @staticmethod
    def action_mask(sw: SwitchInfo, port, sem_bits):
        """switch_agents.py:104-134"""
        free = dict(zip(sw.ports, sem_bits))
        m = [int(src == port) & int(free[dst]) for src, dst in sw.outcomes] + [1]
        return np.array(m, dtype=np.int8)

    def last(self):
        agent = self.agent_selection
        obs, info = self.observe(agent)
        return obs, self.rewards[agent], self.terminations[agent], self.truncations[agent], info

    def reward(self, tr, plan, blocked):
        """reward_func.py:23-78"""
        pos, d = tr.position, tr.direction
        for a in plan:
            if a != ACT.STOP_MOVING:
                _, (pos, d), _, _ = self.rail_env.rail.check_action_on_agent(a, (pos, d))
        cur = self.compute_delay(tr, pos, d)
        diff = self.last_node[tr.handle][1] - cur
        stop_free = plan[0] == ACT.STOP_MOVING and not all(blocked)
        return (diff - self.STOP_PENALTY if stop_free else diff), cur

    def _apply_action(self, agent, action):
        """switch_env.py:203-294 (+ switch_agents.py:136-168 for the rail-action plan)."""
        sid = switch_id(agent)
        sw = self.net.switches[sid]
        assert 0 <= int(action) < sw.n_actions
        h = self.active_train
        tr = self.train(h)
        in_port_of_train = self.next_port.get(h)
        moving = None
        if action == len(sw.outcomes):
            new_plan = [ACT.STOP_MOVING]
        else:
            src, _ = sw.outcomes[action]
            if in_port_of_train in sw.ports:
                new_plan = list(sw.plans[action]) if src == in_port_of_train else [ACT.STOP_MOVING, ACT.STOP_MOVING]
                if new_plan[0] != ACT.STOP_MOVING:
                    moving = h
            else:
                new_plan = []
        if new_plan[0] == ACT.STOP_MOVING:
            in_port = out_port = self.next_port[h]
        else:
            in_port, out_port = sw.outcomes[action]
        if moving is not None:
            next_sid, next_port = self.transition_train(tr, in_port, out_port)
        else:
            next_sid, next_port = sid, None
        plan = self.plan[h]
        if moving is not None and plan:
            new_plan.pop(0)
            if len(plan) > 1:
                del plan[1:]
            plan.extend(new_plan)
        elif moving is None:
            plan.insert(0, ACT.STOP_MOVING)
        else:
            plan.extend(new_plan)
        if moving is not None:
            blocked = [self.port_blocked(next_port, out_port, h)]
        else:
            blocked = []
            for src, dst in sw.outcomes:
                if src == in_port:
                    blocked.append(self.port_blocked(self.net.neighbor[dst][1], dst, h))
        r, cur = self.reward(tr, plan, blocked)
        self.rewards[switch_name(next_sid)][h] = r
        self.last_node[h] = (sid, cur)
        return next_sid

    def step(self, action):
        """switch_env.py:632-666"""
        if self.terminations[self.agent_selection] or self.truncations[self.agent_selection] or action is None:
            return {}
        nxt = self._apply_action(self.agent_selection, action)
        if not self.active_agents:
            self._tick_until_decision()
        self.step_counter += 1
        if self.step_counter > self.max_steps:
            self.truncations = {a: True for a in self.truncations}
            self.truncated = True
        arrived = [tr.handle for tr in self.rail_env.agents if tr.position is None and tr.arrival_time is not None]
        return {"next_switch": nxt, "arrived_trains": arrived}


# ---------------------------------------------------------------------------
# learner
# ---------------------------------------------------------------------------

class OracleDistrQ:
    """distr_q.py:11-527 restated; ``events`` mirrors tests/golden/make_golden.py's trace."""

    OPTIMAL_INIT = 500.0
    DESTINATION_BONUS = 1000.0

    def __init__(self, env: OracleEnv, gamma=1.0, epsilon=0.4, epsilon_decay_rate=0.0, lr=0.4,
                 lr_decay_rate=0.0, default_q=0.0, seed=450565, trace=True):
        self.env = env
        self.gamma, self.eps0, self.eps_decay = gamma, epsilon, epsilon_decay_rate
        self.lr0, self.lr_decay, self.default_q, self.seed = lr, lr_decay_rate, default_q, seed
        self.q: Dict[tuple, list] = {}
        self.trace = trace
        self.events: list = []
        self.on_step = None  # optional callback(env, obs, action, reward, post) after every env.step

    # table primitives (distr_q.py:47-79, 449-490)
    def _row(self, state, agent):
        k = tuple(int(x) for x in state)
        if k not in self.q:
            self.q[k] = [self.default_q] * self.env.n_actions(agent)
        return self.q[k]

    def max_q(self, state, agent):
        if state is None:
            return 0.0
        return max(self._row(state, agent))

    def max_action(self, state, agent, mask):
        row = self._row(state, agent)
        best = int(np.argmax(row))
        if mask[best]:
            return best
        allowed = np.nonzero(mask)[0]
        return int(allowed[np.argmax(np.array(row)[allowed])])

    def update(self, state, action, reward, next_state, prev_agent, next_agent, counts):
        row = self._row(state, prev_agent)
        lr = self.lr0 * (self.lr_decay ** counts[prev_agent])
        if next_agent != prev_agent:
            row[action] = (1 - lr) * row[action] + lr * (reward + self.gamma * self.max_q(next_state, next_agent))
        else:
            row[action] = (1 - lr) * row[action] + lr * reward
        if self.trace:
            self.events.append(["U", [int(x) for x in state], int(action), float(reward), next_state is None,
                                prev_agent, next_agent, float(row[action])])

    def init_q_table(self):
        """distr_q.py:81-181 (including its stale ``optimal_action`` carry-over)."""
        env, net, rail_env = self.env, self.env.net, self.env.rail_env
        optimal_action = None
        for tr in rail_env.agents:
            if tr.state.is_off_map_state():
                pos = tr.initial_position
            elif tr.state.is_on_map_state():
                pos = tr.position
            elif tr.state == TS.DONE:
                pos = tr.target
            else:
                continue
            path = shortest_path(rail_env.rail, env.dist[tr.handle], pos, tr.direction, tr.target)
            for wi, wp in enumerate(path):
                if not net.is_switch(wp.position):
                    continue
                sw = net.switches[tuple(wp.position)]
                P = len(sw.ports)
                ind = inverse_side(wp.direction)
                in_port = tuple(x + ind / 10 for x in wp.position)
                slot = [i for i, p in enumerate(sw.ports) if p == in_port]
                sems = list(itertools.product([0, 1], repeat=P))[1:]
                tgt = [-1] * (2 * P)
                dls = []
                for lvl in range(3):
                    dls.append(tuple(lvl if p == in_port else -1 for p in sw.ports))
                for i in slot:
                    tgt[2 * i], tgt[2 * i + 1] = tr.target
                states = [tuple(int(x) for x in (*wp.position, *s, *tgt, *dl)) for s in sems for dl in dls]
                nxt_wp = None
                for k in range(wi + 1, len(path)):
                    if net.is_switch(path[k].position):
                        nxt_wp = path[k]
                        break
                best = math.inf
                if nxt_wp is not None:
                    nd = inverse_side(nxt_wp.direction)
                    want = tuple(x + nd / 10 for x in nxt_wp.position)
                    for ai, (src, dst) in enumerate(sw.outcomes):
                        if src == in_port and net.neighbor[dst][1] == want:
                            dd = net.port_distance(dst, want)
                            if dd < best:
                                optimal_action, best = ai, dd
                    value = self.OPTIMAL_INIT
                else:
                    for ai, (src, dst) in enumerate(sw.outcomes):
                        if src == in_port:
                            cells = self._segment_cells(dst)
                            for dd, cell in enumerate(cells):
                                if cell == tr.target:
                                    if dd < best:
                                        best, optimal_action = dd, ai
                                    break
                    value = self.DESTINATION_BONUS
                if optimal_action is None:
                    raise UnboundLocalError("optimal_action referenced before assignment")
                for st in states:
                    row = [self.default_q] * sw.n_actions
                    row[optimal_action] = value
                    self.q[st] = row

    def _segment_cells(self, port):
        """Plain cells on the rail edge leaving ``port`` (only membership / length matter here)."""
        net = self.env.net
        cells = []
        s = side_of(port)
        cell, heading = fl.get_new_position(node_of(port), s), s
        while cell not in net.switches:
            cells.append(cell)
            heading = [e for e, ok in enumerate(net.rail.get_transitions(cell, heading)) if ok][0]
            cell = fl.get_new_position(cell, heading)
        return cells

    def _trace_decision(self, obs, rew, info):
        env = self.env
        self.events.append(["D", int(env.now()), env.agent_selection, int(env.active_train),
                            [int(x) for x in obs], float(rew), [int(x) for x in info["action_mask"]], False, False])

    def _trace_step(self, action, post):
        env = self.env
        self.events.append(["S", int(action), [int(x) for x in post["next_switch"]], list(post["arrived_trains"]),
                            int(env.now()), sem_digest(env.sem)])

    def test(self):
        """distr_q.py:184-241 — greedy episode; returns (cum_reward, arrived, delays)."""
        env = self.env
        if self.trace:
            self.events.append(["R"])
        env.reset(seed=self.seed)
        cum = 0.0
        post = {"arrived_trains": []}
        for agent in env.agent_iter():
            obs, rew, term, trunc, info = env.last()
            r = rew[env.active_train]
            if self.trace:
                self._trace_decision(obs, r, info)
            if term or trunc:
                break
            a = self.max_action(obs, agent, info["action_mask"])
            post = env.step(a)
            if self.trace:
                self._trace_step(a, post)
            if self.on_step:
                self.on_step(env, obs, a, r, post)
            cum += r
        delays = [v[1] for v in env.last_node.values()]
        return cum, len(post["arrived_trains"]), delays

    def learn(self, num_episodes, exploit_freq=None, checkpoint_freq=None):
        """distr_q.py:244-379; returns the arrays the reference writes as .npz.  With checkpoint_freq,
        out["checkpoints"][t + 1] is the Q dict the reference pickles at distr_q.py:288-289 -- after
        that episode's exploit round (278-281), before its reset."""
        env = self.env
        cum = np.zeros(num_episodes)
        arrived, delays, mfs, cum_x, arr_x = [], [], [], [], []
        counts = {a: 0 for a in env.agents}
        rng = np.random.default_rng(self.seed)
        post = None
        ckpt = {}
        for t in range(num_episodes):
            if exploit_freq is not None and (t + 1) % exploit_freq == 0:
                tr_, ta_, _ = self.test()
                cum_x.append(tr_)
                arr_x.append(ta_)
            if checkpoint_freq and (t + 1) % checkpoint_freq == 0:
                ckpt[t + 1] = {k: list(v) for k, v in self.q.items()}
            pending: Dict[tuple, tuple] = {}
            at_dest: List[int] = []
            if self.trace:
                self.events.append(["R"])
            env.reset(seed=self.seed)
            if t == 0:
                self.init_q_table()
            for agent in env.agent_iter():
                obs, rew, term, trunc, info = env.last()
                r = rew[env.active_train]
                if self.trace:
                    self._trace_decision(obs, r, info)
                if term or trunc:
                    break
                eps = self.eps0 * (self.eps_decay ** counts[agent])
                if rng.random() < eps:
                    sub = np.random.Generator(np.random.PCG64(np.random.SeedSequence(int(rng.integers(0, np.iinfo(np.int32).max)))))
                    valid = np.where(info["action_mask"] == 1)[0]
                    action = int(sub.choice(valid)) if len(valid) else 0
                else:
                    action = self.max_action(obs, agent, info["action_mask"])
                post = env.step(action)
                if self.trace:
                    self._trace_step(action, post)
                if self.on_step:
                    self.on_step(env, obs, action, r, post)
                h = info["active_train"]
                key = (switch_id(agent), h)
                if key in pending:
                    p_obs, p_act, p_agent = pending.pop(key)
                    self.update(p_obs, p_act, r, obs, p_agent, agent, counts)
                pending[(post["next_switch"], h)] = (obs, action, agent)
                for tr in post["arrived_trains"]:
                    if tr not in at_dest:
                        at_dest.append(tr)
                        for (k_sw, k_tr), (u_obs, u_act, u_agent) in list(pending.items()):
                            if k_tr == tr:
                                self.update(u_obs, u_act, self.DESTINATION_BONUS, None, u_agent, None, counts)
                                del pending[(k_sw, k_tr)]
                cum[t] += r
                counts[agent] += 1
            arrived.append(len(post["arrived_trains"]))
            delays.append([v[1] for v in env.last_node.values()])
            mfs.append(env.num_malfunctions)
        out = dict(cum_reward=cum.tolist(), arrived_trains=arrived, delays=delays, num_malfunctions=mfs,
                   trains_at_dest=list(post["arrived_trains"]))
        if exploit_freq is not None:
            out["cum_reward_exploit"] = cum_x
            out["arrived_trains_exploit"] = arr_x
        if checkpoint_freq:
            out["checkpoints"] = ckpt
        return out


def run_decisions(model: "OracleDistrQ", total: int, state: dict = None) -> dict:
    """The learn loop (distr_q.py:275-362) with episodes restarting as they end, stopped after
    ``total`` decisions — the product's ``sfl_step`` (the benchmark step).  ``state`` carries the
    loop across calls; returns it."""
    env = model.env
    if state is None:
        state = dict(rng=np.random.default_rng(model.seed), counts={a: 0 for a in env.agents}, t=0,
                     in_episode=False, pending={}, at_dest=[], it=None, done=0)
    rng, counts = state["rng"], state["counts"]
    while state["done"] < total:
        if not state["in_episode"]:
            env.reset(seed=model.seed)
            if state["t"] == 0:
                model.init_q_table()
            state.update(in_episode=True, pending={}, at_dest=[], it=env.agent_iter())
        try:
            agent = next(state["it"])
        except StopIteration:
            state["in_episode"] = False
            state["t"] += 1
            continue
        obs, rew, term, trunc, info = env.last()
        r = rew[env.active_train]
        eps = model.eps0 * (model.eps_decay ** counts[agent])
        if rng.random() < eps:
            sub = np.random.Generator(np.random.PCG64(np.random.SeedSequence(int(rng.integers(0, np.iinfo(np.int32).max)))))
            action = int(sub.choice(np.where(info["action_mask"] == 1)[0]))
        else:
            action = model.max_action(obs, agent, info["action_mask"])
        post = env.step(action)
        if model.on_step:
            model.on_step(env, obs, action, r, post)
        h = info["active_train"]
        pending, at_dest = state["pending"], state["at_dest"]
        key = (switch_id(agent), h)
        if key in pending:
            p_obs, p_act, p_agent = pending.pop(key)
            model.update(p_obs, p_act, r, obs, p_agent, agent, counts)
        pending[(post["next_switch"], h)] = (obs, action, agent)
        for tr in post["arrived_trains"]:
            if tr not in at_dest:
                at_dest.append(tr)
                for (k_sw, k_tr), (u_obs, u_act, u_agent) in list(pending.items()):
                    if k_tr == tr:
                        model.update(u_obs, u_act, model.DESTINATION_BONUS, None, u_agent, None, counts)
                        del pending[(k_sw, k_tr)]
        counts[agent] += 1
        state["done"] += 1
    return state


def sem_digest(semaphores) -> int:
    import zlib
    items = sorted((tuple(float(x) for x in p), int(v[0]), str(v[1]), int(v[2]), int(v[3]), int(v[4]))
                   for p, v in semaphores.items())
    return zlib.crc32(repr(items).encode()) & 0xFFFFFFFF


def build(scenario, seed, hp, max_steps=100_000, trace=True, mf_stream="counter", delay_threshold=20):
    """Oracle (env, learner) for a ``mapgen.Scenario`` and reference-style hyper-parameters."""
    rail_env = fl.RailEnv(scenario, mf_stream=mf_stream)
    rail_env.reset()
    env = OracleEnv(rail_env, max_steps=max_steps)
    env.DELAY_THRESHOLD = delay_threshold  # StandardObserver(delay_threshold=...), observer.py:221
    model = OracleDistrQ(env, gamma=hp["gamma"], epsilon=hp["epsilon"], epsilon_decay_rate=hp["epsilon_decay_rate"],
                         lr=hp["lr"], lr_decay_rate=hp["lr_decay_rate"], default_q=hp["default_q"], seed=seed,
                         trace=trace)
    return env, model
