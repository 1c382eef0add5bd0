"""Synthetic SwitchFL scenarios: square Flatland-format rail grids + trains + timetable.

The reference builds its maps with Flatland's ``sparse_rail_generator`` /
``sparse_line_generator`` (test_model.py:31-44, main.py:45-60), which are not
installed here.  This module generates the same *kind* of input — a square
grid of 16-bit Flatland cell transitions whose junctions are only the four
switch classes SwitchFL accepts (switch_agents.py:262-267: (ports, routes) =
(3,4) T/Y, (4,4) diamond, (4,6) single slip, (4,8) double slip), trains with
start cell/heading, target station, earliest departure and latest arrival —
deterministically from a seed.

Conventions (Flatland's): headings/sides N=0, E=1, S=2, W=3; bit
``15 - (4*heading + exit)`` of a cell's 16-bit word says a train *moving* in
``heading`` may leave the cell through side ``exit`` (the ``dir_combo`` table
of rail_graph.py:168-187).

A cell is described by the set of undirected side pairs its rails connect;
every pair is traversable both ways, so every intra-switch edge gets
``rail_nodes=[]`` in the reference's port graph (rail_graph.py:222-235).

The generator lays a Manhattan grid of track lines, removes a few boundary
segments to hit the requested switch count, picks a junction layout per
intersection, and retries until the (cell, heading) state graph is strongly
connected (so every Flatland distance the reference evaluates in
observer.compute_delay is finite — observer.py:35-36 raises otherwise).
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass, field, asdict
from typing import Dict, FrozenSet, List, Optional, Sequence, Set, Tuple

import numpy as np

N, E, S, W = 0, 1, 2, 3
DELTA = ((-1, 0), (0, 1), (1, 0), (0, -1))


def opposite(d: int) -> int:
    return (d + 2) % 4


def pairs_to_bits(pairs) -> int:
    """16-bit Flatland transition word of a cell from its undirected side pairs."""
    bits = 0
    for pr in pairs:
        a, b = tuple(pr)
        for enter_side, exit_side in ((a, b), (b, a)):
            heading = opposite(enter_side)  # entering through side a means moving away from it
            bits |= 1 << (15 - (4 * heading + exit_side))
    return bits


def transitions(word: int, heading: int) -> Tuple[int, int, int, int]:
    """Exit bits (N, E, S, W) for a train moving in ``heading`` inside a cell."""
    nib = (word >> ((3 - heading) * 4)) & 0xF
    return ((nib >> 3) & 1, (nib >> 2) & 1, (nib >> 1) & 1, nib & 1)


@dataclass
class Train:
    initial_position: Tuple[int, int]
    initial_direction: int
    target: Tuple[int, int]
    earliest_departure: int = 0
    latest_arrival: int = 0


@dataclass
class Scenario:
    """Everything the hot path needs to (re)start an episode; the map is static."""
    height: int
    width: int
    grid: List[List[int]]            # [H][W] 16-bit transition words
    trains: List[Train]
    max_episode_steps: int
    malfunction_rate: float = 0.0
    malfunction_min: int = 0
    malfunction_max: int = 0
    name: str = ""
    seed: int = 0

    # -- helpers ---------------------------------------------------------
    def grid_array(self) -> np.ndarray:
        return np.asarray(self.grid, dtype=np.int64)

    def to_json(self) -> str:
        d = asdict(self)
        return json.dumps(d, sort_keys=True)

    @staticmethod
    def from_json(s: str) -> "Scenario":
        d = json.loads(s)
        trains = [Train(tuple(t["initial_position"]), int(t["initial_direction"]), tuple(t["target"]),
                        int(t["earliest_departure"]), int(t["latest_arrival"])) for t in d.pop("trains")]
        return Scenario(trains=trains, **d)

    def save(self, path: str) -> None:
        with open(path, "w") as f:
            f.write(self.to_json())

    @staticmethod
    def load(path: str) -> "Scenario":
        with open(path) as f:
            return Scenario.from_json(f.read())

    def with_malfunctions(self, rate: float, lo: int, hi: int) -> "Scenario":
        d = Scenario.from_json(self.to_json())
        d.malfunction_rate, d.malfunction_min, d.malfunction_max = float(rate), int(lo), int(hi)
        return d


# ---------------------------------------------------------------------------
# state graph utilities (used for validation + timetable)
# ---------------------------------------------------------------------------

def _step_state(grid: np.ndarray, r: int, c: int, heading: int):
    """All successor states (r', c', heading') of a train moving in ``heading`` at (r, c)."""
    word = int(grid[r, c])
    out = []
    for e, ok in enumerate(transitions(word, heading)):
        if ok:
            dr, dc = DELTA[e]
            out.append((r + dr, c + dc, e))
    return out


def rail_states(grid: np.ndarray):
    H, W = grid.shape
    res = []
    for r in range(H):
        for c in range(W):
            if grid[r, c] == 0:
                continue
            for h in range(4):
                if any(transitions(int(grid[r, c]), h)):
                    res.append((r, c, h))
    return res


def strongly_connected(grid: np.ndarray) -> bool:
    states = rail_states(grid)
    if not states:
        return False
    idx = {s: i for i, s in enumerate(states)}
    fwd = [[] for _ in states]
    bwd = [[] for _ in states]
    for s in states:
        for t in _step_state(grid, *s):
            if t not in idx:
                return False  # leads off-rail / into a state with no exit
            fwd[idx[s]].append(idx[t])
            bwd[idx[t]].append(idx[s])

    def reach(adj):
        seen = [False] * len(states)
        stack = [0]
        seen[0] = True
        while stack:
            u = stack.pop()
            for v in adj[u]:
                if not seen[v]:
                    seen[v] = True
                    stack.append(v)
        return all(seen)

    return reach(fwd) and reach(bwd)


def distance_to_cell(grid: np.ndarray, target: Tuple[int, int]) -> np.ndarray:
    """BFS distance (in moves) from every (r, c, heading) state to ``target``; -1 = unreachable."""
    H, W = grid.shape
    dist = -np.ones((H, W, 4), dtype=np.int64)
    tr, tc = target
    # reverse adjacency on the fly: predecessor p of state (r,c,h) is any state whose move lands in (r,c) with heading h
    from collections import deque
    q = deque()
    for h in range(4):
        dist[tr, tc, h] = 0
        q.append((tr, tc, h))
    while q:
        r, c, h = q.popleft()
        # predecessor cell is one step against heading h
        pr, pc = r - DELTA[h][0], c - DELTA[h][1]
        if not (0 <= pr < H and 0 <= pc < W) or grid[pr, pc] == 0:
            continue
        for ph in range(4):
            if transitions(int(grid[pr, pc]), ph)[h] and dist[pr, pc, ph] < 0:
                dist[pr, pc, ph] = dist[r, c, h] + 1
                q.append((pr, pc, ph))
    return dist


# ---------------------------------------------------------------------------
# grid-of-lines network
# ---------------------------------------------------------------------------

def _junction_pairs(sides: Set[int], rng: np.random.Generator, slip_weights) -> FrozenSet[FrozenSet[int]]:
    sides = sorted(sides)
    if len(sides) == 2:
        return frozenset({frozenset(sides)})
    if len(sides) == 3:
        trunk = sides[int(rng.integers(0, 3))]
        others = [s for s in sides if s != trunk]
        return frozenset({frozenset((trunk, others[0])), frozenset((trunk, others[1]))})
    # four-way: diamond / single slip / double slip
    straight = {frozenset((N, S)), frozenset((E, W))}
    curves_a = [frozenset((W, S)), frozenset((E, N))]
    curves_b = [frozenset((W, N)), frozenset((E, S))]
    kind = rng.choice(3, p=slip_weights)
    if kind == 0:
        return frozenset(straight)
    if kind == 1:
        c = (curves_a + curves_b)[int(rng.integers(0, 4))]
        return frozenset(straight | {c})
    pick = curves_a if rng.integers(0, 2) == 0 else curves_b
    return frozenset(straight | set(pick))


def grid_network(nx_lines: int, ny_lines: int, spacing: int, margin: int, n_switches: int,
                 rng: np.random.Generator, slip_weights=(0.2, 0.3, 0.5), size: Optional[int] = None):
    """Lay out the line grid and return (grid words [H][W], set of junction cells)."""
    span = (max(nx_lines, ny_lines) - 1) * spacing + 1
    side_len = max(size or 0, 2 * margin + span)
    rows = [margin + i * spacing for i in range(ny_lines)]
    cols = [margin + j * spacing for j in range(nx_lines)]
    seg = {}  # ((i,j),(i2,j2)) -> present
    for i in range(ny_lines):
        for j in range(nx_lines):
            if j + 1 < nx_lines:
                seg[((i, j), (i, j + 1))] = True
            if i + 1 < ny_lines:
                seg[((i, j), (i + 1, j))] = True

    def sides_of(i, j):
        s = set()
        if seg.get(((i, j - 1), (i, j))):
            s.add(W)
        if seg.get(((i, j), (i, j + 1))):
            s.add(E)
        if seg.get(((i - 1, j), (i, j))):
            s.add(N)
        if seg.get(((i, j), (i + 1, j))):
            s.add(S)
        return s

    def n_sw():
        return sum(1 for i in range(ny_lines) for j in range(nx_lines) if len(sides_of(i, j)) >= 3)

    # remove boundary segments between two boundary T junctions until the count matches
    excess = n_sw() - n_switches
    if excess < 0:
        raise ValueError(f"grid {nx_lines}x{ny_lines} has only {n_sw()} switches < {n_switches}")
    boundary = [k for k in seg if (k[0][0] == k[1][0] and k[0][0] in (0, ny_lines - 1)) or
                (k[0][1] == k[1][1] and k[0][1] in (0, nx_lines - 1))]
    order = list(rng.permutation(len(boundary)))
    for bi in order:
        if excess <= 0:
            break
        a, b = boundary[bi]
        if not seg[(a, b)]:
            continue
        da, db = len(sides_of(*a)), len(sides_of(*b))
        if excess >= 2 and da == 3 and db == 3:
            seg[(a, b)] = False
            excess -= 2
    # odd remainder: drop an inward segment of a boundary T (T -> straight, 4-way -> T)
    if excess == 1:
        for (a, b), on in list(seg.items()):
            if not on:
                continue
            ca, cb = len(sides_of(*a)), len(sides_of(*b))
            ab = a[0] in (0, ny_lines - 1) or a[1] in (0, nx_lines - 1)
            bb = b[0] in (0, ny_lines - 1) or b[1] in (0, nx_lines - 1)
            if ab != bb and {ca, cb} == {3, 4}:
                seg[(a, b)] = False
                excess -= 1
                break
    if excess != 0 or n_sw() != n_switches:
        raise ValueError("could not reach requested switch count")

    pairs: Dict[Tuple[int, int], Set[FrozenSet[int]]] = {}
    # plain track along present segments
    for ((i, j), (i2, j2)), on in seg.items():
        if not on:
            continue
        if i == i2:  # horizontal
            r = rows[i]
            for c in range(cols[j] + 1, cols[j2]):
                pairs.setdefault((r, c), set()).add(frozenset((E, W)))
        else:
            c = cols[j]
            for r in range(rows[i] + 1, rows[i2]):
                pairs.setdefault((r, c), set()).add(frozenset((N, S)))
    junctions = set()
    for i in range(ny_lines):
        for j in range(nx_lines):
            sides = sides_of(i, j)
            if len(sides) < 2:
                if sides:
                    raise ValueError("dead end produced")
                continue
            pairs[(rows[i], cols[j])] = set(_junction_pairs(sides, rng, slip_weights))
            if len(sides) >= 3:
                junctions.add((rows[i], cols[j]))
    grid = np.zeros((side_len, side_len), dtype=np.int64)
    for (r, c), prs in pairs.items():
        grid[r, c] = pairs_to_bits(prs)
    return grid, junctions


def _first_switch_chain(grid: np.ndarray, junctions, pos, heading):
    """Cells visited from ``pos`` (inclusive) until the first junction cell (inclusive)."""
    r, c, h = pos[0], pos[1], heading
    cells = [(r, c)]
    for _ in range(grid.size + 1):
        nxt = _step_state(grid, r, c, h)
        if len(nxt) != 1:
            raise ValueError("plain cell with != 1 exit")
        r, c, h = nxt[0]
        cells.append((r, c))
        if (r, c) in junctions:
            return cells
    raise ValueError("no switch ahead")


def timetable(path_lengths: List[int], width: int, height: int, n_cities: int, rs: np.random.RandomState):
    """Earliest departure / latest arrival / max_episode_steps, restating the arithmetic of
    flatland_patch/timetable_generators.py:44-136 (single-segment lines, speed 1)."""
    num_agents = len(path_lengths)
    max_episode_steps = int(4 * 2 * (width + height + (num_agents / n_cities)))
    lengths = np.array(path_lengths, dtype=float)
    mean_path_delay = float(np.mean(lengths)) * 0.2
    new_steps = int(np.ceil(float(np.max(lengths)) * 1.5) + mean_path_delay)
    old_steps = int(max_episode_steps * 3.0)
    max_episode_steps = min(new_steps, old_steps)
    end_buffer = int(max_episode_steps * 0.05)
    latest_arrival_max = max_episode_steps - end_buffer
    eds, las = [], []
    for L in lengths:
        travel_max = int(np.ceil(L * 1.3 + mean_path_delay))
        window = max(latest_arrival_max - travel_max, 1)
        ed = int(rs.randint(0, window))
        eds.append(ed)
        las.append(ed + travel_max)
    return eds, las, max_episode_steps


def generate(n_switches: int, n_trains: int, n_stations: int, seed: int, *,
             nx_lines: Optional[int] = None, ny_lines: Optional[int] = None,
             spacing: int = 5, margin: int = 3, size: Optional[int] = None,
             malfunction: Tuple[float, int, int] = (0.0, 0, 0), name: str = "",
             slip_weights=(0.2, 0.3, 0.5), max_tries: int = 200) -> Scenario:
    """Deterministic scenario for (switch count, train count, station count, seed)."""
    if nx_lines is None or ny_lines is None:
        # smallest near-square line grid with nx*ny - 4 >= n_switches
        best = None
        for ny in range(2, 64):
            for nx in range(ny, ny + 2):
                if nx * ny - 4 >= n_switches and (best is None or nx * ny < best[0] * best[1]):
                    best = (nx, ny)
        nx_lines, ny_lines = best
    rng = np.random.default_rng(seed)
    for _ in range(max_tries):
        grid, junctions = grid_network(nx_lines, ny_lines, spacing, margin, n_switches, rng,
                                       slip_weights=slip_weights, size=size)
        if not strongly_connected(grid):
            continue
        Hh, Ww = grid.shape
        # candidate cells: straight plain cells not adjacent to a junction
        plain = []
        for r in range(Hh):
            for c in range(Ww):
                w = int(grid[r, c])
                if w == 0 or (r, c) in junctions:
                    continue
                if w not in (pairs_to_bits({frozenset((E, W))}), pairs_to_bits({frozenset((N, S))})):
                    continue
                if any((r + dr, c + dc) in junctions for dr, dc in DELTA):
                    continue
                plain.append((r, c))
        if len(plain) < n_trains + n_stations:
            raise ValueError("map too small for trains + stations")
        perm = rng.permutation(len(plain))
        stations = [plain[i] for i in perm[:n_stations]]
        starts_pool = [plain[i] for i in perm[n_stations:]]
        dists = {s: distance_to_cell(grid, s) for s in stations}
        trains: List[Train] = []
        ok = True
        for k in range(n_trains):
            placed = False
            for _try in range(50):
                if not starts_pool:
                    break
                pos = starts_pool.pop(int(rng.integers(0, len(starts_pool))))
                w = int(grid[pos])
                heads = [h for h in range(4) if any(transitions(w, h))]
                h0 = heads[int(rng.integers(0, len(heads)))]
                tgt = stations[int(rng.integers(0, n_stations))]
                chain = _first_switch_chain(grid, junctions, pos, h0)
                if tgt in chain:
                    continue
                if dists[tgt][pos[0], pos[1], h0] < 0:
                    continue
                trains.append(Train((int(pos[0]), int(pos[1])), int(h0), (int(tgt[0]), int(tgt[1]))))
                placed = True
                break
            if not placed:
                ok = False
                break
        if not ok:
            continue
        trains.sort(key=lambda t: (t.initial_position[0], t.initial_position[1], t.initial_direction))
        # shortest path lengths in waypoints (Flatland's len(path) counts start and target)
        lens = [int(dists[t.target][t.initial_position[0], t.initial_position[1], t.initial_direction]) + 1
                for t in trains]
        rs = np.random.RandomState(seed & 0x7FFFFFFF)
        eds, las, mes = timetable(lens, Ww, Hh, max(2, n_stations), rs)
        for t, ed, la in zip(trains, eds, las):
            t.earliest_departure, t.latest_arrival = ed, la
        return Scenario(height=Hh, width=Ww, grid=[[int(x) for x in row] for row in grid], trains=trains,
                        max_episode_steps=int(mes), malfunction_rate=float(malfunction[0]),
                        malfunction_min=int(malfunction[1]), malfunction_max=int(malfunction[2]),
                        name=name, seed=int(seed))
    raise RuntimeError("could not generate a strongly connected scenario")


# ---------------------------------------------------------------------------
# Flatland-like city maps
# ---------------------------------------------------------------------------

def _straight(r0: int, c0: int, r1: int, c1: int, pairs: Dict[Tuple[int, int], Set[FrozenSet[int]]]) -> None:
    """Plain track strictly between two cells of one row or column."""
    if r0 == r1:
        for c in range(min(c0, c1) + 1, max(c0, c1)):
            pairs.setdefault((r0, c), set()).add(frozenset((E, W)))
    else:
        for r in range(min(r0, r1) + 1, max(r0, r1)):
            pairs.setdefault((r, c0), set()).add(frozenset((N, S)))


def _passing_loop(pairs, r0: int, c0: int, r1: int, c1: int, off: int):
    """A second rail beside the plain segment (r0, c0) - (r1, c1) of one row or column, ``off`` cells in from
    each end: T switches on the main line (trunks facing the segment's ends) and a parallel track two cells
    below (rows) or right (columns) -- two rails between the segment's junctions, so trains meeting on it can
    pass (Flatland's max_rails_between_cities = 2)."""
    if r0 == r1:
        xa, xb, rr = min(c0, c1) + off, max(c0, c1) - off, r0 + 2
        pairs[(r0, xa)].add(frozenset((W, S)))
        pairs[(r0, xb)].add(frozenset((E, S)))
        _straight(r0, xa, rr, xa, pairs)
        _straight(r0, xb, rr, xb, pairs)
        pairs.setdefault((rr, xa), set()).add(frozenset((N, E)))
        pairs.setdefault((rr, xb), set()).add(frozenset((N, W)))
        _straight(rr, xa, rr, xb, pairs)
        return [(r0, xa), (r0, xb)]
    else:
        ya, yb, cc = min(r0, r1) + off, max(r0, r1) - off, c0 + 2
        pairs[(ya, c0)].add(frozenset((N, E)))
        pairs[(yb, c0)].add(frozenset((S, E)))
        _straight(ya, c0, ya, cc, pairs)
        _straight(yb, c0, yb, cc, pairs)
        pairs.setdefault((ya, cc), set()).add(frozenset((W, S)))
        pairs.setdefault((yb, cc), set()).add(frozenset((W, N)))
        _straight(ya, cc, yb, cc, pairs)
        return [(ya, c0), (yb, c0)]


def city_network(n_lines: int, spacing: int, margin: int, cities: List[Tuple[int, int, int]],
                 rng: np.random.Generator, slip_weights=(0.2, 0.3, 0.5), size: Optional[int] = None,
                 rails: int = 1, loop_off: int = 4):
    """A square backbone of ``n_lines`` x ``n_lines`` rail lines (the inter-city connections) with
    cities on horizontal backbone segments, the way Flatland's sparse_rail_generator lays out a
    city: ``P`` parallel tracks (the backbone line plus P-1 sidings two rows apart) between two
    throats, each siding joining the main line through a T switch whose trunk faces out of the
    city.  ``cities``: (row line i, column line j, tracks P) -- the city sits between column lines
    j and j+1 on row line i.  ``size``: pad the grid to at least size x size (empty cells).  Returns
    (grid, junction cells, per-city track cells, throat cells).  ``rails`` = 2: every backbone segment that
    holds no city gets a passing loop (``_passing_loop``), the stand-in for Flatland's parallel inter-city
    rails (max_rails_between_cities); a city's own parallel tracks already give its segment several rails."""
    side_len = max(size or 0, 2 * margin + (n_lines - 1) * spacing + 1)
    pos = [margin + k * spacing for k in range(n_lines)]
    pairs: Dict[Tuple[int, int], Set[FrozenSet[int]]] = {}
    for i in range(n_lines):
        for j in range(n_lines - 1):
            _straight(pos[i], pos[j], pos[i], pos[j + 1], pairs)
            _straight(pos[j], pos[i], pos[j + 1], pos[i], pairs)
    junctions = set()
    for i in range(n_lines):
        for j in range(n_lines):
            sides = {d for d, ok in ((N, i > 0), (S, i < n_lines - 1), (W, j > 0), (E, j < n_lines - 1)) if ok}
            pairs[(pos[i], pos[j])] = set(_junction_pairs(sides, rng, slip_weights))
            if len(sides) >= 3:
                junctions.add((pos[i], pos[j]))
    city_tracks, throats = [], set()
    for (i, j, P) in cities:
        r0, cw, ce = pos[i], pos[j], pos[j + 1]
        a, b = cw + 2 * P, ce - 2 * P  # the city's platform span on every track
        if b - a < (6 if P <= 3 else 4) or (i + 1 < n_lines and pos[i + 1] - r0 < 2 * P + 2) or (i + 1 >= n_lines and 2 * P > margin + 1):
            raise ValueError("city does not fit its backbone segment")
        tracks = [[(r0, c) for c in range(a + 1, b)]]
        for k in range(1, P):
            rk, xw, xe = r0 + 2 * k, a - (2 * k - 1), b + (2 * k - 1)
            # throats: the main line's cell becomes a T (trunk out of the city)
            pairs[(r0, xw)].add(frozenset((W, S)))
            pairs[(r0, xe)].add(frozenset((E, S)))
            junctions.update({(r0, xw), (r0, xe)})
            throats.update({(r0, xw), (r0, xe)})
            _straight(r0, xw, rk, xw, pairs)
            _straight(r0, xe, rk, xe, pairs)
            pairs.setdefault((rk, xw), set()).add(frozenset((N, E)))
            pairs.setdefault((rk, xe), set()).add(frozenset((N, W)))
            _straight(rk, xw, rk, xe, pairs)
            tracks.append([(rk, c) for c in range(a + 1, b)])
        city_tracks.append(tracks)
    if rails >= 2:
        with_city = {(i, j) for (i, j, _) in cities}
        for i in range(n_lines):
            for j in range(n_lines - 1):
                if (i, j) not in with_city and pos[j + 1] - pos[j] >= 2 * loop_off + 3:
                    junctions.update(_passing_loop(pairs, pos[i], pos[j], pos[i], pos[j + 1], loop_off))
                if pos[j + 1] - pos[j] >= 2 * loop_off + 3:
                    junctions.update(_passing_loop(pairs, pos[j], pos[i], pos[j + 1], pos[i], loop_off))
    grid = np.zeros((side_len, side_len), dtype=np.int64)
    for (r, c), prs in pairs.items():
        grid[r, c] = pairs_to_bits(prs)
    return grid, junctions, city_tracks, throats


def generate_cities(n_cities: int, n_trains: int, seed: int, *, n_lines: Optional[int] = None, spacing: int = 20,
                    margin: int = 7, tracks: Tuple[int, int] = (2, 3), malfunction: Tuple[float, int, int] = (0.0, 0, 0),
                    name: str = "", slip_weights=(0.2, 0.3, 0.5), max_tries: int = 200,
                    size: Optional[int] = None, rails: int = 1, track_choices: Optional[Sequence[int]] = None) -> Scenario:
    """Flatland-like scenario: ``n_cities`` cities of 2-3 parallel tracks with one station each on a
    square backbone of inter-city lines; every train starts on a city track and targets the station
    of another city; timetable as flatland_patch/timetable_generators.py (``timetable``)."""
    if n_lines is None:
        n_lines = 2
        while n_lines * (n_lines - 1) < n_cities:
            n_lines += 1
    slots = [(i, j) for i in range(n_lines) for j in range(n_lines - 1)]
    if n_cities > len(slots) or n_cities < 2:
        raise ValueError("2 <= n_cities <= n_lines * (n_lines - 1)")
    rng = np.random.default_rng(seed)
    for _ in range(max_tries):
        pick = sorted(int(x) for x in rng.choice(len(slots), size=n_cities, replace=False))
        if track_choices:  # Flatland: 2 * randint(1, max_rail_pairs_in_city + 1) tracks per city
            cities = [(slots[q][0], slots[q][1], int(track_choices[int(rng.integers(0, len(track_choices)))]))
                      for q in pick]
        else:
            cities = [(slots[q][0], slots[q][1], int(rng.integers(tracks[0], tracks[1] + 1))) for q in pick]
        grid, junctions, city_tracks, throats = city_network(n_lines, spacing, margin, cities, rng, slip_weights,
                                                             size=size, rails=rails)
        if not strongly_connected(grid):
            continue
        near_junction = lambda rc: any((rc[0] + dr, rc[1] + dc) in junctions for dr, dc in DELTA)  # noqa: E731
        stations, pools = [], []
        for tr in city_tracks:
            t = tr[int(rng.integers(0, len(tr)))]
            cells = t[len(t) // 3: 2 * len(t) // 3 + 1]
            st = cells[int(rng.integers(0, len(cells)))]
            stations.append(st)
            pools.append([c for trk in tr for c in trk if c != st and not near_junction(c)])
        dists = {st: distance_to_cell(grid, st) for st in stations}
        trains: List[Train] = []
        used = set()
        for k in range(n_trains):
            placed = False
            for _try in range(100):
                home = int(rng.integers(0, n_cities))
                cand = [c for c in pools[home] if c not in used]
                if not cand:
                    continue
                p0 = cand[int(rng.integers(0, len(cand)))]
                h0 = (E, W)[int(rng.integers(0, 2))]
                dest = int(rng.integers(0, n_cities - 1))
                dest = dest + 1 if dest >= home else dest
                tgt = stations[dest]
                if tgt in _first_switch_chain(grid, junctions, p0, h0) or dists[tgt][p0[0], p0[1], h0] < 0:
                    continue
                used.add(p0)
                trains.append(Train((int(p0[0]), int(p0[1])), int(h0), (int(tgt[0]), int(tgt[1]))))
                placed = True
                break
            if not placed:
                break
        if len(trains) != n_trains:
            continue
        trains.sort(key=lambda t: (t.initial_position[0], t.initial_position[1], t.initial_direction))
        lens = [int(dists[t.target][t.initial_position[0], t.initial_position[1], t.initial_direction]) + 1
                for t in trains]
        Hh, Ww = grid.shape
        rs = np.random.RandomState(seed & 0x7FFFFFFF)
        eds, las, mes = timetable(lens, Ww, Hh, n_cities, rs)
        for t, ed, la in zip(trains, eds, las):
            t.earliest_departure, t.latest_arrival = ed, la
        return Scenario(height=Hh, width=Ww, grid=[[int(x) for x in row] for row in grid], trains=trains,
                        max_episode_steps=int(mes), malfunction_rate=float(malfunction[0]),
                        malfunction_min=int(malfunction[1]), malfunction_max=int(malfunction[2]),
                        name=name, seed=int(seed))
    raise RuntimeError("could not generate a strongly connected city scenario")


# Named configurations (BASELINE.json configs)
CONFIGS = {
    # C1: stands in for test_model.py's 18x18 / 5 cities / 2 trains map (Flatland's own map is unobtainable offline)
    "c1": dict(n_switches=5, n_trains=2, n_stations=2, nx_lines=3, ny_lines=3, spacing=6, margin=2, size=18),
    "c2": dict(n_switches=16, n_trains=8, n_stations=4, nx_lines=5, ny_lines=4, spacing=5, margin=2),
    "c3": dict(n_switches=64, n_trains=32, n_stations=8, nx_lines=9, ny_lines=8, spacing=5, margin=3),
    "c5": dict(n_switches=256, n_trains=128, n_stations=16, nx_lines=17, ny_lines=16, spacing=5, margin=3),
}

MAP_SEED = 450565  # the reference default seed (test_model.py:30)


def make_config(name: str, seed: int = MAP_SEED, malfunction=(0.01, 5, 15)) -> Scenario:
    kw = dict(CONFIGS[name])
    return generate(seed=seed, malfunction=malfunction, name=name, **kw)


CITY_SPACING = 18  # backbone line spacing a 3-track city needs (city_network: 4 P + 6 cells)
CITY_MARGIN = 7


def from_flatland_params(width: int, height: int, max_num_cities: int, number_of_agents: int, seed: int,
                         malfunction=(0.0, 0, 0), spacing: int = 5, margin: int = 3,
                         max_rails_between_cities: Optional[int] = None,
                         max_rail_pairs_in_city: Optional[int] = None, layout: str = "auto") -> Scenario:
    """Scenario for the reference's [ENV] config keys (main.py:21-60) on a width x height grid.

    Flatland's sparse_rail_generator is absent, so this is a stand-in layout, not its output (parity
    of the generated map is unpinned).  With two or more cities: a ``generate_cities`` layout (cities
    of parallel tracks on a square backbone of >= 3 x 3 lines) inside width x height;
    ``max_num_cities`` is a cap, as in Flatland, which places as many cities as fit -- here the
    largest backbone that fits the grid decides.  With one city, or a grid too small for a backbone
    (< 51 cells), a line grid of that size with one station per city.
    ``max_rails_between_cities`` >= 2 gives every backbone segment without a city a passing loop (two rails
    between its junctions; a city's segment has its own parallel tracks); ``max_rail_pairs_in_city`` = k gives
    each city 2 * randint(1, k + 1) tracks, as Flatland draws them.  Left out (None), the round-2 layout:
    single-track backbone, 2-3 tracks per city.

    Round 4: with ``max_rails_between_cities`` given, the cities are joined as Flatland joins them -- each link
    between neighbouring cities a rail path of its own (``max_rails_between_cities`` of them, at most two),
    switches only at the cities -- on a lattice of as many cities as fit the grid, up to ``max_num_cities``
    (``generate_city_grid``).  ``layout="backbone"`` keeps the round-3 layout (cities on a square backbone of
    shared four-way junctions, a passing loop per segment) for the fixtures recorded on it."""
    import warnings
    size = max(int(width), int(height))
    n_cities, n_agents = int(max_num_cities), int(number_of_agents)
    rails = int(max_rails_between_cities) if max_rails_between_cities is not None else 1
    choices = None
    spacing_need = CITY_SPACING
    if max_rail_pairs_in_city is not None:
        choices = [2 * k for k in range(1, max(1, int(max_rail_pairs_in_city)) + 1)]
        spacing_need = max(CITY_SPACING if max(choices) <= 3 else 0, 4 * max(choices) + 4)
    if rails > 2:
        warnings.warn(f"max_rails_between_cities={rails}: the stand-in layout lays at most two rails per link",
                      stacklevel=2)
    if layout not in ("auto", "backbone"):
        raise ValueError(f"layout {layout!r}: 'auto' or 'backbone'")
    if max_rails_between_cities is not None and n_cities >= 2 and layout == "auto":
        # round 4: Flatland's way of joining cities -- every link between two neighbouring cities a rail path of
        # its own, switches only at the cities (generate_city_grid); as many cities as fit the grid, up to
        # max_num_cities (Flatland places cities until it runs out of room or reaches the cap)
        pairs = int(max_rail_pairs_in_city) if max_rail_pairs_in_city is not None else 1
        tracks = [2 * k for k in range(1, max(1, pairs) + 1)]
        r_fit, c_fit = city_grid_fit(size, max(tracks))
        if r_fit * c_fit >= 2:
            cols = min(c_fit, max(1, n_cities))
            rows = min(r_fit, max(1, n_cities // cols))
            if rows * cols < 2:
                rows, cols = min(r_fit, 2), 1
            if n_cities > rows * cols:
                warnings.warn(f"max_num_cities={n_cities}: only {rows * cols} cities fit a {size}x{size} grid",
                              stacklevel=2)
            return generate_city_grid(rows, cols, n_agents, seed=int(seed), track_choices=tracks,
                                      rails=min(max(rails, 1), 2), size=size, malfunction=malfunction,
                                      name=f"flatland_{width}x{height}")
    n_fit = (size - 2 * CITY_MARGIN - 1) // spacing_need + 1  # backbone lines that fit the grid
    if n_cities >= 2 and n_fit >= 3:  # (a two-line backbone is a loop a train cannot turn around on)
        n_lines = 3
        while n_lines * (n_lines - 1) < n_cities and n_lines < n_fit:
            n_lines += 1
        cap = n_lines * (n_lines - 1)
        if n_cities > cap:
            warnings.warn(f"max_num_cities={n_cities}: only {cap} cities fit a {size}x{size} grid", stacklevel=2)
            n_cities = cap
        c_spacing = (size - 2 * CITY_MARGIN - 1) // (n_lines - 1)
        return generate_cities(n_cities, n_agents, seed=int(seed), n_lines=n_lines, spacing=c_spacing,
                               margin=CITY_MARGIN, malfunction=malfunction, name=f"flatland_{width}x{height}",
                               size=size, rails=rails, track_choices=choices)
    n_lines = max(3, (size - 2 * margin - 1) // spacing + 1)
    n_sw = n_lines * n_lines - 4
    return generate(n_switches=n_sw, n_trains=n_agents, n_stations=max(1, min(n_cities, n_agents)), seed=int(seed),
                    nx_lines=n_lines, ny_lines=n_lines, spacing=spacing, margin=margin, size=size,
                    malfunction=malfunction, name=f"flatland_{width}x{height}")


# ---------------------------------------------------------------------------
# Flatland-like city graph (round 4): cities joined by their own rail paths
# ---------------------------------------------------------------------------

def city_grid_network(n_rows: int, n_cols: int, tracks: List[List[int]], *, plat: int = 6, margin: int = 2,
                      rails: int = 1, size: Optional[int] = None):
    """Cities on an ``n_rows`` x ``n_cols`` lattice, joined the way Flatland's sparse_rail_generator joins them --
    each link between two neighbouring cities is a rail path of its own, and switches sit at the cities (there is
    no shared junction between links):

    * city (i, j) has ``tracks[i][j]`` parallel platform tracks; the first lies on its row's main line, the others
      below it, each joined to the main line at both ends of the platforms by a T switch whose trunk faces out of
      the city (a throat, as in ``city_network``);
    * the cities of a row are joined by that main line (west-east links); its two ends turn into a return track two
      rows above, and a chord near each end joins the two (T switches), so a train can turn round on its row;
    * city (i, j) is joined to city (i + 1, j) by ``rails`` vertical rail paths (Flatland's
      max_rails_between_cities) on the east side of both cities: each leaves the upper city's main line at a T
      switch (trunk facing the city) and enters the lower city's main line at another (trunk facing the city), so
      a train leaving either city eastwards may take it and arrives heading into the other city; a path crossing
      the lower row's return track does so at a diamond crossing (no switching).

    Returns (grid, junction cells, per-city track cells, per-city (row, platform span))."""
    Pm = max(max(r) for r in tracks)
    tw = 2 * Pm - 1                 # a throat's extent beyond the platform span
    # per link column pair: rows i even use columns +2 / +4, rows i odd +6 / +8 past the city's east throat
    foot = 2 * tw + plat + 1         # a city's span on its row, throats included
    sp_c = foot + 12                 # + its east links (2 columns) and the next city's west links (2), with gaps
    sp_r = 2 * (Pm - 1) + 4
    xL = margin
    R0 = margin + 2
    xR = xL + 10 + (n_cols - 1) * sp_c + foot + 8
    rows = [R0 + i * sp_r for i in range(n_rows)]
    side = max(size or 0, xR + margin + 1, rows[-1] + 2 * (Pm - 1) + margin + 1)
    if rows[-1] + 2 * (Pm - 1) > side - 1 or xR > side - 1:
        raise ValueError("city grid does not fit")
    pairs: Dict[Tuple[int, int], Set[FrozenSet[int]]] = {}

    def add(r, c, a, b):
        pairs.setdefault((r, c), set()).add(frozenset((a, b)))

    junctions: Set[Tuple[int, int]] = set()
    city_tracks, city_spans = [], []
    for i, R in enumerate(rows):
        # the row loop: main line R from xL to xR, return track R - 2, end verticals
        _straight(R, xL, R, xR, pairs)
        _straight(R - 2, xL, R - 2, xR, pairs)
        add(R, xL, E, N)
        add(R - 1, xL, N, S)
        add(R - 2, xL, S, E)
        add(R, xR, W, N)
        add(R - 1, xR, N, S)
        add(R - 2, xR, S, W)
        # a chord near each end, so that a train can turn round on its row: westbound on the main line it may
        # climb the west chord and come back eastbound (round the west end), eastbound the east chord
        for xc, tm, tr_ in ((xL + 2, E, W), (xR - 2, W, E)):
            add(R, xc, tm, N)
            add(R - 1, xc, N, S)
            add(R - 2, xc, tr_, S)
            junctions.update({(R, xc), (R - 2, xc)})
        for j in range(n_cols):
            P = int(tracks[i][j])
            a = xL + 10 + j * sp_c + tw      # platform cells a + 1 .. b - 1
            b = a + plat + 1
            trk = [[(R, c) for c in range(a + 1, b)]]
            for k in range(1, P):
                rk, xw, xe = R + 2 * k, a - (2 * k - 1), b + (2 * k - 1)
                add(R, xw, W, S)
                add(R, xe, E, S)
                junctions.update({(R, xw), (R, xe)})
                _straight(R, xw, rk, xw, pairs)
                _straight(R, xe, rk, xe, pairs)
                add(rk, xw, N, E)
                add(rk, xe, N, W)
                _straight(rk, xw, rk, xe, pairs)
                trk.append([(rk, c) for c in range(a + 1, b)])
            city_tracks.append(trk)
            city_spans.append((R, a, b))
            if i + 1 < n_rows:
                R2 = rows[i + 1]
                for q in range(max(1, int(rails))):
                    # the first link on the cities' east side, the second on their west side (trunks facing the
                    # cities: trains leaving a city may take a link, trains off a link head into the city)
                    east = q % 2 == 0
                    X = (b + tw + 2 + (2 if i % 2 else 0)) if east else (a - tw - 3 - (2 if i % 2 else 0))
                    tk = W if east else E
                    add(R, X, tk, S)
                    add(R2, X, tk, N)
                    _straight(R, X, R2, X, pairs)
                    add(R2 - 2, X, N, S)  # crosses the lower row's return track (diamond)
                    junctions.update({(R, X), (R2, X), (R2 - 2, X)})
    grid = np.zeros((side, side), dtype=np.int64)
    for (r, c), prs in pairs.items():
        grid[r, c] = pairs_to_bits(prs)
    return grid, junctions, city_tracks, city_spans


def city_grid_fit(size: int, max_tracks: int, plat: int = 6, margin: int = 2) -> Tuple[int, int]:
    """(rows, columns) of cities ``city_grid_network`` fits into a size x size grid."""
    tw = 2 * max_tracks - 1
    foot = 2 * tw + plat + 1
    sp_c, sp_r = foot + 12, 2 * (max_tracks - 1) + 4
    cols = 0
    while margin + 10 + cols * sp_c + foot + 8 + margin + 1 <= size:
        cols += 1
    rows = 0
    while margin + 2 + rows * sp_r + 2 * (max_tracks - 1) + margin + 1 <= size:
        rows += 1
    return rows, cols


def generate_city_grid(n_rows: int, n_cols: int, n_trains: int, seed: int, *, track_choices: Sequence[int] = (2, 4),
                       rails: int = 1, plat: int = 6, size: Optional[int] = None,
                       malfunction: Tuple[float, int, int] = (0.0, 0, 0), name: str = "", max_tries: int = 200) -> Scenario:
    """Scenario on ``city_grid_network``: one station per city (a platform cell in the middle third of one of its
    tracks), trains starting on city tracks and targeting another city's station, timetable as
    flatland_patch/timetable_generators.py (``timetable``).  ``track_choices``: a city's track count is drawn from it
    (Flatland: 2 * randint(1, max_rail_pairs_in_city + 1))."""
    n_cities = n_rows * n_cols
    if n_cities < 2:
        raise ValueError("at least two cities")
    rng = np.random.default_rng(seed)
    for _ in range(max_tries):
        tracks = [[int(track_choices[int(rng.integers(0, len(track_choices)))]) for _j in range(n_cols)]
                  for _i in range(n_rows)]
        grid, junctions, city_tracks, _spans = city_grid_network(n_rows, n_cols, tracks, plat=plat, rails=rails, size=size)
        if not strongly_connected(grid):
            continue
        near_junction = lambda rc: any((rc[0] + dr, rc[1] + dc) in junctions for dr, dc in DELTA)  # noqa: E731
        stations, pools = [], []
        for tr in city_tracks:
            t = tr[int(rng.integers(0, len(tr)))]
            cells = t[len(t) // 3: 2 * len(t) // 3 + 1]
            st = cells[int(rng.integers(0, len(cells)))]
            stations.append(st)
            pools.append([c for trk in tr for c in trk if c != st and not near_junction(c)])
        dists = {st: distance_to_cell(grid, st) for st in stations}
        trains: List[Train] = []
        used = set()
        for _k in range(n_trains):
            placed = False
            for _try in range(100):
                home = int(rng.integers(0, n_cities))
                cand = [c for c in pools[home] if c not in used]
                if not cand:
                    continue
                p0 = cand[int(rng.integers(0, len(cand)))]
                h0 = (E, W)[int(rng.integers(0, 2))]
                dest = int(rng.integers(0, n_cities - 1))
                dest = dest + 1 if dest >= home else dest
                tgt = stations[dest]
                if tgt in _first_switch_chain(grid, junctions, p0, h0) or dists[tgt][p0[0], p0[1], h0] < 0:
                    continue
                used.add(p0)
                trains.append(Train((int(p0[0]), int(p0[1])), int(h0), (int(tgt[0]), int(tgt[1]))))
                placed = True
                break
            if not placed:
                break
        if len(trains) != n_trains:
            continue
        trains.sort(key=lambda t: (t.initial_position[0], t.initial_position[1], t.initial_direction))
        lens = [int(dists[t.target][t.initial_position[0], t.initial_position[1], t.initial_direction]) + 1
                for t in trains]
        Hh, Ww = grid.shape
        rs = np.random.RandomState(seed & 0x7FFFFFFF)
        eds, las, mes = timetable(lens, Ww, Hh, n_cities, rs)
        for t, ed, la in zip(trains, eds, las):
            t.earliest_departure, t.latest_arrival = ed, la
        return Scenario(height=Hh, width=Ww, grid=[[int(x) for x in row] for row in grid], trains=trains,
                        max_episode_steps=int(mes), malfunction_rate=float(malfunction[0]),
                        malfunction_min=int(malfunction[1]), malfunction_max=int(malfunction[2]),
                        name=name, seed=int(seed))
    raise RuntimeError("could not generate a strongly connected city-grid scenario")
