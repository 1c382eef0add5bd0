"""Graph-partitioned SwitchFL learner (BASELINE.json configs[4], SURVEY.md §8(e) "C5").

The reference's learner is a network of switch agents: each switch keeps its own Q-table
(the dict partitioned by the switch coordinates, distr_q.py:47-57) and bootstraps from the
*successor* agent's row, ``max_q(next_state, next_agent)`` (distr_q.py:419-466).  Here the
switch agents are partitioned over the ranks (one process per GPU): rank r owns the Q rows of
its switches for every env of the job and answers the row lookups for them; envs are sharded
over the ranks as in the env-sharded mode.  Each round every env makes one decision:

    sfl_part_local    apply last round's reply, run to the next decision, emit its request
                      (and the update records of the post step), packed per destination rank
                      with each env's records as one contiguous group
    all-to-all        the message segments  (RCCL over xGMI: torch.distributed "nccl")
    sfl_part_owner    owner, per env group: the bootstrapped updates in order, then max over
                      the requested row + masked argmax
    all-to-all        replies back

Two collectives per round.  Every env performs exactly the operations of the fused kernels in
the same order, so the results are bit-identical to the single-process run
(tests/test_partition.py).  Message buffers are [world][k + 1] record segments whose first
record carries the count; an env whose group does not fit a segment is deferred whole to a later
round (k_part_compact), so each exchange is a fixed-size all-to-all.  On the GPU the rounds queue on one stream (this batch's
torch stream, handed to the library with sfl_set_stream; RCCL collectives follow it): the host
reads the counts only at checkpoint rounds (1, 2, 4, ..., 32, then every 32nd), where the ranks
also agree on the next segment sizes -- no host synchronisation in the rounds between.

CohortPipeline splits a rank's envs into independent cohorts -- each a PartitionedBatch with its own segments,
stream and process group -- and issues their rounds alternately, so one cohort's exchange and owner step run
beside another's local step (bench.py --partition --cohorts).
"""
from __future__ import annotations

import contextlib
import ctypes as C
from collections import deque
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .compiler import CompiledMap
from .runtime import Batch, _ptr


def partition_switches(cm: CompiledMap, world: int) -> np.ndarray:
    """owner[S]: contiguous blocks of a breadth-first order of the switch graph, so most rail
    edges (successor lookups) stay inside one rank."""
    S = cm.S
    nb = np.asarray(cm.arrays["port_nb"]).reshape(S, 4)
    adj = [sorted({int(p) >> 2 for p in nb[s] if p >= 0} - {s}) for s in range(S)]
    order: List[int] = []
    seen = [False] * S
    for s0 in range(S):
        if seen[s0]:
            continue
        seen[s0] = True
        dq = deque([s0])
        while dq:
            s = dq.popleft()
            order.append(s)
            for t in adj[s]:
                if not seen[t]:
                    seen[t] = True
                    dq.append(t)
    owner = np.zeros(S, np.int32)
    for i, s in enumerate(order):
        owner[s] = i * world // S
    return owner


def cut_fraction(cm: CompiledMap, owner: np.ndarray) -> float:
    """Fraction of switch-to-switch rail edges whose ends have different owners."""
    nb = np.asarray(cm.arrays["port_nb"]).reshape(cm.S, 4)
    e = c = 0
    for s in range(cm.S):
        for p in nb[s]:
            if p >= 0 and (int(p) >> 2) != s:
                e += 1
                c += int(owner[int(p) >> 2] != owner[s])
    return c / max(1, e)


class PartitionedBatch:
    """This rank's envs + its switch agents' Q rows.  ``dist``: torch.distributed (or None for one rank);
    ``device``: a torch device for the message buffers ("cuda" for the HIP library, "cpu" for the host build)."""

    def __init__(self, cm: CompiledMap, hp: dict, seeds: Sequence[int], env_base: int, envs_total: int,
                 rank: int = 0, world: int = 1, dist=None, lib: Optional[_lib.Lib] = None, device: int = 0,
                 owner: Optional[np.ndarray] = None, upd_per_env: int = 16, ntab: Optional[int] = None,
                 buffer_device: str = "cuda", local_rows=True, malfunction_stream: str = "counter",
                 delay_threshold: int = 20, k_init: Optional[int] = None, checkpoint_every_round: bool = False,
                 group=None, exchange_collective: bool = False):
        import torch
        self.torch = torch
        kw = {} if ntab is None else dict(ntab=ntab)
        kw["malfunction_stream"] = malfunction_stream
        kw["delay_threshold"] = int(delay_threshold)  # StandardObserver(delay_threshold=...), observer.py:221
        self.batch = Batch(cm, hp, seeds, lib=lib, device=device, **kw)
        self.lib = self.batch.lib
        self.cm, self.rank, self.world, self.dist = cm, int(rank), int(world), dist
        self.group = group  # the process group of this job's collectives (None: the default group)
        # (tests) with one rank too, exchange the segments as collectives of `dist` between separate send and receive
        # buffers -- with RCCL, the same stream ordering as a multi-GPU job's, on one GPU
        self.exchange_collective = bool(exchange_collective) and dist is not None
        self.E = self.batch.E
        self.env_base, self.envs_total = int(env_base), int(envs_total)
        self.owner = np.ascontiguousarray(owner if owner is not None else partition_switches(cm, world), np.int32)
        # a receiver's request segment from rank s must hold one request per env of s: size the
        # segments by the largest rank's env count, and check the job's env ranges add up
        e_max, e_sum = self._job_env_counts(buffer_device)
        if e_sum != self.envs_total:
            raise ValueError(f"envs_total={self.envs_total} but the ranks hold {e_sum} envs")
        self.cap_req = e_max
        # a rank with more envs may send more update records to a smaller rank than 16 per receiver env:
        # size every update segment from the job's largest shard, like the request segments
        self.cap_upd = max(64, upd_per_env * e_max)
        self.lib.check(self.lib.dll.sfl_part_config(self.batch.h, self.rank, self.world, _ptr(self.owner, C.c_int32),
                                                    self.env_base, self.envs_total, self.cap_req, self.cap_upd),
                       "sfl_part_config")
        ms, rp = C.c_uint32(), C.c_uint32()
        self.lib.check(self.lib.dll.sfl_part_record_sizes(C.byref(ms), C.byref(rp)), "sfl_part_record_sizes")
        # one segment per destination holds every env group of the largest rank: its requests and updates
        self.cap_msg = self.cap_req + self.cap_upd
        dev = torch.device(buffer_device)
        nmsg = self.world * (self.cap_msg + 1) * ms.value
        nrep = self.world * (self.cap_msg + 1) * rp.value
        z = lambda n: torch.zeros(n, dtype=torch.uint8, device=dev)  # noqa: E731
        if self.world == 1 and not self.exchange_collective:
            # one rank: every segment is addressed to this rank, so the exchange is the identity
            # and each receive buffer is its send buffer (no copies, no stream synchronisation)
            self.msg_send = self.msg_recv = z(nmsg)
            self.rep_send = self.rep_recv = z(nrep)
        else:
            self.msg_send, self.msg_recv = z(nmsg), z(nmsg)
            self.rep_send, self.rep_recv = z(nrep), z(nrep)
        self.on_gpu = dev.type == "cuda"
        self.rec = (ms.value, rp.value)
        self.rounds = 0
        self.last_rounds = 0  # rounds of the last completed step
        self._counts = (C.c_uint32 * (2 * self.world + 3))()   # sfl_part_counts, sfl_part.h PART_C_*
        self.k_msg = self.cap_msg
        self.host_reads = 0   # checkpoint reads of the counts (the host's only look at a round's results)
        self.checkpoints = 0
        self.deferrals = 0    # envs deferred by a full segment, summed over rounds
        # (tests) read the counts after every round, so that an error surfaces in the round that set it
        self.checkpoint_every_round = bool(checkpoint_every_round)
        self.error_round = None  # the round (within its step) at which the last step raised
        if k_init is not None:  # (tests: start below the demand, so that envs are deferred)
            self.set_caps(k_init)
        # rows of this rank's own switches are decided on / updated in place (no message to itself).
        # local_rows: True (all own switches), False (every row operation as a message: the message
        # path measured on one rank) or a [S] mask of own switches (e.g. one block of a bigger job's
        # partition: that job's message traffic rehearsed on one rank)
        if local_rows is True:
            mask = (self.owner == self.rank).astype(np.uint8)
        elif local_rows is False:
            mask = np.zeros(cm.S, np.uint8)
        else:
            mask = np.ascontiguousarray(local_rows, np.uint8)
        self.local_mask = mask
        self.local_rows = bool(mask.any())
        self.lib.check(self.lib.dll.sfl_part_set_local_rows(self.batch.h, _ptr(mask, C.c_uint8)),
                       "sfl_part_set_local_rows")
        self.stream = None
        if self.on_gpu:
            # the round's kernels, copies and collectives queue on one stream (torch's, inside
            # step()), so the owner steps need no host synchronisation: one per round, for the counts
            torch.cuda.current_stream().synchronize()
            self.stream = torch.cuda.Stream(device=dev)
            self.lib.check(self.lib.dll.sfl_set_stream(self.batch.h, C.c_void_p(self.stream.cuda_stream)),
                           "sfl_set_stream")

    def close(self):
        self.batch.close()

    def _job_env_counts(self, buffer_device):
        """(max, sum) of the ranks' local env counts (one small collective when world > 1)."""
        if self.dist is None or self.world == 1:
            return self.E, self.E
        torch = self.torch
        dev = "cuda" if (buffer_device == "cuda" and self.dist.get_backend(self.group) != "gloo") else "cpu"
        t = torch.tensor([self.E, -self.E], dtype=torch.int64, device=dev)
        mx = t.clone()
        self.dist.all_reduce(mx, op=self.dist.ReduceOp.MAX, group=self.group)
        sm = torch.tensor([self.E], dtype=torch.int64, device=dev)
        self.dist.all_reduce(sm, group=self.group)
        return int(mx[0]), int(sm[0])

    def _all_max(self, vals):
        """Element-wise MAX of per-rank integer vectors over the job (every rank gets the same answer)."""
        if self.dist is None or self.world == 1:
            return list(vals)
        dev = "cuda" if (self.on_gpu and self.dist.get_backend(self.group) != "gloo") else "cpu"
        t = self.torch.tensor(list(vals), dtype=self.torch.int64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return t.cpu().tolist()

    # ---- the reference's learn() set-up, on the partitioned tables ----------------------------
    def learn_begin(self):
        self.batch.learn_begin()

    def apply_qinit(self):
        self.batch.apply_qinit()

    # ---- segment capacity ------------------------------------------------------------------------
    # A round's buffers are [world][k + 1] records: k message records (requests and update records)
    # per destination.  An env whose group does not fit is deferred whole by k_part_compact (it sends
    # nothing that round, sits out the next local step and sends the same records again), so results
    # never depend on k.  At a checkpoint the ranks agree (one MAX all-reduce) on k from the peak
    # per-destination demand since the previous checkpoint: every round in between is a fixed-size
    # all-to-all that needs no counts from the host.  One rank keeps the full capacity (its exchange
    # is the identity: nothing to save, nothing to defer).
    def set_caps(self, k_msg: int):
        k_msg = int(k_msg)
        if k_msg != self.k_msg:
            self.lib.check(self.lib.dll.sfl_part_set_caps(self.batch.h, k_msg), "sfl_part_set_caps")
            self.k_msg = k_msg

    @staticmethod
    def _resize(k: int, peak: int, cap: int) -> int:
        want = min(cap, max(16, -(-(peak + peak // 4 + 16) // 16) * 16))
        return want if (want > k or 2 * want < k) else k

    def _view(self, buf, k, rec):
        return buf[:self.world * (k + 1) * rec]

    def _a2a(self, recv, send, k, rec):
        """Fixed-size all-to-all of the [world][k + 1]-record segments (RCCL device to device; gloo with
        device buffers stages them through host memory)."""
        r, s_ = self._view(recv, k, rec), self._view(send, k, rec)
        if self.world == 1 and not self.exchange_collective:
            if r.data_ptr() != s_.data_ptr():
                r.copy_(s_)
            return
        if self.on_gpu and self.dist.get_backend(self.group) == "gloo":
            rc = self.torch.empty(r.numel(), dtype=self.torch.uint8)
            self.dist.all_to_all_single(rc, s_.cpu(), group=self.group)
            r.copy_(rc)
        else:
            self.dist.all_to_all_single(r, s_, group=self.group)

    def _read_counts(self):
        """This rank's counts since the previous checkpoint (sfl_part_counts: the checkpoint's host
        synchronisation), or None if its envs reported an error."""
        self.host_reads += 1
        if self.lib.dll.sfl_part_counts(self.batch.h, self._counts, len(self._counts)):
            return None
        return list(self._counts)

    def sync_count(self):
        """(device waits, count reads) of this rank's library handle so far (sfl_get_sync_count)."""
        w, r = C.c_uint64(), C.c_uint64()
        self.lib.check(self.lib.dll.sfl_get_sync_count(self.batch.h, C.byref(w), C.byref(r)), "sfl_get_sync_count")
        return w.value, r.value

    def step(self, decisions_per_env: int) -> int:
        """Advance every local env by ``decisions_per_env`` learning decisions (the sfl_step contract);
        returns the number of rounds.  Collective over the ranks."""
        with self.stream_context():
            for _ in self.rounds_of_step(decisions_per_env):
                pass
        return self.last_rounds

    def stream_context(self):
        """The context the job's work is issued in: its own stream on the GPU."""
        return contextlib.nullcontext() if self.stream is None else self.torch.cuda.stream(self.stream)

    def _checkpoint(self, r: int, last: int) -> bool:
        """Rounds after which the host reads the counts: 1, 2, 4, ..., 32, every 32nd, the round a step
        without deferrals ends at (decisions + 1), and every 8th after it (every round with
        checkpoint_every_round)."""
        return (self.checkpoint_every_round or (r & (r - 1) == 0 and r <= 32) or r % 32 == 0 or r == last
                or (r > last and (r - last) % 8 == 0))

    def rounds_of_step(self, decisions_per_env: int):
        """One step as a generator (issue it in ``stream_context()``): each iteration issues one round
        (local step, message all-to-all, owner step, reply all-to-all) without waiting for it and yields;
        a checkpoint round's counts are read at the next iteration, so that a caller alternating several
        jobs (CohortPipeline) issues the others' rounds before this one's host wait.  ``last_rounds``
        holds the step's rounds when the generator ends."""
        d = self.lib.dll
        h = self.batch.h
        W = self.world
        ptr = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        self.lib.check(d.sfl_part_begin(h), "sfl_part_begin")
        ms, rp = self.rec
        last = int(decisions_per_env) + 1
        limit = 4 * last + 64  # (deferrals add rounds; each checkpoint resizes the segments to the demand)
        rounds, failed, msg = 0, False, ""
        self.error_round = None

        def fail(what):
            # a failure on this rank (a launch error) must not leave the others waiting in the next
            # exchange: it sends empty segments until the checkpoint, where every rank stops
            nonlocal failed, msg
            failed, msg = True, what + ": " + d.sfl_last_error().decode(errors="replace")
        while True:
            rounds += 1
            if not failed and d.sfl_part_local(h, int(decisions_per_env), ptr(self.rep_recv), ptr(self.msg_send), None):
                fail("sfl_part_local")
            if failed and W > 1:
                self._view(self.msg_send, self.k_msg, ms).view(W, -1)[:, :ms].zero_()
            self._a2a(self.msg_recv, self.msg_send, self.k_msg, ms)
            if not failed and d.sfl_part_owner(h, ptr(self.msg_recv), ptr(self.rep_send)):
                fail("sfl_part_owner")
            if failed and W > 1:
                self._view(self.rep_send, self.k_msg, rp).zero_()
            self._a2a(self.rep_recv, self.rep_send, self.k_msg, rp)
            yield rounds
            if not self._checkpoint(rounds, last) and rounds < limit:
                continue
            self.checkpoints += 1
            c = None if failed else self._read_counts()
            if c is None and not msg:
                msg = "sfl_part_local: " + d.sfl_last_error().decode(errors="replace")
            err = 1 if c is None else 0
            c = c or [0] * len(self._counts)
            self.deferrals += c[2 * W + 2]
            job = self._all_max([err, c[2 * W], max(c[W:2 * W])])
            if job[0]:
                self.error_round = rounds
                raise _lib.SflError(f"rank {self.rank}: " + (msg or "stopped because another rank failed"))
            if job[1] == 0:
                break  # every env has made its decisions (this round's updates are applied)
            if rounds >= limit:
                raise _lib.SflError(f"rank {self.rank}: requests still open after {rounds} rounds "
                                    f"({c[2 * W]} envs on this rank)")
            if W > 1:
                self.set_caps(self._resize(self.k_msg, job[2], self.cap_msg))
        self.rounds += rounds
        self.last_rounds = rounds

    def sim_env(self, global_env: int):
        """(Batch, local index) of a job env this rank simulates, else None."""
        le = int(global_env) - self.env_base
        return (self.batch, le) if 0 <= le < self.E else None

    # ---- owned Q blocks (assembled over ranks by the caller) --------------------------------------
    def owned_q(self, global_env: int):
        """(q, touched) in the full per-env layout: this rank's owned blocks, NaN elsewhere."""
        q = np.full(self.cm.q_per_env, np.nan)
        t = np.zeros((self.cm.rows_per_env + 31) // 32, np.uint32)
        self.lib.check(self.lib.dll.sfl_part_get_q(self.batch.h, int(global_env), _ptr(q, C.c_double),
                                                   _ptr(t, C.c_uint32)), "sfl_part_get_q")
        return q, t

    def owned_mask(self) -> np.ndarray:
        """Boolean mask over the full per-env Q layout: entries of switches this rank owns."""
        cm = self.cm
        A = cm.arrays
        mk = np.zeros(cm.q_per_env, bool)
        for s in range(cm.S):
            if self.owner[s] != self.rank:
                continue
            P_ = len(cm.ports[s])
            for slot in range(P_):
                g = 4 * s + slot
                n = (1 << P_) * cm.K * 3 * int(A["q_w"][g])
                mk[int(A["q_off"][g]):int(A["q_off"][g]) + n] = True
        return mk


def cohort_sizes(E: int, cohorts: int) -> List[int]:
    """A rank's E envs split into ``cohorts`` consecutive cohorts as evenly as possible."""
    return [E // cohorts + (1 if c < E % cohorts else 0) for c in range(cohorts)]


class CohortPipeline:
    """The rank's envs as ``cohorts`` independent partitioned jobs whose rounds overlap.

    A round's phases depend on one another (local step -> message exchange -> owner step -> reply exchange
    -> next local step), so within one job the exchanges and the small compaction / owner kernels leave the
    GPU waiting, and the local step's last waves run with the chip mostly idle.  The envs are independent
    (an env's records touch only that env's rows), so splitting them into cohorts -- each a PartitionedBatch
    of its own, with its own message segments, owned-row table, stream and process group (its collectives
    never queue behind another cohort's) -- and issuing the cohorts' rounds alternately lets one cohort's
    exchange and owner step run beside another's local step.  Every env still performs the fused run's
    operations in order, so the results are those of one PartitionedBatch over the same envs (tests).

    Job env numbering: rank r's envs are [env_base, env_base + E) as for PartitionedBatch; the rank's
    cohort c holds its envs [off_c, off_c + E_c) (``cohort_sizes``), and cohort c's job numbers them after
    the lower ranks' cohort-c envs."""

    def __init__(self, cm: CompiledMap, hp: dict, seeds: Sequence[int], env_base: int, envs_total: int,
                 cohorts: int = 2, rank: int = 0, world: int = 1, dist=None, buffer_device: str = "cuda", **kw):
        import torch
        self.torch = torch
        E, C_ = len(seeds), int(cohorts)
        if C_ < 1:
            raise ValueError(f"CohortPipeline: {C_} cohorts")
        if kw.get("exchange_collective") and int(world) == 1 and C_ > 1:
            # (one rank has no per-cohort process groups: the cohorts' collectives would share one communicator
            # from several streams)
            raise ValueError("CohortPipeline: exchange_collective with one rank needs cohorts=1")
        self.cm, self.rank, self.world, self.dist = cm, int(rank), int(world), dist
        self.E, self.env_base, self.envs_total, self.cohorts = E, int(env_base), int(envs_total), C_
        # every rank's env count (its cohorts' sizes follow from it)
        if dist is None or self.world == 1:
            counts = [E]
        else:
            dev = "cuda" if (buffer_device == "cuda" and dist.get_backend() != "gloo") else "cpu"
            t = torch.zeros(self.world, dtype=torch.int64, device=dev)
            t[self.rank] = E
            dist.all_reduce(t)
            counts = [int(x) for x in t.cpu().tolist()]
        # (checked on the job's counts, after the all-reduce, so that every rank raises, not only the one short of
        # envs while its peers wait in the collective)
        if min(counts) < C_:
            raise ValueError(f"CohortPipeline: the ranks' env counts {counts} cannot each form {C_} cohorts")
        if sum(counts[:self.rank]) != self.env_base or sum(counts) != self.envs_total:
            raise ValueError(f"CohortPipeline: env_base={env_base} / envs_total={envs_total} do not match the "
                             f"ranks' env counts {counts}")
        self.rank_base = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        self.split = [cohort_sizes(n, C_) for n in counts]          # [rank][cohort] sizes
        # one process group per cohort (created in the same order on every rank), so a cohort's collectives
        # run on a communicator of their own
        groups = [None] * C_
        if dist is not None and self.world > 1 and C_ > 1:
            groups = [dist.new_group(list(range(self.world))) for _ in range(C_)]
        self._groups = [g for g in groups if g is not None]
        self.parts: List[PartitionedBatch] = []
        off = 0
        for c in range(C_):
            n = self.split[self.rank][c]
            base_c = sum(self.split[r][c] for r in range(self.rank))
            tot_c = sum(self.split[r][c] for r in range(self.world))
            self.parts.append(PartitionedBatch(cm, hp, list(seeds[off:off + n]), base_c, tot_c, rank=rank, world=world,
                                               dist=dist, buffer_device=buffer_device, group=groups[c], **kw))
            off += n
        p0 = self.parts[0]
        self.lib, self.owner, self.local_mask = p0.lib, p0.owner, p0.local_mask
        self.last_rounds = 0
        self.error_round = None

    def close(self):
        for p in self.parts:
            p.close()
        for g in self._groups:  # (collective: every rank closes its pipeline)
            self.dist.destroy_process_group(g)
        self._groups = []

    def learn_begin(self):
        for p in self.parts:
            p.learn_begin()

    def apply_qinit(self):
        for p in self.parts:
            p.apply_qinit()

    def step(self, decisions_per_env: int) -> int:
        """Advance every local env by ``decisions_per_env`` decisions: the cohorts' rounds issued
        alternately (each in its own stream); returns the most rounds any cohort took.  Collective."""
        live = [(p, p.rounds_of_step(decisions_per_env)) for p in self.parts]
        self.error_round = None
        try:
            while live:
                nxt = []
                for p, g in live:
                    with p.stream_context():
                        try:
                            next(g)
                            nxt.append((p, g))
                        except StopIteration:
                            pass
                live = nxt
        except _lib.SflError:
            self.error_round = max((p.error_round or 0) for p in self.parts) or None
            raise
        self.last_rounds = max(p.last_rounds for p in self.parts)
        return self.last_rounds

    # ---- counters summed over the cohorts ----------------------------------------------------------
    @property
    def rounds(self):
        return max(p.rounds for p in self.parts)

    @property
    def checkpoints(self):
        return sum(p.checkpoints for p in self.parts)

    @property
    def deferrals(self):
        return sum(p.deferrals for p in self.parts)

    @property
    def host_reads(self):
        return sum(p.host_reads for p in self.parts)

    @property
    def k_msg(self):
        return max(p.k_msg for p in self.parts)

    @property
    def cap_msg(self):
        return max(p.cap_msg for p in self.parts)

    def sync_count(self):
        w = r = 0
        for p in self.parts:
            a, b = p.sync_count()
            w, r = w + a, r + b
        return w, r

    # ---- job env -> (cohort, the cohort job's env) -------------------------------------------------
    def _locate(self, global_env: int):
        g = int(global_env)
        r = int(np.searchsorted(self.rank_base, g, side="right")) - 1
        if not (0 <= r < self.world) or g >= self.rank_base[r + 1]:
            raise ValueError(f"env {g} outside the job's {self.envs_total} envs")
        i = g - int(self.rank_base[r])
        for c, n in enumerate(self.split[r]):
            if i < n:
                return r, c, sum(self.split[q][c] for q in range(r)) + i
            i -= n
        raise AssertionError("unreachable")

    def owned_q(self, global_env: int):
        _, c, ge = self._locate(global_env)
        return self.parts[c].owned_q(ge)

    def owned_mask(self) -> np.ndarray:
        return self.parts[0].owned_mask()

    def sim_env(self, global_env: int):
        r, c, ge = self._locate(global_env)
        return self.parts[c].sim_env(ge) if r == self.rank else None
