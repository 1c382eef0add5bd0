"""Graph-partitioned SwitchFL learner (BASELINE.json configs[4], SURVEY.md §8(e) "C5").

The reference's learner is a network of switch agents: each switch keeps its own Q-table
(the dict partitioned by the switch coordinates, distr_q.py:47-57) and bootstraps from the
*successor* agent's row, ``max_q(next_state, next_agent)`` (distr_q.py:419-466).  Here the
switch agents are partitioned over the ranks (one process per GPU): rank r owns the Q rows of
its switches for every env of the job and answers the row lookups for them; envs are sharded
over the ranks as in the env-sharded mode.  Each round every env makes one decision:

    sfl_part_local    apply last round's reply, run to the next decision, emit its request
                      (and the update records of the post step)
    all-to-all        update + request buffers  (RCCL over xGMI: torch.distributed "nccl")
    sfl_part_update   owner applies the bootstrapped updates (stage-ordered)
    sfl_part_answer   owner: max over the row + masked argmax
    all-to-all        replies back

Every env performs exactly the operations of the fused kernels in the same order, so the
results are bit-identical to the single-process run (tests/test_partition.py).  Message
buffers are [world][cap + 1] record segments whose first record carries the count.  On the GPU
a round is queued on one stream (this batch's torch stream, handed to the library with
sfl_set_stream) and synchronises once, in sfl_part_local, for the record counts; with N > 1
ranks the counts (and each rank's highest update stage) go first, then each segment's filled
prefix point to point.
"""
from __future__ import annotations

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
                 delay_threshold: int = 20):
        import torch
        self.torch = torch
        kw = {} if ntab is None else dict(ntab=ntab)
        kw["malfunction_stream"] = malfunction_stream
        kw["delay_threshold"] = int(delay_threshold)  # StandardObserver(delay_threshold=...), observer.py:221
        self.batch = Batch(cm, hp, seeds, lib=lib, device=device, **kw)
        self.lib = self.batch.lib
        self.cm, self.rank, self.world, self.dist = cm, int(rank), int(world), dist
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
        rq, rp, up = C.c_uint32(), C.c_uint32(), C.c_uint32()
        self.lib.dll.sfl_part_record_sizes(C.byref(rq), C.byref(rp), C.byref(up))
        dev = torch.device(buffer_device)
        nreq = self.world * (self.cap_req + 1) * rq.value
        nrep = self.world * (self.cap_req + 1) * rp.value
        nupd = self.world * (self.cap_upd + 1) * up.value
        z = lambda n: torch.zeros(n, dtype=torch.uint8, device=dev)  # noqa: E731
        if self.world == 1:
            # one rank: every segment is addressed to this rank, so the exchange is the identity
            # and each receive buffer is its send buffer (no copies, no stream synchronisation)
            self.req_send = self.req_recv = z(nreq)
            self.rep_send = self.rep_recv = z(nrep)
            self.upd_send = self.upd_recv = z(nupd)
        else:
            self.req_send, self.req_recv = z(nreq), z(nreq)
            self.rep_send, self.rep_recv = z(nrep), z(nrep)
            self.upd_send, self.upd_recv = z(nupd), z(nupd)
        self.on_gpu = dev.type == "cuda"
        self.rec = (rq.value, rp.value, up.value)
        self.rounds = 0
        self._counts = (C.c_uint32 * (2 * self.world + 1))()
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
        dev = "cuda" if (buffer_device == "cuda" and self.dist.get_backend() != "gloo") else "cpu"
        t = torch.tensor([self.E, -self.E], dtype=torch.int64, device=dev)
        mx = t.clone()
        self.dist.all_reduce(mx, op=self.dist.ReduceOp.MAX)
        sm = torch.tensor([self.E], dtype=torch.int64, device=dev)
        self.dist.all_reduce(sm)
        return int(mx[0]), int(sm[0])

    def _any_rank(self, flag: int) -> int:
        """MAX of a per-rank flag over the job (every rank gets the same answer)."""
        if self.dist is None or self.world == 1:
            return flag
        dev = "cuda" if (self.on_gpu and self.dist.get_backend() != "gloo") else "cpu"
        t = self.torch.tensor([flag], dtype=self.torch.int64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return int(t[0])

    # ---- the reference's learn() set-up, on the partitioned tables ----------------------------
    def learn_begin(self):
        self.batch.learn_begin()

    def apply_qinit(self):
        self.batch.apply_qinit()

    # ---- one part step: every env makes `decisions_per_env` decisions ---------------------------
    def _exchange(self, recv, send):
        """One rank: every segment is addressed to this rank (the receive buffers are the send buffers)."""
        if recv is not send:
            recv.copy_(send)

    # ---- size-aware exchange (N > 1 ranks) ----------------------------------------------------------
    # Each destination segment's filled prefix (header record + its records) travels as one
    # point-to-point message into the same place of the receiver's segment: the owner kernels
    # read a segment only up to its header count, so nothing beyond the prefix is needed.  On
    # NCCL/RCCL the messages go device to device; gloo (the multi-rank rehearsal with GPU buffers on
    # one box, or host buffers) stages each prefix through host memory.
    def _sized(self) -> bool:
        return self.dist is not None and self.world > 1

    def _host_staged(self) -> bool:
        return self.on_gpu and self.dist.get_backend() == "gloo"

    def _p2p(self, recv, send, cap, rec, n_send, n_recv):
        torch, dist = self.torch, self.dist
        rs, ss = recv.view(self.world, (cap + 1) * rec), send.view(self.world, (cap + 1) * rec)
        ops, landing = [], []
        row = (cap + 1) * rec
        staged = self._host_staged()
        for p in range(self.world):
            k_s, k_r = (int(n_send[p]) + 1) * rec, (int(n_recv[p]) + 1) * rec
            if k_s > row or k_r > row:
                raise _lib.SflError(f"rank {self.rank}: segment to/from rank {p} exceeds its capacity ({cap} records)")
            if p == self.rank:
                rs[p, :k_r].copy_(ss[p, :k_s])
                continue
            if staged:
                r = torch.empty(k_r, dtype=torch.uint8)
                landing.append((rs[p, :k_r], r))
                ops.append(dist.P2POp(dist.isend, ss[p, :k_s].cpu(), p))
                ops.append(dist.P2POp(dist.irecv, r, p))
            else:
                ops.append(dist.P2POp(dist.isend, ss[p, :k_s], p))
                ops.append(dist.P2POp(dist.irecv, rs[p, :k_r], p))
        if ops:
            for r in dist.batch_isend_irecv(ops):
                r.wait()
        for dst, r in landing:
            dst.copy_(r)

    def _local_counts(self):
        """(requests, update records) per destination and the highest update stage of this rank's
        last sfl_part_local, or None if its envs reported an error (the round's synchronisation)."""
        w = self.world
        if self.lib.dll.sfl_part_counts(self.batch.h, self._counts, 2 * w + 1):
            return None
        c = list(self._counts)
        return c[:w], c[w:2 * w], c[2 * w]

    def _exchange_sized(self, err: int = 0):
        """Updates and requests: counts first (one small all-to-all, which also carries this rank's
        error flag and highest update stage to every rank), then the filled prefixes.  Returns the
        job-wide error flag; on an error nothing else is exchanged (every rank stops at the same point)."""
        torch = self.torch
        rq, _, up = self.rec
        counts = None if err else self._local_counts()
        if counts is None:
            err = 1
            n_req, n_upd, mst = [0] * self.world, [0] * self.world, 0
        else:
            n_req, n_upd, mst = counts
        # row d: what this rank sends to rank d (and, in every row, its total of requests: the job's
        # open requests end the step)
        dev = "cpu" if self.dist.get_backend() == "gloo" else self.req_send.device
        tot = sum(n_req)
        cs = torch.tensor([[n_req[d], n_upd[d], int(err), mst, tot] for d in range(self.world)], dtype=torch.int64,
                          device=dev)
        cr = torch.empty_like(cs)
        self.dist.all_to_all_single(cr, cs)                    # row s: what rank s sends to this rank
        cr = cr.cpu().tolist()
        if any(c[2] for c in cr):
            return 1
        self._job_open = sum(c[4] for c in cr)
        self._n_req_sent = list(n_req)
        self._n_req_recv = [c[0] for c in cr]
        self._p2p(self.upd_recv, self.upd_send, self.cap_upd, up, n_upd, [c[1] for c in cr])
        self._p2p(self.req_recv, self.req_send, self.cap_req, rq, self._n_req_sent, self._n_req_recv)
        return 0

    def _exchange_replies_sized(self):
        """A reply segment to rank s holds one reply per request received from s."""
        rp = self.rec[1]
        self._p2p(self.rep_recv, self.rep_send, self.cap_req, rp, self._n_req_recv, self._n_req_sent)

    def step(self, decisions_per_env: int) -> int:
        """Advance every local env by ``decisions_per_env`` learning decisions (the sfl_step contract);
        returns the number of rounds.  Collective over the ranks."""
        if self.stream is None:
            return self._step(decisions_per_env)
        with self.torch.cuda.stream(self.stream):
            return self._step(decisions_per_env)

    def _step(self, decisions_per_env: int) -> int:
        d = self.lib.dll
        h = self.batch.h
        ptr = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        self.lib.check(d.sfl_part_begin(h), "sfl_part_begin")
        sized = self._sized()
        # one rank on the GPU: the rounds queue on the stream without a synchronisation, and the counts
        # (open requests, the envs' errors) are read only after rounds 1, 2, 4, ..., 32 and then every
        # 32nd (with every row in place one round is the whole step; with messages the step runs its
        # decisions + 1 rounds, the last few possibly empty).  Otherwise (N > 1 ranks, or the host
        # build) each round's counts end the step as soon as no request is open anywhere
        deferred = self.stream is not None and not sized
        rounds = 0
        n_open = 0
        last = int(decisions_per_env) + 1
        for _ in range(last):
            n = C.c_uint64(0)
            # a failure on one rank (error flags of its envs, message overflow) must stop every rank,
            # or the others would wait forever in the next exchange: the flag travels with the counts
            rc = d.sfl_part_local(h, int(decisions_per_env), ptr(self.rep_recv), ptr(self.req_send),
                                  ptr(self.upd_send), None if (deferred or sized) else C.byref(n))
            msg = d.sfl_last_error().decode(errors="replace") if rc else ""
            if sized:
                failed = self._exchange_sized(err=1 if rc else 0)
                if failed and not msg:
                    msg = d.sfl_last_error().decode(errors="replace")
                n_open = self._job_open if not failed else 0
            else:
                failed = self._any_rank(1 if rc else 0)
                n_open = n.value
            if failed:
                raise _lib.SflError(f"rank {self.rank}: sfl_part_local: " +
                                    (msg or "stopped because another rank failed"))
            if not sized:
                self._exchange(self.upd_recv, self.upd_send)
                self._exchange(self.req_recv, self.req_send)
            self.lib.check(d.sfl_part_update(h, ptr(self.upd_recv)), "sfl_part_update")
            self.lib.check(d.sfl_part_answer(h, ptr(self.req_recv), ptr(self.rep_send)), "sfl_part_answer")
            if sized:
                self._exchange_replies_sized()
            else:
                self._exchange(self.rep_recv, self.rep_send)
            rounds += 1
            if deferred and (rounds & (rounds - 1) == 0 and rounds <= 32 or rounds % 32 == 0 or rounds == last):
                counts = self._local_counts()
                if counts is None:
                    raise _lib.SflError(f"rank {self.rank}: sfl_part_local: " +
                                        d.sfl_last_error().decode(errors="replace"))
                n_open = sum(counts[0])
                if n_open == 0:
                    break
            elif not deferred and n_open == 0:
                break  # every env has made its decisions (this round's updates are applied)
        if (not sized) and self._any_rank(1 if n_open != 0 else 0) or sized and n_open != 0:
            raise _lib.SflError(f"rank {self.rank}: requests still open after the last round "
                                f"({n_open} on this rank)")
        self.rounds += rounds
        return rounds

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
