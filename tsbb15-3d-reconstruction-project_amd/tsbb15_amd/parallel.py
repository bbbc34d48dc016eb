"""Multi-GPU layer: one process per GPU, RCCL over xGMI.

Two shardings:

  * pairs (config C4): independent image pairs are assigned to ranks by longest-processing-
    time greedy on N x H; each rank runs its pairs with no collective -- RANSAC per pair, then
    (optionally) one batched launch of the gold-standard refinement and of E / relative pose
    over all of its pairs -- and one all-gather of fixed-size per-pair records (F_RANSAC,
    count, index, F_gold, R, t, pair id) at the end.
  * hypotheses of one pair (C2/C5 weak scaling): rank r evaluates the contiguous hypothesis
    range [start_r, start_r + n_r) (Philox counters are global hypothesis indices, so the
    union is exactly the single-GPU run); then one max-all-reduce of c* and one all-gather of
    the candidates with count == c*, which every rank replays in global index order with the
    fun.py:320-328 rule (first c* hypothesis, then std/norm tie replacements).
  * the same in parity mode (the reference's own stream, fun.py:305-306), two ways:
    ``ransac_f_split_np`` splits the stream parse itself -- each rank parses only its share
    of the chunks, the small chunk maps are all-gathered and composed on every rank, and each
    rank evaluates the hypotheses that start in its share (np_sharded_segments);
    ``ransac_f_sharded_np`` (the earlier form) has every rank parse the whole stream and
    evaluate a slice.  Either way the winner, S_RANSAC and the MT state equal the
    single-process run.

Communicators: :class:`RcclComm` (librsamd, device buffers, xGMI) on GPUs,
:class:`TorchComm` (torch.distributed, e.g. gloo on the CPU) and :class:`ThreadComm` (ranks as
threads) for tests; all expose ``allgather_bytes`` and ``allreduce_max_int``.  RcclComm needs
only a one-off broadcast of its unique id: :class:`TcpHub` (a socket hub, no torch; bench.py's
harness), :class:`FileBoot` (a shared directory) or a TorchComm.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _ffi

CAND_DTYPE = np.dtype([("index", "<i8"), ("count", "<i8"), ("std", "<f8"), ("norm", "<f8"),
                       ("F", "<f8", (9,))])
PAIR_DTYPE = np.dtype([("pair", "<i8"), ("valid", "<i8"), ("best_index", "<i8"),
                       ("count", "<i8"), ("std", "<f8"), ("F", "<f8", (9,)),
                       ("refined", "<i8"), ("F_gold", "<f8", (9,)), ("gs_cost", "<f8"),
                       ("pose", "<i8"), ("R", "<f8", (9,)), ("t", "<f8", (3,))])


# ------------------------------------------------------------------------------------------
# communicators
# ------------------------------------------------------------------------------------------
class TorchComm:
    """torch.distributed process group (gloo on the host, for tests and bootstrap)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def allgather_bytes(self, b: bytes):
        out = [None] * self.world
        self.dist.all_gather_object(out, b, group=self.group)
        return out

    def allreduce_max_int(self, v: int) -> int:
        import torch
        t = torch.tensor([int(v)], dtype=torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def broadcast_bytes(self, b, src=0):
        obj = [b]
        self.dist.broadcast_object_list(obj, src=src, group=self.group)
        return obj[0]


class FileBoot:
    """Bootstrap without torch.distributed: rank 0 publishes a byte string (the RCCL unique
    id) as a file in a directory every rank can see (written to a temporary name, then
    renamed, so readers never see a partial file); the others poll for it.  Pass it as
    ``RcclComm(ctx, rank, world, boot=FileBoot(path, rank))``."""

    def __init__(self, directory, rank, timeout=60.0, name="rsamd_comm_id"):
        import os
        self.path = os.path.join(directory, name)
        self.rank, self.timeout = int(rank), float(timeout)

    def broadcast_bytes(self, b, src=0):
        import os
        import time
        if self.rank == src:
            tmp = f"{self.path}.{os.getpid()}.tmp"
            with open(tmp, "wb") as f:
                f.write(bytes(b))
            os.replace(tmp, self.path)
            return bytes(b)
        t0 = time.monotonic()
        while not os.path.exists(self.path):
            if time.monotonic() - t0 > self.timeout:
                raise TimeoutError(f"no communicator id at {self.path} after {self.timeout} s")
            time.sleep(0.01)
        with open(self.path, "rb") as f:
            return f.read()


class TcpHub:
    """Host-side collectives for a one-node job without torch.distributed: rank 0 is a hub on
    ``addr:port`` that every other rank connects to; each operation is a gather to the hub
    and a broadcast back of length-prefixed frames.  It carries the RCCL unique id (as a
    ``boot``), the harness barrier and max-reduce -- a few bytes per call, never data.

    ``TcpHub.from_env()`` reads RANK / WORLD_SIZE / MASTER_ADDR and listens on
    MASTER_PORT + 1 (torch.distributed.run's own store holds MASTER_PORT)."""

    def __init__(self, rank, world, addr="127.0.0.1", port=29611, timeout=120.0):
        import socket
        import time
        self.rank, self.world = int(rank), int(world)
        self.peers = {}
        self.sock = None
        if self.world == 1:
            return
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, int(port)))
            srv.listen(self.world)
            srv.settimeout(timeout)
            try:
                while len(self.peers) < self.world - 1:
                    c, _ = srv.accept()
                    c.settimeout(timeout)
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    r = int.from_bytes(self._recvn(c, 4), "little")
                    if not 0 < r < self.world or r in self.peers:
                        raise RuntimeError(f"TcpHub: unexpected rank {r}")
                    self.peers[r] = c
            finally:
                srv.close()
        else:
            t0 = time.monotonic()
            while True:
                try:
                    c = socket.create_connection((addr, int(port)), timeout=timeout)
                    break
                except OSError:
                    if time.monotonic() - t0 > timeout:
                        raise
                    time.sleep(0.05)
            c.settimeout(timeout)
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            c.sendall(self.rank.to_bytes(4, "little"))
            self.sock = c

    @classmethod
    def from_env(cls, timeout=120.0):
        import os
        return cls(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                   os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   int(os.environ.get("MASTER_PORT", "29610")) + 1, timeout)

    @staticmethod
    def _recvn(c, n):
        buf = bytearray()
        while len(buf) < n:
            part = c.recv(n - len(buf))
            if not part:
                raise ConnectionError("TcpHub: peer closed the connection")
            buf += part
        return bytes(buf)

    @classmethod
    def _send(cls, c, b):
        c.sendall(len(b).to_bytes(8, "little") + b)

    @classmethod
    def _recv(cls, c):
        return cls._recvn(c, int.from_bytes(cls._recvn(c, 8), "little"))

    def allgather_bytes(self, b):
        b = bytes(b)
        if self.world == 1:
            return [b]
        if self.rank == 0:
            parts = [b] + [self._recv(self.peers[r]) for r in range(1, self.world)]
            frame = b"".join(len(p).to_bytes(8, "little") + p for p in parts)
            for r in range(1, self.world):
                self._send(self.peers[r], frame)
            return parts
        self._send(self.sock, b)
        frame, parts, o = self._recv(self.sock), [], 0
        while o < len(frame):
            n = int.from_bytes(frame[o:o + 8], "little")
            parts.append(frame[o + 8:o + 8 + n])
            o += 8 + n
        return parts

    def allreduce_max_int(self, v):
        return max(int.from_bytes(x, "little", signed=True)
                   for x in self.allgather_bytes(int(v).to_bytes(8, "little", signed=True)))

    def max_float(self, x):
        return max(float(np.frombuffer(p, np.float64)[0])
                   for p in self.allgather_bytes(np.float64(x).tobytes()))

    def broadcast_bytes(self, b, src=0):
        return self.allgather_bytes(b if self.rank == src else b"")[src]

    def barrier(self):
        self.allgather_bytes(b"")

    def close(self):
        for c in list(self.peers.values()) + ([self.sock] if self.sock else []):
            try:
                c.close()
            except OSError:
                pass
        self.peers, self.sock = {}, None


class RcclComm:
    """RCCL communicator owned by a librsamd context (bootstrapped through ``boot``, any
    object with ``broadcast_bytes``; a TorchComm over gloo works)."""

    def __init__(self, ctx, rank, world, boot):
        self.ctx, self.rank, self.world = ctx, int(rank), int(world)
        uid = np.zeros(_ffi.COMM_ID_BYTES, np.uint8)
        if self.rank == 0:
            _ffi.check(_ffi.lib().rs_comm_unique_id(_ffi.ptr(uid, C.c_uint8)))
        uid = np.frombuffer(boot.broadcast_bytes(uid.tobytes(), 0), np.uint8).copy()
        _ffi.check(_ffi.lib().rs_comm_init(ctx.handle, self.world, self.rank,
                                           _ffi.ptr(uid, C.c_uint8)))

    def allgather_bytes(self, b: bytes):
        n = len(b)
        send = np.frombuffer(b, np.uint8).copy()
        recv = np.zeros(n * self.world, np.uint8)
        _ffi.check(_ffi.lib().rs_comm_allgather(self.ctx.handle,
                                                send.ctypes.data_as(C.c_void_p),
                                                recv.ctypes.data_as(C.c_void_p), n))
        return [recv[i * n:(i + 1) * n].tobytes() for i in range(self.world)]

    def allreduce_max_int(self, v: int) -> int:
        x = C.c_int64(int(v))
        _ffi.check(_ffi.lib().rs_comm_allreduce_max_i64(self.ctx.handle, C.byref(x)))
        return int(x.value)

    def close(self):
        _ffi.lib().rs_comm_destroy(self.ctx.handle)


# ------------------------------------------------------------------------------------------
# sharding and merging (host logic shared by every communicator)
# ------------------------------------------------------------------------------------------
def shard_range(H, world, rank):
    """Contiguous hypothesis range of ``rank``: sizes differ by at most one."""
    base, extra = divmod(int(H), int(world))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def lpt_assign(costs, world):
    """Longest-processing-time greedy: list of item indices per rank (deterministic: ties in
    cost go to the lower index, ties in load to the lower rank)."""
    import heapq
    costs = np.asarray(costs, dtype=np.float64)
    if world == 1:
        return [list(range(len(costs)))]
    order = np.lexsort((np.arange(len(costs)), -costs))
    heap = [(0.0, q) for q in range(world)]
    out = [[] for _ in range(world)]
    for i in order.tolist():
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + float(costs[i]), r))
    return [sorted(v) for v in out]


def replay_rule(cands):
    """fun.py:320-328 over candidate records sorted by global hypothesis index.

    ``cands`` must hold every hypothesis whose count equals the global maximum.  Returns the
    winning record (or None when no hypothesis has a non-empty consensus)."""
    if len(cands) == 0:
        return None
    cands = np.sort(cands, order="index")
    best = None
    for c in cands:
        if best is None:
            if c["count"] > 0:
                best = c
        elif c["count"] > best["count"]:
            best = c
        elif c["count"] == best["count"] and abs(best["std"]) > c["norm"]:
            best = c
    return best


def merge_shard_candidates(comm, local):
    """All-reduce c*, all-gather the local candidates with count == c*, replay globally."""
    local = np.asarray(local, dtype=CAND_DTYPE)
    lmax = int(local["count"].max()) if len(local) else 0
    cstar = comm.allreduce_max_int(lmax)
    mine = local[local["count"] == cstar] if cstar > 0 else local[:0]
    width = comm.allreduce_max_int(len(mine))
    buf = np.zeros(width + 1, dtype=CAND_DTYPE)
    buf[0]["index"] = len(mine)          # header record: number of valid entries
    buf[1:1 + len(mine)] = mine
    parts = comm.allgather_bytes(buf.tobytes())
    allc = []
    for p in parts:
        a = np.frombuffer(p, dtype=CAND_DTYPE)
        allc.append(a[1:1 + int(a[0]["index"])])
    return replay_rule(np.concatenate(allc) if allc else np.zeros(0, CAND_DTYPE))


def candidates_from_plan(plan, hyp_offset):
    recs = plan.candidates()
    out = np.zeros(len(recs), dtype=CAND_DTYPE)
    for i, c in enumerate(recs):
        out[i] = (c.index + hyp_offset, c.count, c.std_d, c.norm_d, np.array(c.F[:]))
    return out


def ransac_f_sharded(comm, ctx, p1, p2, H, seed=0, thresh=1.5, plan=None):
    """Hypotheses [0, H) of one pair split over the ranks of ``comm`` (Philox sampler).

    Returns (winner record, inliers) -- identical on every rank and identical to the
    single-GPU run with the same seed."""
    p1 = _ffi.f64c(p1)
    p2 = _ffi.f64c(p2)
    start, cnt = shard_range(H, comm.world, comm.rank)
    own = plan is None
    if own:
        plan = _ffi.F8Plan(ctx, p1.shape[1], max(cnt, 1))
        plan.set_points(p1, p2)
    local = np.zeros(0, CAND_DTYPE)
    if cnt > 0:
        plan.run(cnt, mode=_ffi.SAMPLER_PHILOX, seed=seed, hyp_offset=start, thresh=thresh)
        plan.result()
        local = candidates_from_plan(plan, start)
    best = merge_shard_candidates(comm, local)
    if own:
        plan.close()
    if best is None:
        return None, np.zeros(0, np.int64)
    from . import lab3
    F = best["F"].reshape(3, 3)
    r = np.abs(lab3.fmatrix_residuals(F, p1, p2))
    d = np.where(np.isnan(r).any(axis=0), np.nan, r.max(axis=0))
    return best, np.flatnonzero(d < thresh)


def np_state(rng=None):
    """(key, pos) of the numpy legacy MT19937 stream (the global np.random when rng is None)."""
    st = (np.random if rng is None else rng).get_state()
    if st[0] != "MT19937":
        raise ValueError("only the legacy MT19937 RandomState stream is supported")
    return np.asarray(st[1], np.uint32), int(st[2])


def ransac_f_sharded_np(comm, p1, p2, H, key, pos, evaluate, thresh=1.5):
    """Parity-mode hypothesis sharding of the fun.py:303-328 loop.

    ``evaluate(start, count, key, pos)`` evaluates hypotheses [start, start + count) of the H
    drawn from the numpy stream (key, pos) and returns (candidate records with GLOBAL indices,
    key', pos') where (key', pos') is the state after all H (:class:`GpuSliceEvaluator` on a
    GPU).  Returns (winner record or None, key', pos'), identical on every rank."""
    start, cnt = shard_range(H, comm.world, comm.rank)
    local, key2, pos2 = evaluate(start, cnt, key, pos)
    best = merge_shard_candidates(comm, local)
    return best, key2, pos2


class GpuSliceEvaluator:
    """This rank's slice of a parity-mode run on its GPU (rs_f8_plan_run_np_slice): the stream
    of all H hypotheses is parsed on the GPU, only the slice is solved, counted and selected."""

    def __init__(self, ctx, p1, p2, H, thresh=1.5, max_slice=None):
        self.p1, self.p2 = _ffi.f64c(p1), _ffi.f64c(p2)
        self.H, self.thresh = int(H), float(thresh)
        self.plan = _ffi.F8Plan(ctx, self.p1.shape[1], max(1, int(max_slice or self.H)))
        self.plan.set_points(self.p1, self.p2)

    def __call__(self, start, count, key, pos):
        if count < 1:  # more ranks than hypotheses: only the state advance
            _, key2, pos2 = _ffi.np_choice_tuples(key, pos, self.p1.shape[1], 8, self.H)
            return np.zeros(0, CAND_DTYPE), key2, pos2
        key2, pos2 = self.plan.run_np_slice(self.H, start, count, key, pos, self.thresh)
        self.plan.result()
        return candidates_from_plan(self.plan, start), key2, pos2

    def inliers(self, best):
        if best is None:
            return np.zeros(0, np.int64)
        from . import lab3
        F = best["F"].reshape(3, 3)
        r = np.abs(lab3.fmatrix_residuals(F, self.p1, self.p2))
        d = np.where(np.isnan(r).any(axis=0), np.nan, r.max(axis=0))
        return np.flatnonzero(d < self.thresh)

    def close(self):
        self.plan.close()


# ------------------------------------------------------------------------------------------
# parity mode with the stream parse itself split across ranks (rs_np_shard_*)
# ------------------------------------------------------------------------------------------
def shard_schedule(stats, count, rank):
    """Host logic of the sharded parse, identical on every rank.

    ``stats`` = [(own start count, first start)] of every rank in rank order (rank 0's first
    start is the segment's draw 0).  Start i (global, in stream order) begins hypothesis i; a
    hypothesis is complete when the next start exists, so the segment delivers
    got = min(count, starts - 1).  Returns (got, base, hi, next_start, final_rank): this rank's
    hypotheses are [base, hi), the first start of the next rank holding any (-1: none) ends
    its last one, and final_rank holds start ``got`` (the state after the segment)."""
    ns = [int(s[0]) for s in stats]
    total = sum(ns)
    got = min(int(count), total - 1)
    if got < 1:
        raise RuntimeError("parity stream: the segment holds no complete hypothesis")
    bases = np.concatenate([[0], np.cumsum(ns)[:-1]]).astype(np.int64)
    base = int(bases[rank])
    hi = max(base, min(base + ns[rank], got))
    nxt = -1
    for q in range(rank + 1, len(ns)):
        if ns[q] > 0:
            nxt = int(stats[q][1])
            break
    final_rank = next(q for q in range(len(ns)) if bases[q] <= got < bases[q] + ns[q])
    return got, base, hi, nxt, final_rank


def np_sharded_segments(comm, shard, key, pos, H, consume):
    """The exchange of a sharded parity-stream parse (fun.py:305-306 / ransac.py:12-19 over
    all ranks).  Per segment: every rank parses its own chunks
    (``shard.parse``), the chunk maps are all-gathered and composed on every rank
    (``shard.compose``), the (start count, first start) pairs are all-gathered, and
    ``consume(offset, base, hi, next_start, final_idx, key)`` handles this rank's hypotheses
    [offset + base, offset + hi) of the H (``shard.tuples`` or ``F8Plan.run_np_shard``) and
    returns the (key, pos) after the segment on the rank with final_idx >= 0; that state is
    all-gathered and starts the next segment.  Returns the (key, pos) after all H hypotheses,
    identical on every rank (and to the single-stream replay)."""
    key = np.array(key, dtype=np.uint32, copy=True)
    pos = int(pos)
    done = 0
    while done < H:
        shard.parse(key, pos, H - done)
        blob = shard.maps()
        width = comm.allreduce_max_int(len(blob))
        blobs = comm.allgather_bytes(blob + bytes(width - len(blob)))
        ns, first = shard.compose(blobs)
        stats = [np.frombuffer(b, np.int64) for b in
                 comm.allgather_bytes(np.array([ns, first], np.int64).tobytes())]
        got, base, hi, nxt, final_rank = shard_schedule(stats, H - done, comm.rank)
        fin = consume(done, base, hi, nxt, got if final_rank == comm.rank else -1, key)
        rec = np.zeros(_MT_REC, np.uint32)
        if final_rank == comm.rank:
            rec[:624] = fin[0]
            rec[624] = int(fin[1])
        rec = np.frombuffer(comm.allgather_bytes(rec.tobytes())[final_rank], np.uint32)
        key, pos = rec[:624].copy(), int(rec[624])
        done += got
    return key, pos


_MT_REC = 625


def np_sharded_tuples(comm, shard, key, pos, H):
    """This rank's share of the next H tuples of the stream: (list of (global start index,
    (count, k) int32 rows)), key', pos')."""
    parts = []

    def consume(off, base, hi, nxt, fidx, key):
        rows, fin = shard.tuples(base, hi, nxt, fidx, key)
        if hi > base:
            parts.append((off + base, rows))
        return fin

    key2, pos2 = np_sharded_segments(comm, shard, key, pos, H, consume)
    return parts, key2, pos2


def ransac_f_split_np(comm, ctx, p1, p2, H, key, pos, thresh=1.5, plan=None, shard=None):
    """Parity-mode fun.py:303-328 loop with the stream parse itself split across the ranks:
    each rank parses and evaluates only the hypotheses that start in its share of the stream,
    then the c* all-reduce / candidate all-gather / global-order replay decides.  Returns
    (winner record or None, key', pos'), identical on every rank and equal to the
    single-GPU run (winner, S_RANSAC via :func:`inliers_of`, MT state)."""
    p1, p2 = _ffi.f64c(p1), _ffi.f64c(p2)
    own_plan, own_shard = plan is None, shard is None
    if own_plan:
        plan = _ffi.F8Plan(ctx, p1.shape[1], max(1, int(H)))
        plan.set_points(p1, p2)
    if own_shard:
        shard = _ffi.NpShard(ctx, p1.shape[1], 8, comm.world, comm.rank)
    cands = []

    def consume(off, base, hi, nxt, fidx, key):
        fin = plan.run_np_shard(shard, base, hi, nxt, fidx, key, thresh)
        if hi > base:
            cands.append(candidates_from_plan(plan, off + base))
        return fin

    try:
        key2, pos2 = np_sharded_segments(comm, shard, key, pos, H, consume)
    finally:
        if own_shard:
            shard.close()
    local = np.concatenate(cands) if cands else np.zeros(0, CAND_DTYPE)
    best = merge_shard_candidates(comm, local)
    if own_plan:
        plan.close()
    return best, key2, pos2


def project_split_np(ctx, p1, p2, H, key, pos, world, thresh=1.5, plans=None, shards=None):
    """One-GPU PROJECTION of :func:`ransac_f_split_np` at ``world`` ranks: every rank's steps
    run one after another on this GPU (nothing else on the device while a step runs), each
    timed alone, with the exchanges done in host memory.  Per rank: ``parse`` (its chunks'
    jump / stream / entry / track), ``maps`` (its blob to the host), ``compose`` (all blobs ->
    its start count), ``evaluate`` (its hypotheses' tuples + solve / count / select, result
    header).  A rank's projected time is the sum of its steps; the job's is the slowest rank's
    plus the collectives (not timed here: per segment two all-gathers of a few KB and two of
    8 B / 2.5 KB, and the final c* all-reduce + candidate all-gather).

    ``plans`` / ``shards`` (one per rank) may be passed in so that a second call times warm
    buffers.  Returns (report dict, winner record, key', pos'); the winner and state equal
    the serial run's (the caller checks), so the projection times the exact computation."""
    import time
    p1, p2 = _ffi.f64c(p1), _ffi.f64c(p2)
    W = int(world)
    own_sh, own = shards is None, plans is None
    if own_sh:
        shards = [_ffi.NpShard(ctx, p1.shape[1], 8, W, r) for r in range(W)]
    if own:
        plans = []
    try:
        if own:
            for _ in range(W):
                pl = _ffi.F8Plan(ctx, p1.shape[1], max(1, int(H)))
                pl.set_points(p1, p2)
                plans.append(pl)
        steps = {s: [0.0] * W for s in ("parse", "maps", "compose", "evaluate")}
        blob_bytes = [0] * W
        cands = [[] for _ in range(W)]
        key = np.array(key, dtype=np.uint32, copy=True)
        pos, done, segments = int(pos), 0, 0

        def timed(step, r, f):
            ctx.synchronize()
            t = time.perf_counter()
            out = f()
            ctx.synchronize()
            steps[step][r] += time.perf_counter() - t
            return out

        while done < H:
            segments += 1
            blobs = []
            for r in range(W):
                timed("parse", r, lambda: shards[r].parse(key, pos, H - done))
                blobs.append(timed("maps", r, shards[r].maps))
                blob_bytes[r] = max(blob_bytes[r], len(blobs[-1]))
            width = max(len(b) for b in blobs)
            blobs = [b + bytes(width - len(b)) for b in blobs]
            stats = [timed("compose", r, lambda: shards[r].compose(blobs)) for r in range(W)]
            fin = None
            for r in range(W):
                got, base, hi, nxt, final_rank = shard_schedule(stats, H - done, r)
                fidx = got if final_rank == r else -1

                def ev():
                    f = plans[r].run_np_shard(shards[r], base, hi, nxt, fidx, key, thresh)
                    if hi > base:
                        plans[r].result()
                    return f
                f = timed("evaluate", r, ev)
                if hi > base:
                    cands[r].append(candidates_from_plan(plans[r], done + base))
                if fidx >= 0:
                    fin = f
            key, pos = fin[0].copy(), int(fin[1])
            done += got
        local = [np.concatenate(c) if c else np.zeros(0, CAND_DTYPE) for c in cands]
        allc = np.concatenate(local)
        cstar = int(allc["count"].max()) if len(allc) else 0
        best = replay_rule(allc[allc["count"] == cstar] if cstar > 0 else allc[:0])
    finally:
        if own_sh:
            for s in shards:
                s.close()
        if own:
            for pl in plans:
                pl.close()
    per_rank = [sum(steps[s][r] for s in steps) * 1e3 for r in range(W)]
    rep = {"world": W, "segments": segments,
           "per_rank_ms": {s: [v * 1e3 for v in steps[s]] for s in steps},
           "rank_total_ms": per_rank, "projected_ms": max(per_rank),
           "slowest_rank": int(np.argmax(per_rank)), "blob_bytes": blob_bytes}
    return rep, best, key, pos


def inliers_of(best, p1, p2, thresh=1.5):
    """S_RANSAC of a merged winner record (fun.py:316-317, reference-order residuals)."""
    if best is None:
        return np.zeros(0, np.int64)
    from . import lab3
    r = np.abs(lab3.fmatrix_residuals(best["F"].reshape(3, 3), _ffi.f64c(p1), _ffi.f64c(p2)))
    d = np.where(np.isnan(r).any(axis=0), np.nan, r.max(axis=0))
    return np.flatnonzero(d < thresh)


class ThreadComm:
    """Ranks as threads of one process (a multi-rank rehearsal on one GPU, tests): all-gather
    through a shared board and a barrier.  ``ThreadComm.group(world)`` gives one per rank."""

    class _Board:
        def __init__(self, world):
            import threading
            self.world = world
            self.slots = [None] * world
            self.barrier = threading.Barrier(world)

    def __init__(self, board, rank):
        self.board, self.rank, self.world = board, int(rank), board.world

    @classmethod
    def group(cls, world):
        board = cls._Board(int(world))
        return [cls(board, r) for r in range(int(world))]

    def allgather_bytes(self, b):
        bd = self.board
        bd.slots[self.rank] = bytes(b)
        bd.barrier.wait()
        out = list(bd.slots)
        bd.barrier.wait()
        return out

    def allreduce_max_int(self, v):
        return max(int.from_bytes(x, "little", signed=True)
                   for x in self.allgather_bytes(int(v).to_bytes(8, "little", signed=True)))


def run_ranks(world, fn):
    """fn(rank, comm) on ``world`` threads with ThreadComm; returns the per-rank results
    (the first exception of any rank is re-raised)."""
    import threading
    comms = ThreadComm.group(world)
    out, errs = [None] * world, [None] * world

    def body(r):
        try:
            out[r] = fn(r, comms[r])
        except BaseException as e:  # noqa: BLE001
            errs[r] = e
            comms[r].board.barrier.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in errs:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    for e in errs:
        if e is not None:
            raise e
    return out


class GpuPairSolver:
    """Runs one pair's RANSAC on this rank's GPU (plans cached per correspondence count)."""

    def __init__(self, ctx, H, seed_base=1000, thresh=1.5):
        self.ctx, self.H, self.seed_base, self.thresh = ctx, int(H), seed_base, thresh
        self.plans = {}

    def __call__(self, i, p1, p2):
        n = p1.shape[1]
        plan = self.plans.get(n)
        if plan is None:
            plan = self.plans[n] = _ffi.F8Plan(self.ctx, n, self.H)
        plan.set_points(p1, p2)
        plan.run(self.H, mode=_ffi.SAMPLER_PHILOX, seed=self.seed_base + i, thresh=self.thresh)
        r, inl = plan.result()
        return (1 if r.best_index >= 0 else 0, r.best_index, r.best_count, r.best_std,
                np.array(r.F[:]), inl)

    def close(self):
        for p in self.plans.values():
            p.close()
        self.plans = {}


class GpuPairBatchSolver:
    """All of this rank's pairs in one batched pass (rs_pairs_f8_ransac): same Philox stream
    per pair as GpuPairSolver (seed_base + pair index), so the results are identical; the
    solve / count / select stages each run as one launch over every pair."""

    def __init__(self, ctx, H, seed_base=1000, thresh=1.5):
        self.ctx, self.H, self.seed_base, self.thresh = ctx, int(H), seed_base, thresh

    def many_arrays(self, ids, p1, p2, off):
        """The same on pre-concatenated points: (PAIR_RESULT_DTYPE array, inlier buffer)."""
        from . import pairs as pairs_mod
        return pairs_mod.ransac_pairs_raw(p1, p2, off, self.H, self.seed_base, self.thresh,
                                          ids=ids, ctx=self.ctx)

    def many_two_view(self, ids, p1, p2, off, K):
        """many_arrays and a GpuPairRefiner's stages in one device call (rs_pairs_two_view):
        (results, inliers, F_gold (B,9), gs info, R (B,9), t (B,3), found (B,))."""
        from . import pairs as pairs_mod
        return pairs_mod.two_view_pairs_raw(p1, p2, off, self.H, K, self.seed_base, self.thresh,
                                            ids=ids, ctx=self.ctx)

    def many(self, ids, pairs):
        from . import pairs as pairs_mod
        if not ids:
            return []
        rr = pairs_mod.ransac_pairs(pairs, self.H, self.seed_base, self.thresh, ids=ids,
                                    ctx=self.ctx)
        return [(1 if r.best_index >= 0 else 0, r.best_index, r.count, r.std, r.F.ravel(),
                 r.inliers) for r in rr]


class GpuPairRefiner:
    """After RANSAC, for all of this rank's pairs in one launch each: the gold standard
    (fun.py:336-369) on the inliers, then -- given the calibration K -- E = K^T F_gold K and
    the relative pose from the pair's first correspondence (fun.py:91-102, 209-258, as
    main.py:50-63 does for the initial pair)."""

    def __init__(self, ctx, K=None, fused=True):
        self.ctx = ctx
        self.K = None if K is None else np.ascontiguousarray(K, dtype=np.float64)
        # run_pairs with a GpuPairBatchSolver on the same context: RANSAC and these stages in
        # one device call (the inlier points never leave the GPU); False: separate calls
        self.fused = fused

    def arrays(self, F, pl, pr, off, first1, first2):
        """The same on arrays: F (B,9) F_RANSAC, the inlier points concatenated (pl, pr
        (2, total), off (B + 1)), each pair's first correspondence first1, first2 (B,2).
        Returns (F_gold (B,9), gs_cost (B,), pose found (B,), R (B,9), t (B,3))."""
        from . import twoview
        B = len(off) - 1
        Fg, _, _, info = twoview.gold_standard_arrays(np.asarray(F).reshape(B, 3, 3), pl, pr, off,
                                                      ctx=self.ctx, want_points=False)
        if self.K is None:
            return (Fg.reshape(B, 9), info["cost"], np.zeros(B, dtype=np.int64),
                    np.full((B, 9), np.nan), np.full((B, 3), np.nan))
        E = twoview.essential_batch(self.K, Fg, ctx=self.ctx)
        y1 = twoview.normalise_each(self.K, first1)[:, :2]
        y2 = twoview.normalise_each(self.K, first2)[:, :2]
        R, t, found = twoview.relative_camera_pose_batch(E, y1, y2, ctx=self.ctx)
        return Fg.reshape(B, 9), info["cost"], found, R.reshape(B, 9), t

    def __call__(self, items):
        from . import twoview
        if not items:
            return []
        Fs = np.stack([np.asarray(it[1]).reshape(3, 3) for it in items])
        gs = twoview.gold_standard_batch(Fs, [it[2] for it in items], [it[3] for it in items],
                                         ctx=self.ctx)
        Fg = np.stack([g.F for g in gs])
        nan9, nan3 = np.full(9, np.nan), np.full(3, np.nan)
        if self.K is None:
            return [(g.F.ravel(), g.cost, 0, nan9, nan3) for g in gs]
        E = twoview.essential_batch(self.K, Fg, ctx=self.ctx)
        y1 = twoview.normalise_each(self.K, np.stack([it[4] for it in items]))[:, :2]
        y2 = twoview.normalise_each(self.K, np.stack([it[5] for it in items]))[:, :2]
        R, t, found = twoview.relative_camera_pose_batch(E, y1, y2, ctx=self.ctx)
        return [(g.F.ravel(), g.cost, int(f), R[k].ravel(), t[k])
                for k, (g, f) in enumerate(zip(gs, found))]


def run_pairs(comm, pairs, H, solve, refine=None):
    """Config C4: ``pairs`` = list of (p1, p2); ``solve(i, p1, p2)`` -> (valid, best_index,
    count, std, F[9][, inliers]) runs one pair on this rank (GpuPairSolver on a GPU).  Pairs
    with N < 8 are skipped (valid = 0).  ``refine(items)`` (GpuPairRefiner on a GPU), with
    items = [(i, F, pl_inliers, pr_inliers, first p1 point, first p2 point)], returns per item
    (F_gold[9], gs_cost, pose found, R[9], t[3]) for all of the rank's valid pairs at once.
    Returns the PAIR_DTYPE table of every pair, identical on every rank, after one
    all-gather in which each rank sends only the records of the pairs it owns (padded to the
    largest owner list, as an all-gather needs equal sizes; every rank derives the same
    owner lists from the costs)."""
    ns_all = np.fromiter((p1.shape[1] for p1, _ in pairs), dtype=np.int64, count=len(pairs))
    costs = np.where(ns_all >= 8, ns_all * H, 0)
    owners = lpt_assign(costs, comm.world)
    recs = np.zeros(len(pairs), dtype=PAIR_DTYPE)
    recs["pair"] = np.arange(len(pairs))
    recs["best_index"] = -1
    for f in ("F_gold", "gs_cost", "R", "t"):
        recs[f] = np.nan
    items = []
    own = np.asarray(owners[comm.rank], dtype=np.int64)
    mine = own[ns_all[own] >= 8].tolist()
    if hasattr(solve, "many_arrays") and (refine is None or hasattr(refine, "arrays")):
        if mine:
            _pairs_arrays(pairs, H, mine, ns_all, solve, refine, recs)
        return _pairs_gather(comm, pairs, owners, recs)
    if hasattr(solve, "many"):
        outs = solve.many(mine, [pairs[i] for i in mine])
    else:
        outs = [solve(i, *pairs[i]) for i in mine]
    if mine:  # column-wise record fill (one fancy-indexed store per field)
        idx = np.asarray(mine, dtype=np.int64)
        recs["valid"][idx] = [o[0] for o in outs]
        recs["best_index"][idx] = [o[1] for o in outs]
        recs["count"][idx] = [o[2] for o in outs]
        recs["std"][idx] = [o[3] for o in outs]
        recs["F"][idx] = np.stack([np.asarray(o[4], dtype=np.float64).ravel() for o in outs])
    for i, out in zip(mine, outs):
        if refine is not None and out[0] and len(out) > 5 and len(out[5]) > 0:
            p1, p2 = pairs[i]
            S = np.asarray(out[5])
            items.append((i, np.asarray(out[4]), p1[:, S], p2[:, S], p1[:, 0], p2[:, 0]))
    if refine is not None and items:
        ref = refine(items)
        idx = np.asarray([it[0] for it in items], dtype=np.int64)
        recs["refined"][idx] = 1
        recs["F_gold"][idx] = np.stack([np.asarray(r[0], dtype=np.float64).ravel() for r in ref])
        recs["gs_cost"][idx] = [r[1] for r in ref]
        recs["pose"][idx] = [r[2] for r in ref]
        recs["R"][idx] = np.stack([np.asarray(r[3], dtype=np.float64).ravel() for r in ref])
        recs["t"][idx] = np.stack([np.asarray(r[4], dtype=np.float64).ravel() for r in ref])
    return _pairs_gather(comm, pairs, owners, recs)


def _pairs_arrays(pairs, H, mine, ns_all, solve, refine, recs):
    """run_pairs' stages on concatenated arrays (a solver with many_arrays, a refiner with
    arrays): one concatenation of the rank's pairs, the inlier columns gathered by one fancy
    index, the records filled column-wise -- no Python object per pair."""
    idx = np.asarray(mine, dtype=np.int64)
    off = np.zeros(len(mine) + 1, dtype=np.int64)
    np.cumsum(ns_all[idx], out=off[1:])
    p1 = np.concatenate([pairs[i][0] for i in mine], axis=1).astype(np.float64, copy=False)
    p2 = np.concatenate([pairs[i][1] for i in mine], axis=1).astype(np.float64, copy=False)
    if (refine is not None and getattr(refine, "fused", False) and hasattr(solve, "many_two_view")
            and getattr(refine, "ctx", None) is getattr(solve, "ctx", None)):
        res, _, Fg, info, R, t, found = solve.many_two_view(idx, p1, p2, off, refine.K)
        _fill_ransac(recs, idx, res)
        sel = np.flatnonzero((res["best_index"] >= 0) & (res["best_count"] > 0))
        ri = idx[sel]
        recs["refined"][ri] = 1
        recs["F_gold"][ri] = Fg[sel]
        recs["gs_cost"][ri] = info["cost"][sel]
        recs["pose"][ri] = found[sel]
        recs["R"][ri] = R[sel]
        recs["t"][ri] = t[sel]
        return
    res, inl = solve.many_arrays(idx, p1, p2, off)
    valid, cnt = _fill_ransac(recs, idx, res)
    sel = np.flatnonzero(valid & (cnt > 0))
    if refine is None or len(sel) == 0:
        return
    k = cnt[sel]
    goff = np.zeros(len(sel) + 1, dtype=np.int64)
    np.cumsum(k, out=goff[1:])
    base = np.repeat(off[sel], k)  # pair b's inlier j: column off[b] + inl[off[b] + j]
    cols = base + inl[base + (np.arange(int(goff[-1])) - np.repeat(goff[:-1], k))]
    Fg, cost, found, R, t = refine.arrays(res["F"][sel], p1[:, cols], p2[:, cols], goff,
                                          p1[:, off[sel]].T, p2[:, off[sel]].T)
    ri = idx[sel]
    recs["refined"][ri] = 1
    recs["F_gold"][ri] = Fg
    recs["gs_cost"][ri] = cost
    recs["pose"][ri] = found
    recs["R"][ri] = R
    recs["t"][ri] = t


def _fill_ransac(recs, idx, res):
    """The RANSAC columns of the rank's records from a PAIR_RESULT_DTYPE array."""
    valid = res["best_index"] >= 0
    cnt = np.where(valid, res["best_count"], 0)
    recs["valid"][idx] = valid
    recs["best_index"][idx] = res["best_index"]
    recs["count"][idx] = cnt
    recs["std"][idx] = res["best_std"]
    recs["F"][idx] = res["F"]
    return valid, cnt


def _pairs_gather(comm, pairs, owners, recs):
    """run_pairs' exchange: each rank's own records, one all-gather, the full table."""
    if comm.world == 1:  # every record is this rank's already
        table = recs.copy()
        table["pair"] = np.arange(len(pairs))
        table["best_index"][table["valid"] == 0] = -1
        return table
    width = max(len(o) for o in owners)
    send = np.zeros(width, dtype=PAIR_DTYPE)
    own = np.asarray(owners[comm.rank], dtype=np.int64)
    send[:len(own)] = recs[own]
    parts = comm.allgather_bytes(send.tobytes())
    table = np.zeros(len(pairs), dtype=PAIR_DTYPE)
    for r, p in enumerate(parts):
        a = np.frombuffer(p, dtype=PAIR_DTYPE)
        table[np.asarray(owners[r], dtype=np.int64)] = a[:len(owners[r])]
    table["pair"] = np.arange(len(pairs))
    table["best_index"][table["valid"] == 0] = -1
    return table
