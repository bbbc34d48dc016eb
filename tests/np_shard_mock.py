"""CPU stand-in for tsbb15_amd._ffi.NpShard (test infrastructure only).

It implements the same four steps (parse / maps / compose / tuples) with the same meaning, so
the exchange logic of tsbb15_amd.parallel.np_sharded_segments (start offsets, the next rank's
first start, the rank holding the final state, multi-segment continuation) can be checked under
gloo / thread ranks without a GPU.  Inside, it simply replays the raw MT19937 word stream
(numpy's bit generator, whose legacy state is the (key, pos) pair of np.random.get_state) and
walks the Fisher-Yates parse of fun.py:305-306 (numpy's random_interval: w & mask(i) <= i) or
ransac.py:12-19 (CPython's randbelow: w >> (32 - bit_length(i + 1)) <= i) draw by draw.
"""
import math

import numpy as np


def _accept(w, i, py):
    if py:
        return (w >> (32 - (i + 1).bit_length())) <= i
    return (w & ((1 << i.bit_length()) - 1)) <= i


def _draw(w, i, py):
    if py:
        return w >> (32 - (i + 1).bit_length())
    return w & ((1 << i.bit_length()) - 1)


def raw_words(key, pos, count):
    bg = np.random.MT19937()
    bg.state = {"bit_generator": "MT19937",
                "state": {"key": np.asarray(key, np.uint32), "pos": int(pos)}}
    return bg.random_raw(int(count)).astype(np.uint64)


def state_after(key, pos, steps):
    bg = np.random.MT19937()
    bg.state = {"bit_generator": "MT19937",
                "state": {"key": np.asarray(key, np.uint32), "pos": int(pos)}}
    if steps:
        bg.random_raw(int(steps))
    st = bg.state["state"]
    return np.asarray(st["key"], np.uint32), int(st["pos"])


def parse_starts(words, n, py):
    """Start draw of every complete hypothesis in ``words`` (plus the end of the last)."""
    starts, d, nw = [0], 0, len(words)
    while True:
        for i in range(n - 1, 0, -1):
            while d < nw and not _accept(int(words[d]), i, py):
                d += 1
            if d >= nw:
                return starts
            d += 1
        starts.append(d)


def tuple_of(words, a, n, k, py):
    x = list(range(n))
    d = a
    for i in range(n - 1, 0, -1):
        while not _accept(int(words[d]), i, py):
            d += 1
        j = _draw(int(words[d]), i, py)
        x[i], x[j] = x[j], x[i]
        d += 1
    return x[:k], d


class MockNpShard:
    """The NpShard interface on the CPU.  ``seg_cap`` bounds the hypotheses per segment (the
    GPU's bound is memory), ``slack`` is the draw margin beyond the expected need."""

    def __init__(self, n, k, world, rank, py=False, seg_cap=None, slack=None):
        self.n, self.k, self.world, self.rank, self.py = int(n), int(k), int(world), int(rank), py
        self.seg_cap = seg_cap
        self.slack = 16 * self.n + 4096 if slack is None else int(slack)

    def close(self):
        pass

    def parse(self, key, pos, count):
        n = self.n
        E = 0.0
        for i in range(1, n):
            m = (1 << (i + 1 if self.py else i).bit_length()) - 1
            E += (m + 1) / (i + 1)
        hs = int(count) if self.seg_cap is None else min(int(count), int(self.seg_cap))
        D = int(math.ceil(hs * E * 1.03)) + self.slack
        self.Dr = -(-D // self.world)
        self.key, self.pos = np.asarray(key, np.uint32).copy(), int(pos)
        lo, hi = self.rank * self.Dr, (self.rank + 1) * self.Dr
        total = self.world * self.Dr
        # the words of the whole segment plus a margin (the straddling hypothesis)
        self.words = raw_words(key, pos, total + 64 * n + 4096)
        starts = parse_starts(self.words[:total], n, self.py)
        self.own = np.array([s for s in starts if lo <= s < hi], np.int64)
        return {"count": hs, "C": self.world, "Cr": 1, "Wc": self.Dr, "D": total,
                "map_bytes": 16}

    def maps(self):
        return np.array([self.rank, len(self.own)], np.int64).tobytes()

    def compose(self, blobs):
        assert len(blobs) == self.world
        for r, b in enumerate(blobs):
            assert int(np.frombuffer(b[:16], np.int64)[0]) == r, "blobs out of rank order"
        first = int(self.own[0]) if len(self.own) else -1
        return len(self.own), first

    def tuples(self, base, hi, next_start, final_idx, key):
        cnt = int(hi) - int(base)
        out = np.zeros((max(cnt, 0), self.k), np.int32)
        for h in range(cnt):
            a = int(self.own[h])
            b = int(self.own[h + 1]) if h + 1 < len(self.own) else int(next_start)
            out[h], d = tuple_of(self.words, a, self.n, self.k, self.py)
            assert d == b, (h, d, b)
        fin = None
        if final_idx >= 0:
            used = int(self.own[int(final_idx) - int(base)])
            fin = state_after(self.key, self.pos, used)
        return out, fin
