"""CPU model of a bit-set all-entry parse, checked against a brute-force parse of every entry
state (round 3, measured and not kept: DESIGN.md section 5, "Dense phase as bit sets").

State set X (bit s = state s occupied, s in 1..n1), boundary set B (entry indices that start a
trajectory's member range), cur = member-range start of the highest state (the list head).
The trajectories in descending state order have the boundaries in cyclic ascending order from
cur.  A draw w moves every state s with (w & mask(s)) <= s down by one; states keep their order,
so two trajectories can only meet as (old v, old v - 1) inside one bucket (the lower one's
boundary is deleted) or when the wrapped state lands on an occupied n1 (the head's boundary is
deleted); the wrapping trajectory (state 1, the list tail) becomes the head."""
import numpy as np


def mask_of(s):
    return (1 << int(s).bit_length()) - 1


def bits_parse(words, n1, stop_m=64):
    X = sum(1 << s for s in range(1, n1 + 1))
    B = (1 << n1) - 1
    m, cur, ev = n1, 0, []
    masks = {}
    for s in range(1, n1 + 1):
        masks.setdefault(mask_of(s), []).append(s)
    for t, w in enumerate(words):
        w = int(w)
        if m <= stop_m:
            return X, B, cur, m, ev, t
        # accept set
        A = 0
        for mk, ss in masks.items():
            v = w & mk
            lo, hi = ss[0], ss[-1]
            if v <= hi:
                a0 = max(v, lo)
                A |= ((1 << (hi + 1)) - 1) & ~((1 << a0) - 1)
        stay = X & ~A
        moved = (X & A) >> 1
        ov = stay & moved
        Xn = stay | moved
        Bs = sorted(b for b in range(n1) if (B >> b) & 1)
        r0 = Bs.index(cur)
        dels = []
        # bucket merges: at u (lower trajectory = old state u, position = #old states > u)
        u = ov
        while u:
            s = (u & -u).bit_length() - 1
            u &= u - 1
            pos = bin(X >> (s + 1)).count("1")
            dels.append((r0 + pos) % m)
        wrap = Xn & 1
        newcur_rank = r0
        if wrap:
            Xn &= ~1
            lo = Bs[(r0 - 1) % m]
            ev.append((t + 1, lo, cur))
            if (Xn >> n1) & 1:
                dels.append(r0)
            Xn |= 1 << n1
            newcur_rank = (r0 - 1) % m
        newcur = Bs[newcur_rank]
        for d in dels:
            B &= ~(1 << Bs[d])
        m -= len(dels)
        cur = newcur
        X = Xn
        assert bin(X).count("1") == m == bin(B).count("1"), (t, m)
    return X, B, cur, m, ev, len(words)


def brute(words, n1, T):
    st = n1 - np.arange(n1, dtype=np.int64)  # entry a <-> state n1 - a
    wraps = [[] for _ in range(n1)]
    msk = np.array([0] + [mask_of(s) for s in range(1, n1 + 1)], dtype=np.int64)
    for t in range(T):
        w = int(words[t])
        acc = (w & msk[st]) <= st
        st = st - acc
        z = st == 0
        if z.any():
            for a in np.nonzero(z)[0]:
                wraps[a].append(t + 1)
            st[z] = n1
    return st, wraps


def check(n1, T, seed):
    rng = np.random.RandomState(seed)
    words = rng.randint(0, 2**32, size=T, dtype=np.uint64).astype(np.uint32)
    X, B, cur, m, ev, t = bits_parse(words, n1)
    st, wraps = brute(words, n1, t)
    Bs = sorted(b for b in range(n1) if (B >> b) & 1)
    states = sorted((s for s in range(1, n1 + 1) if (X >> s) & 1), reverse=True)
    r0 = Bs.index(cur)
    lst = [(Bs[(r0 + q) % m], states[q]) for q in range(m)]
    # every entry's state at t = the state of the list element whose range holds it
    for q, (lo, s) in enumerate(lst):
        hi = lst[(q + 1) % m][0]
        ents = [a for a in range(n1) if ((lo <= a < hi) if lo < hi else (a >= lo or a < hi))]
        assert all(st[a] == s for a in ents), (q, lo, hi, s)
    # every entry's wraps = the logged wraps whose range holds it, each once
    got = [[] for _ in range(n1)]
    for tt, lo, hi in ev:
        for a in range(n1):
            if (lo <= a < hi) if lo < hi else (a >= lo or a < hi):
                got[a].append(tt)
    assert got == wraps
    return t, m, len(ev)


if __name__ == "__main__":
    for n1, T, seed in [(100, 3000, 1), (257, 20000, 2), (1000, 20000, 3), (1999, 40000, 4), (65, 5000, 5)]:
        print(n1, check(n1, T, seed))


def lane_emulation(words, n1, stop=64):
    """k_np_entry_bits step by step at lane level (accept masks, DPP shift, event bookkeeping
    with the inclusive boundary prefix Pb, the deletion list and the rank adjustments)."""
    M32 = 0xffffffff
    popc = lambda x: bin(x).count("1")
    T0 = [0] * 32
    for ln in range(32):
        for k in range(5):
            lo, hi = 1 << k, (2 << k) - 1
            v = ln & hi
            for s in range(lo, hi + 1):
                if s >= v:
                    T0[ln] |= 1 << s
    base = [32 * l for l in range(64)]
    mk = [0] + [M32 >> (32 - (b | 1).bit_length()) for b in base[1:]]
    def accept(w):
        out = []
        for l in range(64):
            if l == 0:
                out.append(T0[w & 31]); continue
            d = (w & mk[l]) - base[l]
            cl = 0 if d < 0 else (32 if d > 32 else d)
            out.append(((M32 << cl) & 0xffffffffffffffff) & M32)
        return out
    X = [0] * 64; B = [0] * 64; Pb = [0] * 64
    for l in range(64):
        for s in range(max(1, base[l]), min(n1, base[l] + 31) + 1):
            X[l] |= 1 << (s - base[l])
        for e in range(base[l], min(n1 - 1, base[l] + 31) + 1):
            B[l] |= 1 << (e - base[l])
        Pb[l] = min(n1, base[l] + 32)
    m, r0, cur, ev = n1, 0, 0, []
    Ln, nbit = n1 >> 5, 1 << (n1 & 31)

    def locate(g):
        Lb = sum(1 for l in range(64) if Pb[l] <= g)
        bl, pl = B[Lb], Pb[Lb]
        j = g - (pl - popc(bl))
        for i in range(32):
            if (bl >> i) & 1 and popc(bl & ((1 << i) - 1)) == j:
                return Lb, i
        raise AssertionError("select")

    for t, w in enumerate(words):
        w = int(w)
        A = accept(w)
        xa = [X[l] & A[l] for l in range(64)]
        y = [xa[l + 1] if l < 63 else 0 for l in range(64)]
        mv = [((y[l] << 32 | xa[l]) >> 1) & M32 for l in range(64)]
        st = [X[l] ^ xa[l] for l in range(64)]
        ov = [st[l] & mv[l] for l in range(64)]
        Xn = [st[l] | mv[l] for l in range(64)]
        if any(ov) or (Xn[0] & 1):
            mo = m
            wrap = Xn[0] & 1
            dl = []
            lo_w = 0
            if wrap:
                Lb, bit = locate(mo - 1 if r0 == 0 else r0 - 1)
                lo_w = 32 * Lb + bit
            P = [sum(popc(X[j]) for j in range(l + 1)) for l in range(64)]
            for L in range(64):
                o = ov[L]
                while o:
                    b = (o & -o).bit_length() - 1
                    o &= o - 1
                    pos = (mo - P[L]) + popc(0 if b == 31 else X[L] >> (b + 1))
                    g = r0 + pos
                    dl.append(g - mo if g >= mo else g)
            if wrap:
                Xn[0] &= ~1
                hit = Xn[Ln] & nbit
                Xn[Ln] |= nbit
                if hit:
                    dl.append(r0)
                ev.append((t + 1, lo_w, cur))
            R = (mo - 1 if r0 == 0 else r0 - 1) if wrap else r0
            dec = 0
            for i, g in enumerate(dl):
                adj = sum(1 for j in range(i) if dl[j] < g)
                Lb, bit = locate(g - adj)
                B[Lb] &= ~(1 << bit)
                for l in range(Lb, 64):
                    Pb[l] -= 1
                dec += 1 if g < R else 0
            r0 = R - dec
            if wrap:
                cur = lo_w
            m = mo - len(dl)
            X = Xn
            if m <= stop:
                return X, B, r0, m, ev, t + 1
        else:
            X = Xn
    return X, B, r0, m, ev, len(words)


def check_lanes(n1, T, seed):
    rng = np.random.RandomState(seed)
    words = rng.randint(0, 2**32, size=T, dtype=np.uint64).astype(np.uint32)
    Xb, Bb, cur, m, ev, t = bits_parse(words, n1)
    X, B, r0, m2, ev2, t2 = lane_emulation(words, n1)
    assert (t, m) == (t2, m2), ((t, m), (t2, m2))
    assert ev == ev2
    Xi = sum(X[l] << (32 * l) for l in range(64))
    Bi = sum(B[l] << (32 * l) for l in range(64))
    assert Xi == Xb and Bi == Bb
    Bs = sorted(b for b in range(n1) if (Bb >> b) & 1)
    assert Bs[r0] == cur
    return t, m, len(ev)
