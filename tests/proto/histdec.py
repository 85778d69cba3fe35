"""Python model of the bucket-history decoder (rc_dec4.hip) -- TEST INFRASTRUCTURE.

The decoder keeps, per packet, one record per previous byte b ("bucket b"):
the history of the positions i with x[i-1] = b, each as (a = x[i-2], v =
x[i], decoded at order 2, new to its order-2 context, new to its order-1
context).  Both sub-contexts of position i live in
its bucket (order 1 = (x[i-1]), order 2 = (x[i-2], x[i-1])), and their
statistics follow from that history (compress.c:159-199, :536-615; no
rescale while a bucket holds <= 64 positions):
  order 2: the bucket's positions with the same a; t2 of them, dist2 of
           them new to that context;  escapes = 5 dist2, total =
           escapes + 2 t2
  order 1: the bucket's positions not decoded at order 2 (those visit order
           1, compress.c:598-615); t1 of them, dist1 of them new to it;
           escapes = 5 dist1, total = escapes + 2 t1
"New" is a property of the history (the symbol was absent from the context
when the position was added: compress.c:306-310 / :606-610), not of the
decode path: a corrupt stream can escape from a context that holds the
symbol, and the reference's patch then finds it there.
  a symbol u of a context has count 2 * (positions with v = u) and
  cumulative count 2 * (positions with v < u): the code r = READ - escapes
  selects the value of rank floor(r / 2) among the positions' values.
Appending the decoded position to its bucket applies every update the
reference makes (its order-2 context always gains v, its order-1 context
when it was visited); the root (order 0) is kept as counts.

decode() returns (return value, bytes), or None where the GPU decoder hands
the packet to the lane kernels (a bucket over 64 positions, the node count
reaching compress.c's model reset, a root code past symbol 255).
"""
from __future__ import annotations

from collections import defaultdict

MAX_BUCKET = 64
NODE_LIMIT = 4096 - 2


class _Dec:
    def __init__(self, data: bytes):
        self.data, self.p = data, 0
        self.low, self.range, self.code = 0, 0xFFFFFFFF, 0
        for _ in range(4):                              # compress.c:344-350
            self.code = (self.code << 8) & 0xFFFFFFFF
            if self.p < len(data):
                self.code |= data[self.p]
                self.p += 1

    def read(self, total):                              # compress.c:352, truncated to u16
        self.range //= total
        return ((self.code - self.low) & 0xFFFFFFFF) // self.range & 0xFFFF

    def decode(self, under, count, total):              # compress.c:354-371
        self.low = (self.low + under * self.range) & 0xFFFFFFFF
        self.range = (self.range * count) & 0xFFFFFFFF
        while True:
            if ((self.low ^ (self.low + self.range)) & 0xFFFFFFFF) >= 1 << 24:
                if self.range >= 1 << 16:
                    break
                self.range = (-self.low) & 0xFFFF
            self.code = (self.code << 8) & 0xFFFFFFFF
            if self.p < len(self.data):
                self.code |= self.data[self.p]
                self.p += 1
            self.range = (self.range << 8) & 0xFFFFFFFF
            self.low = (self.low << 8) & 0xFFFFFFFF


def _sub(dec, elems, esc, tot):
    """One sub-context: None (escape coded or not coded), 'fail', or the value."""
    code = dec.read(tot)
    if code < esc:
        dec.decode(0, esc, tot)
        return None
    r = code - esc
    vals = sorted(e[1] for e in elems)
    if r >= 2 * len(vals):
        return "fail"                                   # compress.c:416 (TRY_DECODE createRight)
    u = vals[r // 2]
    under = esc + 2 * sum(1 for x in vals if x < u)
    cnt = 2 * sum(1 for x in vals if x == u)
    dec.decode(under, cnt, tot)
    return u


def decode(data: bytes, out_limit: int):
    if len(data) == 0:
        return 0, b""
    dec = _Dec(data)
    buckets = defaultdict(list)                         # b -> [(a or None, v, at2, new2, new1)]
    cnt = [0] * 256
    rtot = 257
    out = bytearray()
    nodes = 1
    while True:
        i = len(out)
        hit2 = hit1 = False
        v = None
        elems = buckets[out[i - 1]] if i >= 1 else []
        if i >= 2:
            same = [e for e in elems if e[0] == out[i - 2]]
            if same:
                d2 = sum(1 for e in same if e[3])
                r = _sub(dec, same, 5 * d2, 5 * d2 + 2 * len(same))
                if r == "fail":
                    return 0, b""
                if r is not None:
                    v, hit2 = r, True
        if v is None and i >= 1:
            vis = [e for e in elems if not e[2]]
            if vis:
                d1 = sum(1 for e in vis if e[4])
                r = _sub(dec, vis, 5 * d1, 5 * d1 + 2 * len(vis))
                if r == "fail":
                    return 0, b""
                if r is not None:
                    v, hit1 = r, True
        if v is None:                                   # root, compress.c:570-596
            code = dec.read(rtot)
            if code < 1:
                dec.decode(0, 1, rtot)
                break                                   # end of stream
            code -= 1
            acc = 0                                     # symbol u: [u + acc, u + acc + 1 + cnt[u])
            for u in range(256):
                if code < u + acc + 1 + cnt[u]:
                    break
                acc += cnt[u]
            else:
                return None                             # past symbol 255: the exact path
            v = u
            under = u + acc
            c = cnt[u]
            dec.decode(1 + under, 1 + c, rtot)
            nodes += c == 0
            cnt[u] += 3
            rtot += 3
            if 1 + c > 250 or rtot > 65280:
                for x in range(256):
                    cnt[x] -= cnt[x] >> 1
                rtot = sum(cnt) + 1 + 256
        if i >= 1:
            a = out[i - 2] if i >= 2 else None
            new2 = i >= 2 and all(e[1] != v for e in elems if e[0] == a)
            new1 = not hit2 and all(e[1] != v for e in elems if not e[2])
            nodes += new2 + new1                        # compress.c:165-186 creates a node per new symbol
            elems.append((a, v, hit2, new2, new1))
            if len(elems) > MAX_BUCKET:
                return None
        if len(out) >= out_limit:
            return 0, b""                               # compress.c:617
        out.append(v)
        if nodes >= NODE_LIMIT:
            return None                                 # model reset: the lane kernels
    return len(out), bytes(out)
