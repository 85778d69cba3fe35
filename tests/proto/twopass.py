"""Python model of the two-pass encoder (rc_enc2.hip) -- TEST INFRASTRUCTURE.

compress.c's order-1 and order-2 statistics depend only on the packet's bytes,
never on the coder's output, so the HIP encoder splits compress into
  pass 1 (context scan, one wavefront per packet): every order-1/order-2
         coding interval of the packet, derived from the packet's history;
  pass 2 (coder, one lane per packet): the root context (order 0, in LDS)
         and the range coder, consuming pass 1's per-position records.
This module restates both passes in plain Python with the exact record
format of the kernels, so that tests can check the decomposition against
the oracle on the CPU (tests/test_twopass_model.py).

Statistics of a sub-context (compress.c:159-199, :286-316), no rescale: at a
visit with t earlier visits, of which `dist` introduced a new symbol,
  escapes = 5 * dist, total = escapes + 2 * t                    (:309-312)
and for the visited symbol, with `same` earlier visits of that symbol and
`less` earlier visits of smaller symbols,
  count = 2 * same, under = 2 * less                             (:161-199)
A context is visited at position i (i = index in the packet):
  order 2: i >= 2, context (x[i-2], x[i-1])                      (:286-316)
  order 1: i == 1, or i >= 2 and the order-2 context lacked x[i], context x[i-1]
  root:    i == 0, or order 1 was visited and lacked x[i]        (:318-329)
Both sub-contexts of position i hold positions whose previous byte is x[i-1]:
pass 1 buckets positions by that byte, and the statistics are counts over a
position's bucket predecessors.  A packet takes the fast path when every
bucket holds <= 64 positions (so every statistic is <= 63 and no count can
reach the rescale threshold of 252, compress.c:313) and it is shorter than
1920 bytes (no model reset, compress.c:148-157); other packets go to the
lane kernels.

Record of position i (primary u16, optional ext u32):
  primary bits 0-2 type, 3-8 tA, 9-14 dA
  type 0: no sub-context codes                      -> root
       1: order 1 escape (tA, dA) = (t1, dist1)     -> root
       2: order 1 hit (t1, dist1), ext (same1, less1)
       3: order 2 escape (t2, dist2)                -> root
       4: order 2 escape (t2, dist2), ext order 1 escape (t1, dist1) -> root
       5: order 2 escape (t2, dist2), ext order 1 hit (t1, dist1, same1, less1)
       6: order 2 hit (t2, dist2), ext (same2, less2)
  ext fields are 6-bit, packed from bit 0 in the order listed.
"""
from __future__ import annotations

from collections import defaultdict

MAX_LEN = 1919
MAX_BUCKET = 64


def scan(p: bytes):
    """Pass 1: (primary[N], ext[N]) or None when the packet takes the lane kernels."""
    n = len(p)
    if n == 0 or n > MAX_LEN:
        return None
    buckets = defaultdict(list)
    for i in range(1, n):
        buckets[p[i - 1]].append(i)
    if buckets and max(len(v) for v in buckets.values()) > MAX_BUCKET:
        return None
    prim = [0] * n
    ext = [0] * n
    found2, vis1, found1 = {}, {}, {}
    for lst in buckets.values():
        for j, i in enumerate(lst):
            v = p[i]
            t2 = same2 = less2 = dist2 = 0
            if i >= 2:
                for k in lst[:j]:
                    if k >= 2 and p[k - 2] == p[i - 2]:
                        t2 += 1
                        same2 += p[k] == v
                        less2 += p[k] < v
                        dist2 += not found2[k]
                found2[i] = same2 > 0
            vis1[i] = i == 1 or not found2[i]
            t1 = same1 = less1 = dist1 = 0
            if vis1[i]:
                for k in lst[:j]:
                    if vis1[k]:
                        t1 += 1
                        same1 += p[k] == v
                        less1 += p[k] < v
                        dist1 += not found1[k]
            found1[i] = vis1[i] and same1 > 0
            if i >= 2 and found2[i]:
                typ, a, e = 6, (t2, dist2), (same2, less2)
            elif i >= 2 and t2 > 0:
                if t1 == 0:
                    typ, a, e = 3, (t2, dist2), ()
                elif found1[i]:
                    typ, a, e = 5, (t2, dist2), (t1, dist1, same1, less1)
                else:
                    typ, a, e = 4, (t2, dist2), (t1, dist1)
            elif t1 == 0:
                typ, a, e = 0, (0, 0), ()
            elif found1[i]:
                typ, a, e = 2, (t1, dist1), (same1, less1)
            else:
                typ, a, e = 1, (t1, dist1), ()
            prim[i] = typ | a[0] << 3 | a[1] << 9
            ext[i] = sum(f << (6 * k) for k, f in enumerate(e))
    return prim, ext


class _Enc:
    """compress.c:114-146 (carry-less range coder, output bounded by out_limit)."""

    def __init__(self, out_limit):
        self.low, self.range, self.out, self.lim, self.ok = 0, 0xFFFFFFFF, bytearray(), out_limit, True

    def put(self, b):
        if len(self.out) >= self.lim:
            self.ok = False
            return False
        self.out.append(b)
        return True

    def code(self, under, count, total):
        if not self.ok:
            return
        self.range //= total
        self.low = (self.low + under * self.range) & 0xFFFFFFFF
        self.range = (self.range * count) & 0xFFFFFFFF
        while True:
            if (self.low ^ (self.low + self.range)) & 0xFFFFFFFF >= 1 << 24:
                if self.range >= 1 << 16:
                    break
                self.range = (-self.low) & 0xFFFF
            if not self.put(self.low >> 24):
                return
            self.range = (self.range << 8) & 0xFFFFFFFF
            self.low = (self.low << 8) & 0xFFFFFFFF

    def flush(self):
        while self.ok and self.low:
            if not self.put(self.low >> 24):
                return
            self.low = (self.low << 8) & 0xFFFFFFFF


def _sub(t, dist, same=None, less=None):
    esc = 5 * dist
    tot = esc + 2 * t
    if same is None:
        return (0, esc, tot)
    return (esc + 2 * less, 2 * same, tot)


def code(p: bytes, prim, ext, out_limit: int):
    """Pass 2: root context + range coder over pass 1's records.  Returns
    (return value, bytes) like enet_range_coder_compress."""
    enc = _Enc(out_limit)
    cnt = [0] * 256
    rtot = 257
    for i, v in enumerate(p):
        h, e = prim[i], ext[i]
        typ, ta, da = h & 7, (h >> 3) & 63, (h >> 9) & 63
        f = [(e >> (6 * k)) & 63 for k in range(4)]
        ops = []
        if typ == 1:
            ops.append(_sub(ta, da))
        elif typ == 2:
            ops.append(_sub(ta, da, f[0], f[1]))
        elif typ == 3:
            ops.append(_sub(ta, da))
        elif typ == 4:
            ops += [_sub(ta, da), _sub(f[0], f[1])]
        elif typ == 5:
            ops += [_sub(ta, da), _sub(f[0], f[1], f[2], f[3])]
        elif typ == 6:
            ops.append(_sub(ta, da, f[0], f[1]))
        for op in ops:
            if op[1] > 0 and (op[0] > 0 or op[1] < op[2]):   # an escape is coded only if 0 < esc < total
                enc.code(*op)
        if typ in (0, 1, 3, 4):
            under = v + sum(cnt[:v])
            c = 1 + cnt[v]
            enc.code(1 + under, c, rtot)                    # root escapes = 1 (compress.c:326)
            cnt[v] += 3
            rtot += 3
            if c > 250 or rtot > 65280:                     # compress.c:328-329
                for u in range(256):
                    cnt[u] -= cnt[u] >> 1
                rtot = sum(cnt) + 1 + 256
        if not enc.ok:
            return 0, b""
    enc.flush()
    if not enc.ok:
        return 0, b""
    return len(enc.out), bytes(enc.out)


def compress(p: bytes, out_limit: int):
    r = scan(p)
    if r is None:
        return None
    return code(p, r[0], r[1], out_limit)


# ---------------------------------------------------------------- wide mode
#
# Packets with a bucket over 64 positions (low-entropy data such as game
# state) can rescale their sub-contexts (compress.c:90-112, :313-314), so the
# closed-form statistics above no longer hold for them.  The wide scan
# (rc_enc2.hip, rc_enc2_wscan) still derives every order-2/order-1 interval
# from the packet, as explicit (under, count, total) triples:
#   - buckets of <= 64 positions: the closed form, one lane per bucket;
#   - bigger buckets: their elements sorted (stably) by a = x[i-2] into runs,
#     one run per order-2 context; runs of <= DENSE_MIN visits by the closed
#     form (no rescale before 127 visits), longer runs by a dense walk; then
#     the bucket's order-1 visits (elements order 2 did not find, in position
#     order) the same way.
# A dense walk keeps the context's counts in a table and takes its visits 64
# at a time (one per lane): a visit's count and under are the table's plus
# the contributions of the earlier lanes of the round; the first lane whose
# visit triggers a rescale ends the round (later lanes are redone after it).
#
# Wide record of position i: (A, B, root) with A the order-2 code, B the
# order-1 code (None or (under, count, total)), root whether the root codes.

DENSE_MIN = 32
WAVE = 64


def _closed_form(vals, found):
    """Codes of a run of visits (values in visit order) with no rescale;
    found[k] is set for visits that found their symbol."""
    codes = []
    for j, v in enumerate(vals):
        t = j
        same = sum(1 for k in range(j) if vals[k] == v)
        less = sum(1 for k in range(j) if vals[k] < v)
        dist = sum(1 for k in range(j) if not found[k])
        esc, tot = 5 * dist, 5 * dist + 2 * t
        if same:
            codes.append((esc + 2 * less, 2 * same, tot))
            found[j] = True
        else:
            codes.append((0, esc, tot) if esc > 0 else None)
            found[j] = False
    return codes


def _dense_walk(vals, found):
    """The same codes, rescales included, in rounds of WAVE visits."""
    cnt = [0] * 256
    esc = tot = 0
    codes = [None] * len(vals)
    base = 0
    while base < len(vals):
        lanes = vals[base: base + WAVE]
        c = [cnt[v] + 2 * sum(1 for k in range(l) if lanes[k] == v) for l, v in enumerate(lanes)]
        under = [sum(cnt[:v]) + 2 * sum(1 for k in range(l) if lanes[k] < v) for l, v in enumerate(lanes)]
        new = [x == 0 for x in c]
        jstar, rescale = len(lanes), False
        out = []
        for l, v in enumerate(lanes):
            nb = sum(new[:l])
            e_l, t_l = esc + 5 * nb, tot + 2 * l + 5 * nb
            out.append((e_l + under[l], c[l], t_l) if c[l] else ((0, e_l, t_l) if e_l > 0 else None))
            if c[l] > 251 or t_l + 2 + 5 * new[l] > 65280:     # compress.c:313-314
                jstar, rescale = l + 1, True
                break
        for l in range(jstar):
            codes[base + l] = out[l]
            found[base + l] = not new[l]
            cnt[lanes[l]] += 2
            esc += 5 * new[l]
            tot += 2 + 5 * new[l]
        if rescale:                                            # compress.c:90-112
            cnt = [x - (x >> 1) for x in cnt]
            esc -= esc >> 1
            tot = sum(cnt) + esc
        base += jstar
    return codes


def _walk(vals, found):
    if len(vals) <= DENSE_MIN:
        return _closed_form(vals, found)
    return _dense_walk(vals, found)


def _scan_wide_segment(p: bytes):
    """Records of a model segment (the packet, or the bytes after a model
    reset): (A, B, root) per position, and per position whether order 2 /
    order 1 found its byte."""
    n = len(p)
    recs = [None] * n
    recs[0] = (None, None, True)
    f2all, f1all = [False] * n, [False] * n
    buckets = defaultdict(list)
    for i in range(1, n):
        buckets[p[i - 1]].append(i)
    for lst in buckets.values():
        A = {}
        f2 = {i: False for i in lst}
        if len(lst) <= MAX_BUCKET:
            runs = defaultdict(list)
            for i in lst:
                if i >= 2:
                    runs[p[i - 2]].append(i)
            for run in runs.values():
                found = [False] * len(run)
                for i, cd, fd in zip(run, _closed_form([p[i] for i in run], found), found):
                    A[i], f2[i] = cd, fd
        else:
            # stable sort by a; position 1 (no order-2 context) apart
            order = sorted((i for i in lst if i >= 2), key=lambda i: p[i - 2])
            k = 0
            while k < len(order):
                e = k
                while e < len(order) and p[order[e] - 2] == p[order[k] - 2]:
                    e += 1
                run = order[k:e]
                found = [False] * len(run)
                codes = _walk([p[i] for i in run], found)
                for i, cd, fd in zip(run, codes, found):
                    A[i], f2[i] = cd, fd
                k = e
        vis1 = [i for i in lst if not f2[i]]
        found = [False] * len(vis1)
        codes = _walk([p[i] for i in vis1], found) if len(lst) > MAX_BUCKET else _closed_form([p[i] for i in vis1], found)
        B = {i: (cd, fd) for i, cd, fd in zip(vis1, codes, found)}
        for i in lst:
            f2all[i] = f2[i]
            if f2[i]:
                recs[i] = (A.get(i), None, False)
            else:
                cd, fd = B[i]
                f1all[i] = fd
                recs[i] = (A.get(i), cd, not fd)
    return recs, f2all, f1all


NODE_LIMIT = 4096 - 2          # compress.c:148-157


def _reset_point(p: bytes, f2, f1):
    """compress.c:148-157: the first position after which the segment holds
    NODE_LIMIT symbols (1 for the root, one per symbol created: in the
    order-2 context when it lacks the byte, in the order-1 context when it is
    visited and lacks it, at the root when it is visited for the first time
    with that byte), or None."""
    nodes, seen = 1, set()
    for i, v in enumerate(p):
        nodes += (i >= 2 and not f2[i]) + (i >= 1 and not f2[i] and not f1[i])
        if i == 0 or (not f2[i] and not f1[i]):
            nodes += v not in seen
            seen.add(v)
        if nodes >= NODE_LIMIT:
            return i
    return None


def scan_wide(p: bytes, max_len: int = MAX_LEN):
    """Wide-mode pass 1: one (A, B, root, reset) record per position (reset:
    the model starts over after the position), or None for a packet the wide
    scan does not take (empty, or longer than max_len)."""
    n = len(p)
    if n == 0 or n > max_len:
        return None
    out, s = [], 0
    while s < n:
        recs, f2, f1 = _scan_wide_segment(p[s:])
        r = _reset_point(p[s:], f2, f1)
        if r is None or s + r + 1 >= n:
            out += [rc + (False,) for rc in recs]
            break
        out += [rc + (False,) for rc in recs[: r]] + [recs[r] + (True,)]
        s += r + 1
    return out


def code_wide(p: bytes, recs, out_limit: int):
    """Pass 2 over wide records: as code(), with explicit intervals."""
    enc = _Enc(out_limit)
    cnt = [0] * 256
    rtot = 257
    for i, v in enumerate(p):
        a, b, root, reset = recs[i]
        for op in (a, b):
            if op is not None:
                enc.code(*op)
        if root:
            under = v + sum(cnt[:v])
            c = 1 + cnt[v]
            enc.code(1 + under, c, rtot)
            cnt[v] += 3
            rtot += 3
            if c > 250 or rtot > 65280:
                for u in range(256):
                    cnt[u] -= cnt[u] >> 1
                rtot = sum(cnt) + 1 + 256
        if reset:                                           # compress.c:148-157
            cnt = [0] * 256
            rtot = 257
        if not enc.ok:
            return 0, b""
    enc.flush()
    if not enc.ok:
        return 0, b""
    return len(enc.out), bytes(enc.out)


def compress_wide(p: bytes, out_limit: int, max_len: int = MAX_LEN):
    r = scan_wide(p, max_len)
    if r is None:
        return None
    return code_wide(p, r, out_limit)
