"""Design model of the streamed variable-size decode (CPU; not product, not the
oracle). It restates, step for step, the algorithm a one-pass general decode
kernel needs, so its correctness can be checked against the oracle before any
GPU code exists (tests/test_stream_model_cpu.py):

  1. tiles of T blob bytes, processed in ANY order (on the GPU: a wave per tile,
     the tile plus an E-byte overhang staged in LDS): a speculative entry (the
     first confirmed candidate, or anything -- `pick` may be adversarial), the
     walk to the tile end, every listed frame hashed and compared at once;
  2. group summaries (256 tiles, the general walk's B1 fold) by whichever tile of
     the group finishes last;
  3. the link (the general walk's B2, groups in order, up to 64 per step, a group
     that disagrees linked tile by tile with re-walks), fed only the groups that
     are ready (`ready_prefix` lets a test starve it);
  4. per tile, once its group is linked, the deferred work in ANY order: frame
     positions and stored checksums scattered to walk order, and the tile's words
     of the batch-checksum input (word m = hi32(cs[m-6]) | lo32(cs[m-5]) << 32,
     assigned to the tile holding frame m-6; the next frame's checksum read at the
     tile's exit) added to per-block partial sums and counts;
  5. the chain over blocks whose count reached 128 (provably full blocks), then
     the finisher: the partial block recomputed from the walk-order checksums,
     the last stripe, the merge; precedence as batch.rs:395-421, 461-506.

Word-level XXH3 follows oracle/xxh3_ref.c (hash_long); the record layout and the
errors follow batch.rs (see oracle/codec_ref.c)."""
from __future__ import annotations

import random
import struct

M64 = (1 << 64) - 1
P32_1, P32_2, P32_3 = 0x9E3779B1, 0x85EBCA77, 0xC2B2AE3D
P64_1, P64_2, P64_3 = 0x9E3779B185EBCA87, 0xC2B2AE3D27D4EB4F, 0x165667B19E3779F9
P64_4, P64_5 = 0x85EBCA77C2B2AE63, 0x27D4EB2F165667C5
PMX1 = 0x165667919E3779F9


def _secret() -> bytes:
    """the default 192-byte XXH3 secret, as oracle/xxh3_ref.c holds it"""
    import os
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle",
                            "xxh3_ref.c")).read()
    body = src[src.index("kSecret[192] = {"):]
    body = body[:body.index("};")]
    return bytes(int(x, 16) for x in re.findall(r"0x([0-9a-f]{2})", body))


SECRET = _secret()
assert len(SECRET) == 192
ACC_INIT = [P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1]
HDR, FH = 256, 48
STOP = 1 << 63
NOSTART = M64
NOTLIVE = 0xFFFFFFFF
GRP_TILES = 256
OK, EOF, VALIDATION, BATCH_CS, MSG_CS = 0, 1, 2, 3, 4
V_FRAMES_DO_NOT_TILE = 3


def sw(k: int) -> int:  # secret word at byte offset 8k (kSecretW8)
    return struct.unpack_from("<Q", SECRET, 8 * k)[0]


def s_at(off: int) -> int:  # secret u64 at any byte offset
    return struct.unpack_from("<Q", SECRET, off)[0]


def mul32x32(k: int) -> int:
    return ((k & 0xFFFFFFFF) * (k >> 32)) & M64


def scramble(a: int, j: int) -> int:
    a ^= a >> 47
    a ^= s_at(128 + 8 * j)
    return (a * P32_1) & M64


def fold64(a: int, b: int) -> int:
    p = a * b
    return (p & M64) ^ (p >> 64)


def avalanche(h: int) -> int:
    h ^= h >> 37
    h = (h * PMX1) & M64
    return h ^ (h >> 32)


def u32(b, o):
    return struct.unpack_from("<I", b, o)[0]


def u64(b, o):
    return struct.unpack_from("<Q", b, o)[0]


# ------------------------------------------------------------------ the walk pieces
def frame_at(blob: bytes, p: int):
    """-> frame end if a valid frame header starts at p (reserved zero, fits), else None"""
    bl = len(blob)
    if p >= bl or bl - p < FH:
        return None
    if u64(blob, p + 40) != 0:
        return None
    e = p + FH + u32(blob, p + 32) + u32(blob, p + 36)
    return e if e <= bl else None


def walk(blob: bytes, p: int, hi: int):
    """the candidate chain from p while p < hi -> (offsets, stored checksums, exit | STOP)"""
    lst, lcs = [], []
    while p < hi:
        e = frame_at(blob, p)
        if e is None:
            break
        lst.append(p)
        lcs.append(u64(blob, p))
        p = e
    return lst, lcs, (p | STOP) if p < hi else p


def pick_entry(blob: bytes, lo: int, hi: int, rng: random.Random | None):
    """The speculative entry: the first confirmed candidate (its successor is a
    valid header inside the tile), moved to a later confirmed one of its 16-B
    cluster; else the clean candidate with the nearest exit; else the first valid.
    With rng, a deliberately wrong (but valid) candidate now and then: only the
    speed may depend on the pick, never the result."""
    cands = [p for p in range(lo, hi) if frame_at(blob, p) is not None]
    if not cands:
        return NOSTART
    if rng is not None and rng.random() < 0.25:
        return rng.choice(cands)
    pick = NOSTART
    last_c = None
    clean_p, clean_x = NOSTART, None
    for c in cands:
        if pick != NOSTART and c > last_c + 16:
            break
        e = frame_at(blob, c)
        if e < hi:
            if frame_at(blob, e) is not None:
                pick = c
                last_c = c
                continue
        elif pick == NOSTART and (clean_x is None or e < clean_x):
            clean_p, clean_x = c, e
        if pick != NOSTART:
            last_c = c
    if pick != NOSTART:
        return pick
    return clean_p if clean_p != NOSTART else cands[0]


class Tile:
    __slots__ = ("s", "x", "lst", "lcs", "bad", "pre", "e", "base", "rewalked")


def process_tile(blob: bytes, t: int, T: int, rng, verify: bool) -> Tile:
    bl = len(blob)
    lo, hi = t * T, min((t + 1) * T, bl)
    tl = Tile()
    s = 0 if t == 0 else pick_entry(blob, lo, hi, rng)
    tl.s = s
    if s == NOSTART:
        tl.lst, tl.lcs, tl.x = [], [], NOSTART
    else:
        tl.lst, tl.lcs, tl.x = walk(blob, s, hi)
    tl.bad = hash_list(blob, tl.lst, tl.x) if verify else None
    tl.pre = NOTLIVE
    tl.e = M64
    tl.base = 0
    tl.rewalked = False
    return tl


def hash_list(blob: bytes, lst, x):
    """first listed frame whose XXH3-64 over [p + 8, end) differs from its stored
    checksum (a frame's end is the next listed start, the last one's the exit)"""
    from oracle import oracle as O
    for k, p in enumerate(lst):
        end = lst[k + 1] if k + 1 < len(lst) else (x & ~STOP)
        if O.xxh3_64(blob[p + 8:end]) != u64(blob, p):
            return k
    return None


# ------------------------------------------------------------ group summary (B1 fold)
def group_summary(tiles, g, ntiles, T, bl):
    """decode_general.hip phase B1 for one group, lane by lane (4 tiles per lane)"""
    lanes = []
    for lane in range(64):
        tb = GRP_TILES * g + 4 * lane
        lhas, lok, lterm = False, True, False
        ls, lx, lhi, lc = NOSTART, 0, 0, 0
        pre = [NOTLIVE] * 4
        for i in range(4):
            t = tb + i
            if t >= ntiles or lterm:
                continue
            tl = tiles[t]
            s, x, c = tl.s, tl.x, len(tl.lst)
            hi_t = min((t + 1) * T, bl)
            lhi = hi_t
            if s != NOSTART and not (lhas and lx >= hi_t):
                if lhas:
                    lok &= s == lx
                else:
                    ls = s
                lhas = True
                pre[i] = lc
                lc += c
                lx = x
                lterm = bool(x & STOP) or x >= bl
            elif lhas:
                lok &= lx >= hi_t
        lanes.append((lhas, lok, lterm, ls, lx, lhi, lc, pre))
    term = [ln[0] and ln[2] for ln in lanes]
    last = term.index(True) if any(term) else 63
    live = [ln[0] and k <= last for k, ln in enumerate(lanes)]
    S, X, CNT, ok = NOSTART, 0, 0, True
    if any(live):
        f0 = live.index(True)
        lh = max(k for k in range(64) if live[k])
        pm, run = [], 0
        for k in range(64):
            run = max(run, lanes[k][4] if live[k] else 0)
            pm.append(run)
        inc = 0
        for k in range(64):
            lhas, lok, lterm, ls, lx, lhi, lc, pre = lanes[k]
            pred = pm[k - 1] if k > 0 else 0
            okl = k < f0 or k > last or lhi == 0 or (lok and (k == f0 or (ls == pred if lhas else pred >= lhi)))
            ok &= okl
            c = lc if live[k] else 0
            for i in range(4):
                t = GRP_TILES * g + 4 * k + i
                if t < ntiles:
                    tiles[t].pre = inc + pre[i] if (live[k] and pre[i] != NOTLIVE) else NOTLIVE
            inc += c
        S, X, CNT = lanes[f0][3], lanes[lh][4], inc
    else:
        for k in range(64):
            for i in range(4):
                t = GRP_TILES * g + 4 * k + i
                if t < ntiles:
                    tiles[t].pre = NOTLIVE
    return dict(S=S, X=X, CNT=CNT, ok=ok, term=any(term))


# ------------------------------------------------------------------ the link (B2)
def link(blob, tiles, groups, ntiles, T, ready_prefix):
    """decode_general.hip phase B2, fed the groups that are ready. -> (nwalk, end)
    and per group mode (0 no frames, 1 as summarised, 2 tile by tile) and base."""
    bl = len(blob)
    ng = len(groups)
    e, total, ended = 0, 0, False
    G0 = 0
    while G0 < ng:
        if ended:
            for g in range(G0, ng):
                groups[g]["mode"] = 0
            break
        nready = min(ready_prefix(G0), 64, ng - G0)
        assert nready >= 1
        # fast path over the ready prefix: accept while every group is entered at
        # its summary start (or spanned) and self-consistent
        accepted = 0
        for lane in range(nready):
            q = groups[G0 + lane]
            ghi = min(min(GRP_TILES * (G0 + lane + 1), ntiles) * T, bl)
            has = q["S"] != NOSTART
            okl = q["ok"] and (q["S"] == e if has else e >= ghi)
            if not okl:
                break
            q["base"], q["mode"] = total, (1 if has else 0)
            if has:
                total += q["CNT"]
                e = q["X"]
                if q["term"]:
                    ended = True
            accepted += 1
            if ended:
                break
        G0 += accepted
        if ended or accepted == nready:
            continue
        # group G0, exactly: tile by tile with re-walks (B2 repair)
        g = G0
        G0 += 1
        q = groups[g]
        q["mode"] = 2
        gt0 = GRP_TILES * g
        for t in range(gt0, min(gt0 + GRP_TILES, ntiles)):
            tl = tiles[t]
            lo, hi = t * T, min((t + 1) * T, bl)
            if ended:
                tl.e = M64
                continue
            if e >= hi:  # spanned by the running frame
                tl.e = M64
                continue
            if tl.s != e:  # the pick disagrees with the true entry: re-walk
                lst, lcs, x = walk(blob, e, hi)
                tl.lst, tl.lcs, tl.x, tl.s = lst, lcs, x, e
                tl.rewalked = True
            tl.e = e
            tl.base = total
            total += len(tl.lst)
            e = tl.x
            if (e & STOP) or e >= bl:
                ended = True
    return total, e


# --------------------------------------------------- deferred work and the checksum
def deferred(blob, h, tiles, groups, t, T, fpos, cs, bsums, counts, verify, first_bad):
    bl = len(blob)
    tl = tiles[t]
    q = groups[t // GRP_TILES]
    if q["mode"] == 1:
        if tl.pre == NOTLIVE:
            return
        base = q["base"] + tl.pre
    elif q["mode"] == 2:
        if tl.e == M64:
            return
        base = tl.base
    else:
        return
    cnt = len(tl.lst)
    if verify:
        bad = hash_list(blob, tl.lst, tl.x) if tl.rewalked else tl.bad
        if bad is not None:
            first_bad.append(base + bad)
    for k in range(cnt):
        fpos[base + k] = tl.lst[k]
        cs[base + k] = tl.lcs[k]
    if not verify:
        return

    def add(m, v):
        b, j = m // 128, m & 7
        sec = sw(((m >> 3) & 15) + j)
        bsums.setdefault(b, [0] * 8)
        bsums[b][j] = (bsums[b][j] + mul32x32(v ^ sec)) & M64
        bsums[b][j ^ 1] = (bsums[b][j ^ 1] + v) & M64
        counts[b] = counts.get(b, 0) + 1

    if base == 0 and cnt:  # words 0..5: header fields, count | lo32(cs_0)
        w = [h["partition_id"], h["base_offset"], h["base_timestamp"], h["origin_timestamp"], h["batch_length"],
             h["message_count"] | ((tl.lcs[0] & 0xFFFFFFFF) << 32)]
        for m in range(6):
            add(m, w[m])
    x = tl.x
    nxt = u64(blob, x) if (not (x & STOP) and x + 8 <= bl) else None
    for k in range(cnt):
        n2 = tl.lcs[k + 1] if k + 1 < cnt else nxt
        if n2 is None:
            continue  # the record's last frame: its word is the partial final one
        add(base + k + 6, (tl.lcs[k] >> 32) | ((n2 & 0xFFFFFFFF) << 32))


def finish_checksum(h, cs, nwalk, bsums, counts):
    n = 44 + 8 * nwalk
    if n <= 240:
        from oracle import oracle as O
        b = struct.pack("<QQQQQI", h["partition_id"], h["base_offset"], h["base_timestamp"], h["origin_timestamp"],
                        h["batch_length"], h["message_count"]) + b"".join(struct.pack("<Q", cs[i]) for i in range(nwalk))
        return O.xxh3_64(b)
    nb = (n - 1) // 1024
    ns = ((n - 1) - 1024 * nb) // 64
    Mreg = 8 * (16 * nb + ns)
    acc = list(ACC_INIT)
    for b in range(nb):  # the chain: only blocks the deferred work completed
        assert counts.get(b, 0) == 128, (b, counts.get(b))
        for j in range(8):
            acc[j] = scramble((acc[j] + bsums[b][j]) & M64, j)

    def word(m):
        if m < 5:
            return [h["partition_id"], h["base_offset"], h["base_timestamp"], h["origin_timestamp"],
                    h["batch_length"]][m]
        if m == 5:
            return h["message_count"] | ((cs[0] & 0xFFFFFFFF) << 32)
        return (cs[m - 6] >> 32) | ((cs[m - 5] & 0xFFFFFFFF) << 32)

    for m in range(128 * nb, Mreg):  # the partial block, recomputed by the finisher
        v, j = word(m), m & 7
        acc[j] = (acc[j] + mul32x32(v ^ sw(((m >> 3) & 15) + j))) & M64
        acc[j ^ 1] = (acc[j ^ 1] + v) & M64
    for j in range(8):  # the last stripe: the last 8 stored checksums
        v = cs[nwalk - 8 + j]
        acc[j ^ 1] = (acc[j ^ 1] + v) & M64
        acc[j] = (acc[j] + mul32x32(v ^ s_at(121 + 8 * j))) & M64
    r = (n * P64_1) & M64
    for i in range(4):
        r = (r + fold64(acc[2 * i] ^ s_at(11 + 16 * i), acc[2 * i + 1] ^ s_at(11 + 16 * i + 8))) & M64
    return avalanche(r)


def decode(body: bytes, verify: bool = True, T: int = 4096, seed: int = 0, adversarial_picks: bool = False,
           starve: bool = False):
    """-> (kind, reason, frame positions, computed checksum, (a, b, c)) for a record
    that the uniform-stride speculation handed over (header already valid)."""
    rng = random.Random(seed)
    h = dict(zip(["partition_id", "base_offset", "base_timestamp", "origin_timestamp", "batch_length",
                  "batch_checksum"], struct.unpack_from("<6Q", body, 0)))
    h["message_count"] = u32(body, 48)
    blob = bytes(body[HDR:h["batch_length"]])
    bl = len(blob)
    ntiles = (bl + T - 1) // T
    ng = (ntiles + GRP_TILES - 1) // GRP_TILES
    order = list(range(ntiles))
    rng.shuffle(order)  # tiles finish in any order
    tiles = [None] * ntiles
    done_in_group = [0] * ng
    groups = [None] * ng
    ready = [False] * ng
    pick_rng = rng if adversarial_picks else None
    for t in order:
        tiles[t] = process_tile(blob, t, T, pick_rng, verify)
        g = t // GRP_TILES
        done_in_group[g] += 1
        if done_in_group[g] == min(GRP_TILES, ntiles - GRP_TILES * g):  # the group's last tile summarises it
            groups[g] = group_summary(tiles, g, ntiles, T, bl)
            ready[g] = True

    def ready_prefix(G0):
        n = 0
        while G0 + n < ng and ready[G0 + n]:
            n += 1
        return max(1, rng.randint(1, n)) if starve else n

    nwalk, end = link(blob, tiles, groups, ntiles, T, ready_prefix)
    fpos, cs = [0] * nwalk, [0] * nwalk
    bsums, counts, first_bad = {}, {}, []
    order = list(range(ntiles))
    rng.shuffle(order)  # deferred work in any order
    for t in order:
        deferred(blob, h, tiles, groups, t, T, fpos, cs, bsums, counts, verify, first_bad)
    computed = finish_checksum(h, cs, nwalk, bsums, counts) if verify else 0
    walk_end = end & ~STOP
    if verify and first_bad:
        from oracle import oracle as O
        i = min(first_bad)
        p = fpos[i]
        L = 40 + u32(blob, p + 36) + u32(blob, p + 32)
        return MSG_CS, 0, fpos, computed, (cs[i], O.xxh3_64(blob[p + 8:p + 8 + L]),
                                           min(M64, h["base_offset"] + u32(blob, p + 24)))
    if nwalk != h["message_count"] or (end & STOP) or end != bl:
        return VALIDATION, V_FRAMES_DO_NOT_TILE, fpos, computed, (0, 0, 0)
    if verify and computed != h["batch_checksum"]:
        return BATCH_CS, 0, fpos, computed, (h["batch_checksum"], computed, h["base_offset"])
    del walk_end
    return OK, 0, fpos, computed, (0, 0, 0)
