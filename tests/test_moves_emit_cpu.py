"""The move-table emit's algorithms (csrc/cpd_kernels.hip rle_moves4 — packed
nibbles —, rle_moves<FMB> — per column —, the one-row chunk emit that the
seam repair runs and, since round 6, rle_emit8 — eight rows per lane word),
restated step for step in Python
(wave = 64 lanes x 32 columns, tiles walked right to left, look-ahead carry)
and checked on CPU against the greedy RLE rule expanded per column, on random
first-move rows with short runs, long runs and a single run.  The GPU suite
then checks the kernels themselves bit-exact against the oracle."""
import random



def greedy_moves(fm):
    n = len(fm); S = 0xF; runs = []; h = 0
    for c in range(n):
        f = fm[c]; T = S & f
        if T == 0:
            runs.append((h, (S & -S).bit_length() - 1)); h = c; S = f
        else:
            S = T
    runs.append((h, (S & -S).bit_length() - 1))
    mv = [0] * n; ri = 0
    for c in range(n):
        while ri + 1 < len(runs) and runs[ri + 1][0] <= c: ri += 1
        mv[c] = runs[ri][1]
    return mv, runs

def states(fm):  # entry set per 32-col segment, runs ending (breaks) per segment
    S = 0xF; st = []; rc = []
    for s0 in range(0, len(fm), 32):
        st.append(S); cnt = 0
        for c in range(s0, s0 + 32):
            T = S & fm[c]
            if T == 0: cnt += 1; S = fm[c]
            else: S = T
        rc.append(cnt)
    return st, rc

M32 = 0xFFFFFFFF
def alignbit(hi, lo, sh): return ((hi << 32 | lo) >> sh) & M32
def ctz(x): return (x & -x).bit_length() - 1

def seg4_scan(v, Sin):
    Sw = [0, 0, 0, 0]; S = Sin
    for k in range(32):
        f = (v[k >> 3] >> (4 * (k & 7))) & 0xF; T = S & f; S = T if T else f
        Sw[k >> 3] |= S << (4 * (k & 7))
    P = [((Sw[0] << 4) | Sin) & M32, alignbit(Sw[1], Sw[0], 28), alignbit(Sw[2], Sw[1], 28), alignbit(Sw[3], Sw[2], 28)]
    Z = []
    for i in range(4):
        a = P[i] & v[i]
        Z.append((~((((a & 0x77777777) + 0x77777777) & M32) | a)) & 0x88888888 & M32)
    return Sw, P, Z

def nib(w, i): return (w[i >> 3] >> (4 * (i & 7))) & 0xF

def entry_set(P, Z):
    if Z[0]: b0 = ctz(Z[0]) >> 2
    elif Z[1]: b0 = 8 + (ctz(Z[1]) >> 2)
    elif Z[2]: b0 = 16 + (ctz(Z[2]) >> 2)
    else: b0 = 24 + (ctz(Z[3] | 0x80000000) >> 2)
    return nib(P, b0)

def moves4(fm, st, rc, KT=16):
    npad = len(fm); nseg = npad // 32; ntiles = npad // 2048
    vseg = []
    for s in range(nseg):
        w = [0, 0, 0, 0]
        for k in range(32): w[k >> 3] |= fm[s * 32 + k] << (4 * (k & 7))
        vseg.append(w)
    out = [0] * npad
    for t0 in range(0, ntiles, KT):
        t1 = min(ntiles, t0 + KT)
        have = False; carry = 0; s0 = t1 * 64
        while s0 < nseg and not have:
            m = [l for l in range(64) if s0 + l < nseg and rc[s0 + l] != 0]
            if m:
                sj = s0 + m[0]; Sw, P, Z = seg4_scan(vseg[sj], st[sj]); carry = entry_set(P, Z); have = True
            s0 += 64
        if not have:
            Sw, P, Z = seg4_scan(vseg[nseg - 1], st[nseg - 1]); carry = Sw[3] >> 28
        for t in range(t1 - 1, t0 - 1, -1):
            lanes = [seg4_scan(vseg[t * 64 + l], st[t * 64 + l]) for l in range(64)]
            anyl = [any(z for z in L[2]) for L in lanes]
            fl = [entry_set(L[1], L[2]) for L in lanes]
            for l in range(64):
                Sw, P, Z = lanes[l]
                right = [j for j in range(l + 1, 64) if anyl[j]]
                tail = fl[right[0]] if right else carry
                nz = [(Z[i] | ((Z[i] - (Z[i] >> 3)) & M32)) & M32 for i in range(4)]
                V = [alignbit(nz[1], nz[0], 4), alignbit(nz[2], nz[1], 4), alignbit(nz[3], nz[2], 4), ((nz[3] >> 4) | 0xF0000000)]
                X = [Sw[0], Sw[1], Sw[2], (Sw[3] & 0x0FFFFFFF) | (tail << 28)]
                for sh in (4, 8, 16):
                    xs = [alignbit(X[i + 1], X[i], sh) for i in range(3)] + [X[3] >> sh]
                    vs = [alignbit(V[i + 1], V[i], sh) for i in range(3)] + [V[3] >> sh]
                    for i in range(4):
                        X[i] = (V[i] & X[i]) | (~V[i] & xs[i] & M32); V[i] |= vs[i]
                for w in (1, 2):
                    xs = [X[i + w] if i + w < 4 else 0 for i in range(4)]
                    vs = [V[i + w] if i + w < 4 else 0 for i in range(4)]
                    for i in range(4):
                        X[i] = (V[i] & X[i]) | (~V[i] & xs[i] & M32); V[i] |= vs[i]
                for i in range(4):
                    b0 = ~X[i] & 0x11111111; b1 = ~(X[i] >> 1) & b0; b2 = ~(X[i] >> 2) & b1
                    o = (b0 + b1 + b2) & M32
                    for k in range(8): out[(t * 64 + l) * 32 + i * 8 + k] = (o >> (4 * k)) & 0xF
            if any(anyl): carry = fl[anyl.index(True)]
    return out

# generic (per-column) kernel emulation for wide sets
def greedy_moves_w(fm, ALL):
    n = len(fm); S = ALL; runs = []; h = 0
    for c in range(n):
        f = fm[c]; T = S & f
        if T == 0:
            runs.append((h, ctz(S))); h = c; S = f
        else: S = T
    runs.append((h, ctz(S)))
    mv = [0] * n; ri = 0
    for c in range(n):
        while ri + 1 < len(runs) and runs[ri + 1][0] <= c: ri += 1
        mv[c] = runs[ri][1]
    return mv

def states_w(fm, ALL):
    S = ALL; st = []; rc = []
    for s0 in range(0, len(fm), 32):
        st.append(S); cnt = 0
        for c in range(s0, s0 + 32):
            T = S & fm[c]
            if T == 0: cnt += 1; S = fm[c]
            else: S = T
        rc.append(cnt)
    return st, rc

def low_bit(S): return ctz(S | 0x8000)

def seg_moves(f32, S):
    brk = 0; L = [0, 0, 0, 0]
    for k in range(32):
        f = f32[k]; T = S & f; b = T == 0
        brk |= (1 if b else 0) << k
        S = f if b else T
        L[k >> 3] |= low_bit(S) << (4 * (k & 7))
    return brk, L, S

def entry_move(brk, L, Sin):
    b0 = ctz(brk | 0x80000000)
    return low_bit(Sin) if b0 == 0 else nib(L, b0 - 1)

def moves_generic(fm, st, rc, KT=16):
    npad = len(fm); nseg = npad // 32; ntiles = npad // 2048
    out = [0] * npad
    for t0 in range(0, ntiles, KT):
        t1 = min(ntiles, t0 + KT)
        have = False; carry = 0; s0 = t1 * 64
        while s0 < nseg and not have:
            m = [l for l in range(64) if s0 + l < nseg and rc[s0 + l] != 0]
            if m:
                sj = s0 + m[0]; brk, L, _ = seg_moves(fm[sj*32:sj*32+32], st[sj]); carry = entry_move(brk, L, st[sj]); have = True
            s0 += 64
        if not have:
            _, _, S = seg_moves(fm[(nseg-1)*32:nseg*32], st[nseg - 1]); carry = low_bit(S)
        for t in range(t1 - 1, t0 - 1, -1):
            R = [seg_moves(fm[(t*64+l)*32:(t*64+l)*32+32], st[t*64+l]) for l in range(64)]
            fl = [entry_move(R[l][0], R[l][1], st[t*64+l]) for l in range(64)]
            anyl = [R[l][0] != 0 for l in range(64)]
            for l in range(64):
                brk, L, _ = R[l]
                right = [j for j in range(l + 1, 64) if anyl[j]]
                mv = fl[right[0]] if right else carry
                for k in range(31, -1, -1):
                    out[(t*64+l)*32 + k] = mv
                    if k > 0 and (brk >> k) & 1: mv = nib(L, k - 1)
            if any(anyl): carry = fl[anyl.index(True)]
    return out



def _rows(FMB, kinds, npads, seed):
    rnd = random.Random(seed)
    ALL = (1 << FMB) - 1
    for kind in kinds:
        npad = rnd.choice(npads)
        fm = []
        for _ in range(npad):
            if kind == 0:
                f = rnd.choice([1, 2, 4, 8, 3, 5, 6, 0xF]) if FMB == 4 else 1 << rnd.randint(0, FMB - 2)
            elif kind == 1:
                f = rnd.choice([ALL] * 30 + [1, 2])
            elif kind == 2:
                f = ALL
            else:
                f = rnd.randint(1, ALL)
            fm.append(f)
        yield fm


def test_swar_emit_matches_greedy():
    for i, fm in enumerate(_rows(4, [0, 1, 2, 3, 0, 3], [2048, 4096, 6144], 1)):
        mv, _ = greedy_moves(fm)
        st, rc = states(fm)
        assert moves4(fm, st, rc, KT=[1, 2, 16][i % 3]) == mv


def test_generic_emit_matches_greedy():
    for FMB in (4, 8, 16):
        ALL = (1 << FMB) - 1
        for i, fm in enumerate(_rows(FMB, [0, 1, 3], [2048, 4096], FMB)):
            mv = greedy_moves_w(fm, ALL)
            st, rc = states_w(fm, ALL)
            assert moves_generic(fm, st, rc, KT=[1, 16][i % 2]) == mv


# The table-width conversions of cpd_kernels.hip (nib_to2 / nib_to1 /
# nib_from2 / nib_from1, store_cols32 / load_cols32), restated bit for bit.
M32 = 0xFFFFFFFF


def nib_to2(x):
    x &= 0x33333333
    x = (x | (x >> 2)) & 0x0F0F0F0F
    x = (x | (x >> 4)) & 0x00FF00FF
    return (x | (x >> 8)) & 0x0000FFFF


def nib_to1(x):
    x &= 0x11111111
    x = (x | (x >> 3)) & 0x03030303
    x = (x | (x >> 6)) & 0x000F000F
    return (x | (x >> 12)) & 0x000000FF


def nib_from2(y):
    y &= 0xFFFF
    y = (y | (y << 8)) & 0x00FF00FF
    y = (y | (y << 4)) & 0x0F0F0F0F
    return (y | (y << 2)) & 0x33333333


def nib_from1(y):
    y &= 0xFF
    y = (y | (y << 12)) & 0x000F000F
    y = (y | (y << 6)) & 0x03030303
    return (y | (y << 3)) & 0x11111111


def test_table_width_conversions():
    """8 moves in nibbles <-> 2-bit / 1-bit fields: column k of the nibble
    word lands in field k of the narrow value and back, for every move
    pattern that fits (exhaustive for 1 bit, random for 2)."""
    rnd = random.Random(5)
    for bits, to, frm, cases in ((2, nib_to2, nib_from2, [rnd.getrandbits(16) for _ in range(4000)]),
                                 (1, nib_to1, nib_from1, range(256))):
        for narrow in cases:
            mv = [(narrow >> (bits * k)) & ((1 << bits) - 1) for k in range(8)]
            nib = sum(m << (4 * k) for k, m in enumerate(mv))
            assert to(nib) == narrow, (bits, mv)
            assert frm(narrow) == nib, (bits, mv)


# The fused one-pass emit (cpd_kernels.hip rle_emit4 / emit_chunk4 /
# rle_emit_fix), restated: per chunk of KT tiles the segments' entry sets by
# the lanes' guesses and a fixed point, the closing set of the run open at
# the chunk's right edge by a prefix-AND look-ahead, the backward fill of
# moves4 from those entries; the chunk's own entry guessed from the 16
# columns left of it, and the seam check redoing a chunk from the true entry.
def _segments(fm):
    vseg = []
    for s in range(len(fm) // 32):
        w = [0, 0, 0, 0]
        for k in range(32):
            w[k >> 3] |= fm[s * 32 + k] << (4 * (k & 7))
        vseg.append(w)
    return vseg


def _scan_breaks(v, S):
    brk = 0
    for k in range(32):
        f = (v[k >> 3] >> (4 * (k & 7))) & 0xF
        T = S & f
        brk += T == 0
        S = T if T else f
    return S, brk


def _guess16(w2, w3):
    S = 0xF
    for k in range(16):
        f = ((w2 if k < 8 else w3) >> (4 * (k & 7))) & 0xF
        T = S & f
        S = T if T else f
    return S


def _fill_tile(vseg, t, ent, carry, out):
    """moves4's backward step for tile t from the lanes' entry sets."""
    lanes = [seg4_scan(vseg[t * 64 + l], ent[l]) for l in range(64)]
    anyl = [any(z for z in L[2]) for L in lanes]
    fl = [entry_set(L[1], L[2]) for L in lanes]
    for l in range(64):
        Sw, P, Z = lanes[l]
        right = [j for j in range(l + 1, 64) if anyl[j]]
        tail = fl[right[0]] if right else carry
        nz = [(Z[i] | ((Z[i] - (Z[i] >> 3)) & M32)) & M32 for i in range(4)]
        V = [alignbit(nz[1], nz[0], 4), alignbit(nz[2], nz[1], 4), alignbit(nz[3], nz[2], 4),
             ((nz[3] >> 4) | 0xF0000000)]
        X = [Sw[0], Sw[1], Sw[2], (Sw[3] & 0x0FFFFFFF) | (tail << 28)]
        for sh in (4, 8, 16):
            xs = [alignbit(X[i + 1], X[i], sh) for i in range(3)] + [X[3] >> sh]
            vs = [alignbit(V[i + 1], V[i], sh) for i in range(3)] + [V[3] >> sh]
            for i in range(4):
                X[i] = (V[i] & X[i]) | (~V[i] & xs[i] & M32); V[i] |= vs[i]
        for w in (1, 2):
            xs = [X[i + w] if i + w < 4 else 0 for i in range(4)]
            vs = [V[i + w] if i + w < 4 else 0 for i in range(4)]
            for i in range(4):
                X[i] = (V[i] & X[i]) | (~V[i] & xs[i] & M32); V[i] |= vs[i]
        for i in range(4):
            b0 = ~X[i] & 0x11111111; b1 = ~(X[i] >> 1) & b0; b2 = ~(X[i] >> 2) & b1
            o = (b0 + b1 + b2) & M32
            for k in range(8):
                out[(t * 64 + l) * 32 + i * 8 + k] = (o >> (4 * k)) & 0xF
    return fl[anyl.index(True)] if any(anyl) else carry


def _emit_chunk(vseg, ntiles, t0, t1, Sin, out):
    ents, breaks, carry = [], 0, Sin
    for t in range(t0, t1):  # forward: the lanes' entries, a fixed point
        v = [vseg[t * 64 + l] for l in range(64)]
        ins = [carry] + [_guess16(v[l - 1][2], v[l - 1][3]) for l in range(1, 64)]
        while True:
            outs = [_scan_breaks(v[l], ins[l]) for l in range(64)]
            pe = [carry] + [outs[l - 1][0] for l in range(1, 64)]
            if pe == ins:
                break
            ins = pe  # SIMT: every mismatching lane takes its predecessor's exit
        ents.append(ins)
        breaks += sum(b for _, b in outs)
        carry = outs[63][0]
    exit_s = carry
    P, close = exit_s, None  # ahead: prefix-AND over the segments right of the chunk
    for t in range(t1, ntiles):
        A = []
        for l in range(64):
            a = 0xF
            for k in range(32):
                a &= (vseg[t * 64 + l][k >> 3] >> (4 * (k & 7))) & 0xF
            A.append(a)
        excl = 0xF
        for l in range(64):
            Pl = P & excl
            if Pl & A[l] == 0:
                S = Pl
                for k in range(32):
                    T = S & ((vseg[t * 64 + l][k >> 3] >> (4 * (k & 7))) & 0xF)
                    if not T:
                        break
                    S = T
                close = S
                break
            excl &= A[l]
        if close is not None:
            break
        P &= excl
    if close is None:
        close = P
    carry = close
    for t in range(t1 - 1, t0 - 1, -1):  # backward
        carry = _fill_tile(vseg, t, ents[t - t0], carry, out)
    return exit_s, breaks


def fused4(fm, KT=16):
    vseg = _segments(fm)
    ntiles = len(fm) // 2048
    out = [0] * len(fm)
    chunks = []
    for t0 in range(0, ntiles, KT):
        t1 = min(ntiles, t0 + KT)
        sin = 0xF if t0 == 0 else _guess16(vseg[t0 * 64 - 1][2], vseg[t0 * 64 - 1][3])
        ex, br = _emit_chunk(vseg, ntiles, t0, t1, sin, out)
        chunks.append([sin, ex, br])
    redone, carry, total = 0, 0xF, 0  # the seam check, chunk by chunk
    for c, ck in enumerate(chunks):
        if ck[0] != carry:
            t0 = c * KT
            ex, br = _emit_chunk(vseg, ntiles, t0, min(ntiles, t0 + KT), carry, out)
            chunks[c] = [carry, ex, br]
            redone += 1
        total += chunks[c][2]
        carry = chunks[c][1]
    return out, total + 1, redone


def test_fused_emit_matches_greedy():
    """Tables and run counts of the one-pass emit equal the greedy rule's,
    over rows whose chunk guesses hold (short runs) and fail (long runs)."""
    redone = 0
    # a run over the whole row whose set is fixed by its first column: every
    # chunk's guess (16 wildcard columns) differs from the true set
    crafted = [[1] + [0xF] * 6143, [2, 3] + [0xF] * 4094 + [4] + [0xF] * 2047]
    for i, fm in enumerate(crafted + list(_rows(4, [0, 1, 2, 3, 1, 0], [2048, 4096, 6144], 3))):
        mv, runs = greedy_moves(fm)
        out, count, r = fused4(fm, KT=[1, 2, 16][i % 3])
        assert out == mv and count == len(runs)
        redone += r
    assert redone > 0  # the seam check redid at least one chunk


# The eight-row emit (cpd_kernels.hip rle_emit8, round 6), restated lane by
# lane: a lane holds one column of eight rows per word (nibble r = row r),
# the 8x8 nibble transposes that build those words from the row-group
# sectors, the SWAR greedy step, the lane guesses and fixed point, the
# look-ahead, the backward closing sets with the trailing run left empty,
# the suffix scan that closes it, and the per-(row, chunk) records that
# the seam check (emit_chunk4, restated above as _emit_chunk) repairs.
def _perm(s0, s1, sel):  # v_perm_b32: bytes 0-3 of s1, 4-7 of s0
    src = (s0 << 32) | s1
    return sum(((src >> (8 * ((sel >> (8 * i)) & 0xFF))) & 0xFF) << (8 * i) for i in range(4))


def tr8(a):
    a = list(a)
    for r in range(4):
        x, y = a[r], a[r + 4]
        a[r], a[r + 4] = _perm(y, x, 0x05040100), _perm(y, x, 0x07060302)
    for r in (0, 1, 4, 5):
        x, y = a[r], a[r + 2]
        a[r], a[r + 2] = _perm(y, x, 0x06020400), _perm(y, x, 0x07030501)
    for r in (0, 2, 4, 6):
        x, y = a[r], a[r + 1]
        a[r] = (x & 0x0F0F0F0F) | ((y << 4) & 0xF0F0F0F0)
        a[r + 1] = ((x >> 4) & 0x0F0F0F0F) | (y & 0xF0F0F0F0)
    return a


def zero_nib(a):
    return ~((((a & 0x77777777) + 0x77777777) & M32) | a) & 0x88888888


def nib_mask(z):
    return (z | ((z - (z >> 3)) & M32)) & M32


def step8(S, F):
    T = S & F
    return T | (F & nib_mask(zero_nib(T)))


def low_bits8(X):
    b0 = ~X & 0x11111111
    b1 = ~(X >> 1) & b0
    b2 = ~(X >> 2) & b1
    return (b0 + b1 + b2) & M32


def test_tr8_transposes():
    rnd = random.Random(9)
    for _ in range(200):
        m = [[rnd.randrange(16) for _ in range(8)] for _ in range(8)]
        a = [sum(m[r][k] << (4 * k) for k in range(8)) for r in range(8)]
        b = tr8(a)
        assert all((b[k] >> (4 * r)) & 0xF == m[r][k] for r in range(8) for k in range(8))


def emit8(rows, W=32):
    """Eight rows' moves and chunk records as rle_emit8 computes them (chunks
    of 64 lanes x W columns), then rle_emit_fix's seam check per row."""
    npad = len(rows[0])
    CH = 64 * W
    # the column words, built from the rows' 8-column nibble words by tr8
    F = [0] * npad
    for g in range(npad // 8):
        a = [sum(rows[r][g * 8 + k] << (4 * k) for k in range(8)) for r in range(8)]
        for k, wd in enumerate(tr8(a)):
            F[g * 8 + k] = wd
    out = [[0] * npad for _ in range(8)]
    recs = [[] for _ in range(8)]  # per row: [guessed entry, exit, breaks] per chunk
    for c0 in range(0, npad, CH):
        last = min(63, (npad - c0) // W - 1)
        ins = []
        for L in range(64):
            cl = c0 + L * W
            S = 0xFFFFFFFF
            if 0 < cl < npad:  # the 16 columns before the lane, from a wildcard
                S = F[cl - 16]
                for c in range(cl - 15, cl):
                    S = step8(S, F[c])
            ins.append(S)
        guess0 = ins[0]
        while True:  # forward, until every entry is the left neighbour's exit
            runs = []
            for L in range(64):
                S, col = ins[L], []
                for c in range(W):
                    cc = c0 + L * W + c
                    S = step8(S, F[cc] if cc < npad else 0xFFFFFFFF)
                    col.append(S)
                runs.append(col)
            pe = [ins[0]] + [runs[L - 1][-1] for L in range(1, 64)]
            fix = [c0 + L * W < npad and pe[L] != ins[L] for L in range(64)]
            if not any(fix):
                break
            ins = [pe[L] if fix[L] else ins[L] for L in range(64)]
        E = runs[last][-1]
        A, opn, P = 0, M32, E  # ahead
        cb = c0 + (last + 1) * W
        while cb < npad and opn:
            w = [F[cb + l] if cb + l < npad else 0xFFFFFFFF for l in range(64)]
            incl, acc = [], M32
            for l in range(64):
                acc &= w[l]
                incl.append(acc)
            Rs = [P & incl[l] for l in range(64)]
            z = [zero_nib(Rs[l]) & opn for l in range(64)]
            got = res = 0
            for l in range(64):
                zp, Rp = (0, P) if l == 0 else (z[l - 1], Rs[l - 1])
                first = z[l] & ~zp & M32
                got |= Rp & nib_mask(first)
                res |= first
            A |= got
            opn &= ~nib_mask(res) & M32
            P = Rs[63]
            cb += 64
        A |= P & opn
        X, Wl, cnt = [], [], [[0] * 8 for _ in range(64)]
        for L in range(64):  # backward: closing sets, the trailing run left 0
            col, Sn, x = [0] * W, runs[L][W - 1], 0
            for c in range(W - 2, -1, -1):
                Sc = runs[L][c]
                z = zero_nib(Sc & Sn)
                m = nib_mask(z)
                x = (Sc & m) | (x & ~m & M32)
                col[c] = x
                for r in range(8):
                    cnt[L][r] += (z >> (4 * r + 3)) & 1
                Sn = Sc
            z0 = zero_nib(ins[L] & Sn)
            for r in range(8):
                cnt[L][r] += (z0 >> (4 * r + 3)) & 1
            m0 = nib_mask(z0)
            Wl.append((ins[L] & m0) | (col[0] & ~m0 & M32))
            X.append(col)
        for d in (1, 2, 4, 8, 16, 32):  # tails: the first closing set to the right
            y = [Wl[L + d] if L + d < 64 else A for L in range(64)]
            Wl = [Wl[L] | (nib_mask(zero_nib(Wl[L])) & y[L]) for L in range(64)]
        tail = [Wl[L + 1] if L < 63 else A for L in range(64)]
        for c in range(W - 1, -1, -1):  # the trailing runs, right to left
            z = [zero_nib(X[L][c]) for L in range(64)]
            if not any(z):
                break
            for L in range(64):
                X[L][c] |= nib_mask(z[L]) & tail[L]
        for L in range(64):
            for c in range(W):
                cc = c0 + L * W + c
                if cc < npad:
                    mv = low_bits8(X[L][c])
                    for r in range(8):
                        out[r][cc] = (mv >> (4 * r)) & 0xF
        for r in range(8):
            recs[r].append([(guess0 >> (4 * r)) & 0xF, (E >> (4 * r)) & 0xF,
                            sum(cnt[L][r] for L in range(64))])
    counts, redone, KT = [], 0, W // 32
    for r in range(8):  # the seam check, a row at a time (one-row redo)
        vseg, ntiles = _segments(rows[r]), npad // 2048
        carry, total = 0xF, 0
        for c, ck in enumerate(recs[r]):
            if ck[0] != carry:
                t0 = c * KT
                ex, br = _emit_chunk(vseg, ntiles, t0, min(ntiles, t0 + KT), carry, out[r])
                recs[r][c] = [carry, ex, br]
                redone += 1
            total += recs[r][c][2]
            carry = recs[r][c][1]
        counts.append(total + 1)
    return out, counts, redone


def test_eight_row_emit_matches_greedy():
    """Tables and run counts of the eight-row emit equal the greedy rule's for
    every row, at both lane widths, over short runs, long runs, a row that is
    one run and rows whose chunk guesses fail (seam repairs)."""
    rnd = random.Random(11)
    redone = 0
    for W, npad in ((32, 4096), (64, 4096), (32, 6144)):
        gen = list(_rows(4, [0, 1, 3, 0, 1, 2, 3, 0], [npad], rnd.randrange(1000)))
        rows = [fm[:npad] + [0xF] * (npad - len(fm)) for fm in gen]
        rows[2] = [1] + [0xF] * (npad - 1)  # one run whose set the first column fixes
        rows[5] = [2, 3] + [0xF] * (npad // 2 - 2) + [4] + [0xF] * (npad // 2 - 1)
        out, counts, r = emit8(rows, W)
        redone += r
        for i in range(8):
            mv, runs = greedy_moves(rows[i])
            assert out[i] == mv, (W, npad, i)
            assert counts[i] == len(runs), (W, npad, i)
    assert redone > 0  # crafted long runs force seam repairs
