"""Test-side interpreter of a PARTIAL blob (DGREP_DFA_PARTIAL, include/dgrep_blob.h).

A line runs on the blob's first DFA states; if it reaches CAND (the last
state) it is decided by the blob's NFA program instead -- the contract the GPU
filter stepper + verify_nfa_kernel implement. Used to check the compiler's
partial output against the oracle on the CPU, before any GPU run.
"""
import numpy as np


class NfaProgram:
    def __init__(self, words: np.ndarray):
        g = [int(x) for x in words]
        magic, self.npos, self.nw, self.nrc, self.nnodes, self.nctx, self.fffd, self.has_word = g[:8]
        assert magic == 0x3141464E, hex(magic)
        nw, nctx = self.nw, self.nctx
        at = 8

        def take(n):
            nonlocal at
            v = g[at:at + n]
            at += n
            return v

        child = take(self.nnodes * 256)
        self.child = [[(x - (1 << 32)) if x >= (1 << 31) else x for x in child[i * 256:(i + 1) * 256]]
                      for i in range(self.nnodes)]
        self.depth = take(self.nnodes)
        self.word = take(self.nrc)

        def bitset(v):
            return sum(w << (32 * i) for i, w in enumerate(v))

        has = take(self.nrc * nw)
        self.has = [bitset(has[c * nw:(c + 1) * nw]) for c in range(self.nrc)]
        init = take(2 * nctx * nw)
        self.init = [[bitset(init[(b * nctx + x) * nw:(b * nctx + x + 1) * nw]) for x in range(nctx)] for b in range(2)]
        im = take(2 * nctx)
        self.init_m = [[im[b * nctx + x] for x in range(nctx)] for b in range(2)]
        cl = take(self.npos * nctx * nw)
        self.cl = [[bitset(cl[(p * nctx + x) * nw:(p * nctx + x + 1) * nw]) for x in range(nctx)]
                   for p in range(self.npos)]
        mx = take(nctx * nw)
        self.mx = [bitset(mx[x * nw:(x + 1) * nw]) for x in range(nctx)]
        ei = take(4)
        self.end_init = [[ei[b * 2 + pw] for pw in range(2)] for b in range(2)]
        ex = take(2 * nw)
        self.end_x = [bitset(ex[pw * nw:(pw + 1) * nw]) for pw in range(2)]
        assert at == len(g), (at, len(g))

    def match(self, line: bytes) -> bool:
        """regexp.Match(pattern, line) by the program (line without '\\n')."""
        P, begin, pw, node = 0, 1, 0, 0
        matched = False

        def rune(c):
            nonlocal P, begin, pw, matched
            nwf = self.word[c]
            ctx = (pw * 2 + nwf) if self.has_word else 0
            S = self.init[begin][ctx]
            m = self.init_m[begin][ctx] or (P & self.mx[ctx])
            x, bits = 0, P
            while bits:
                if bits & 1:
                    S |= self.cl[x][ctx]
                bits >>= 1
                x += 1
            if m:
                matched = True
                return
            P = S & self.has[c]
            begin = 0
            pw = nwf if self.has_word else 0

        for b in line:
            if matched:
                return True
            v = self.child[node][b]
            if node != 0 and v == -1:
                for _ in range(self.depth[node]):
                    if not matched:
                        rune(self.fffd)
                node = 0
                if matched:
                    return True
                v = self.child[0][b]
            if v <= -2:
                node = 0
                rune(-2 - v)
            elif v == -1:
                node = 0
                rune(self.fffd)
            else:
                node = v
        for _ in range(self.depth[node]):
            if not matched:
                rune(self.fffd)
        if matched:
            return True
        return bool(self.end_init[begin][pw] or (P & self.end_x[pw]))


def run_partial(cp, data: bytes):
    """(line_no, start, len) of the matching lines of `data` (strings.Split
    semantics) through the partial DFA + NFA program."""
    assert cp.partial
    bc, tr = cp.tables()
    prog = NfaProgram(cp.nfa_program())
    cand = cp.nstates - 1
    nl = int(bc[10])
    ln, st, le = [], [], []
    pos = 0
    for i, line in enumerate(data.split(b"\n")):
        s = cp.start
        for b in line:
            s = int(tr[s, bc[b]])
            if s == cand:
                break
        if prog.match(line) if s == cand else int(tr[s, nl]) == cp.start_m:
            ln.append(i + 1)
            st.append(pos)
            le.append(len(line))
        pos += len(line) + 1
    return np.array(ln, np.uint64), np.array(st, np.uint64), np.array(le, np.uint32)


def nfa_only(cp, data: bytes):
    """The same lines decided by the NFA program alone (every line a candidate)."""
    prog = NfaProgram(cp.nfa_program())
    ln, st, le = [], [], []
    pos = 0
    for i, line in enumerate(data.split(b"\n")):
        if prog.match(line):
            ln.append(i + 1)
            st.append(pos)
            le.append(len(line))
        pos += len(line) + 1
    return np.array(ln, np.uint64), np.array(st, np.uint64), np.array(le, np.uint32)
