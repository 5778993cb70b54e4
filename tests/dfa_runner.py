"""Test-side interpreter of a compiled DFA blob (include/dgrep_blob.h).

Runs the automaton over a split exactly as the GPU kernel's contract says:
restart at '\\n', a line matches iff the state after its '\\n' is start_m,
the last line (no '\\n') matches iff trans[s][class('\\n')] == start_m.
Used to check the pattern compiler against the oracle on the CPU.
"""
import numpy as np


def run_blob(cp, data: bytes):
    bc, tr = cp.tables()
    nl = int(bc[10])
    s = cp.start
    M = cp.start_m
    out_ln, out_st, out_le = [], [], []
    line = 1
    ls = 0
    for i, b in enumerate(data):
        s = int(tr[s, bc[b]])
        if b == 10:
            if s == M:
                out_ln.append(line)
                out_st.append(ls)
                out_le.append(i - ls)
            line += 1
            ls = i + 1
    if int(tr[s, nl]) == M:
        out_ln.append(line)
        out_st.append(ls)
        out_le.append(len(data) - ls)
    return (np.array(out_ln, np.uint64), np.array(out_st, np.uint64), np.array(out_le, np.uint32))


def match_line(cp, line: bytes) -> bool:
    """regexp.Match(pattern, line) through the DFA (line must not contain '\\n')."""
    assert b"\n" not in line
    ln, _, _ = run_blob(cp, line)
    return len(ln) == 1
