"""Instruction mix of a kernel's main loop from gfx950 assembly (hipcc --save-temps):
the backward branch spanning the most MFMAs.  usage: python tools/isa_loop.py <file.s> <symbol-substring>..."""
import collections
import re
import sys


def analyze(L, sym):
    st = [i for i, l in enumerate(L) if l.startswith(sym) and re.match(r'^[\w.$]+:', l)]
    if not st:
        print("no symbol", sym)
        return
    st = st[0]
    en = next(i for i in range(st, len(L)) if 's_endpgm' in L[i])
    body = L[st:en]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r'^(\.LBB\d+_\d+):', l)
        if m:
            labels[m.group(1)] = i
    best = None
    for i, l in enumerate(body):
        m = re.search(r's_c?branch\w* (\.LBB\d+_\d+)', l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            a = labels[m.group(1)]
            n = sum(1 for x in body[a:i] if 'v_mfma' in x)
            if best is None or (n, i - a) > (best[0], best[2] - best[1]):
                best = (n, a, i)
    n, a, b = best
    c = collections.Counter()
    for l in body[a:b + 1]:
        t = l.strip()
        if not t or t.startswith(('.', ';')):
            continue
        op = t.split()[0]
        if op.startswith('v_mfma'):
            k = 'mfma'
        elif 'dot2' in op:
            k = 'v_dot2'
        elif op.startswith('ds_read'):
            k = 'ds_read'
        elif op.startswith('ds_'):
            k = 'ds_other'
        elif op.startswith('buffer_load') and 'lds' in t:
            k = 'lds_dma'
        elif op.startswith(('buffer_', 'global_')):
            k = 'vmem'
        elif op.startswith('s_waitcnt'):
            k = 'waitcnt'
        elif op.startswith('s_barrier'):
            k = 'barrier'
        elif op.startswith('s_'):
            k = 'salu'
        elif op.startswith('v_'):
            k = 'valu'
        else:
            k = op
        c[k] += 1
    print(f"{sym[-50:]}: loop of {b - a} lines: " + ", ".join(f"{k} {v}" for k, v in sorted(c.items(), key=lambda x: -x[1])))


if __name__ == "__main__":
    L = open(sys.argv[1]).read().split('\n')
    for s in sys.argv[2:]:
        analyze(L, s)
