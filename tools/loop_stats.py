"""Instruction mix of a kernel's loops from a hipcc -save-temps gfx950 .s file: for each backward branch (a loop),
the counts of MFMA, VALU (incl. packed), SALU, LDS, buffer / global memory, waitcnt and barrier instructions in
its body -- what the SIMD has to issue per iteration beside the matrix cores.
Usage: python tools/loop_stats.py <file.s> <kernel-name-regex>"""
import re
import sys


def classify(op):
    if op.startswith('v_mfma'):
        return 'mfma'
    if op.startswith('v_pk_'):
        return 'valu_pk'
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('s_waitcnt'):
        return 'waitcnt'
    if op.startswith('s_barrier'):
        return 'barrier'
    if op.startswith(('s_cbranch', 's_branch')):
        return 'branch'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('buffer_', 'global_')):
        return 'vmem'
    return 'other'


def main():
    s = open(sys.argv[1]).read()
    pat = re.compile(sys.argv[2])
    for m in re.finditer(r'^(\S+):\s*(;.*)?$', s, re.M):
        name = m.group(1)
        if not name.startswith('_Z') or not pat.search(name):
            continue
        body = s[m.end():s.find('.Lfunc_end', m.end())]
        lines = body.split('\n')
        labels = {}
        ins = []                                   # (line index, op, text)
        for i, ln in enumerate(lines):
            t = ln.strip()
            lm = re.match(r'^(\.LBB\S+):', t)
            if lm:
                labels[lm.group(1)] = len(ins)
                continue
            if t and not t.startswith(('.', ';')):
                ins.append((i, t.split()[0], t))
        print(name[:110], f'({len(ins)} instructions)')
        for k, (_, op, t) in enumerate(ins):
            if op.startswith('s_cbranch') or op == 's_branch':
                tgt = t.split()[-1]
                if tgt in labels and labels[tgt] <= k:
                    seg = ins[labels[tgt]:k + 1]
                    cnt = {}
                    for _, o, _ in seg:
                        c = classify(o)
                        cnt[c] = cnt.get(c, 0) + 1
                    print(f'  loop {tgt} ({len(seg)} instr): ' + ', '.join(f'{c} {n}' for c, n in sorted(cnt.items())))


if __name__ == '__main__':
    main()
