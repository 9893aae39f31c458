"""Scan a kernel's gfx950 assembly for instructions that touch a register an inline-asm buffer load
is still writing (issued, not yet covered by an s_waitcnt vmcnt).  A linear scan: it follows the
instruction order of the file, not the control flow, so a hit at a loop head may be a false alarm;
a clean scan is what the P16 weight-gradient kernel must show."""
import re
import sys


def regs(tok):
    m = re.match(r'v\[(\d+):(\d+)\]', tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'v(\d+)$', tok)
    return {int(m.group(1))} if m else set()


def scan(asm, name):
    i = asm.index(name + ':')
    j = asm.index('.Lfunc_end', i)
    pending, hits = [], []
    for l in asm[i:j].split('\n'):
        l = l.strip()
        if not l or l.startswith((';', '.')):
            continue
        ops = l.replace(',', ' ').split()
        if ops[0].startswith('buffer_load'):
            pending.append(regs(ops[1]))
            continue
        if ops[0] == 's_waitcnt' and 'vmcnt' in l:
            n = int(re.search(r'vmcnt\((\d+)\)', l).group(1))
            pending = pending[len(pending) - n:] if n < len(pending) else pending
            if n == 0:
                pending = []
            continue
        if ops[0].startswith('s_') or ops[0].endswith(':'):
            continue
        live = set().union(*pending) if pending else set()
        if any(regs(t) & live for t in ops[1:]):
            hits.append(l)
    return hits


if __name__ == '__main__':
    asm = open(sys.argv[1]).read()
    bad = 0
    for name in re.findall(r'^(_ZN4niti16wgrad_p16_kernel\w+):', asm, flags=re.M):
        h = scan(asm, name)
        print(name, len(h), h[:3])
        bad += len(h)
    sys.exit(1 if bad else 0)
