"""Scan gfx950 assembly for instructions that touch a register an inline-asm load is still writing.

Kernels with asm load rings (the P16 weight gradient's buffer_load ring, the GEMM / tap-sharing /
first-layer kernels' ds_read fragment rings) count their own waits: hipcc does not know when such
a load lands, and may hand the destination of a load whose result it believes dead (the last
look-ahead loads of a ring) to another value while the load is still in flight -- the fault found
in round 2.  The scan tracks every load in issue order: loads between hipcc's ;;#ASMSTART /
;;#ASMEND markers hold their destination registers until an s_waitcnt retires them (vmcnt for
buffer / global loads, lgkmcnt for ds_read, in order); compiler-issued loads only take a place in
the counters.  Any other instruction naming a held register is a hit.

A linear scan: it follows the instruction order of the file, not the control flow, so a hit at a
loop head may be a false alarm, and SMEM loads (which retire lgkmcnt out of order) are not
modelled.  A clean scan is what every asm-ring kernel must show.
"""
import re
import sys


def regs(tok):
    m = re.match(r'v\[(\d+):(\d+)\]', tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'v(\d+)$', tok)
    return {int(m.group(1))} if m else set()


def _retire(pending, l, counter):
    m = re.search(counter + r'\((\d+)\)', l)
    if not m:
        return pending
    n = int(m.group(1))
    return pending[len(pending) - n:] if 0 < n < len(pending) else ([] if n == 0 else pending)


def scan(asm, name):
    i = asm.index(name + ':')
    j = asm.index('.Lfunc_end', i)
    vm, lgkm, hits = [], [], []
    in_asm = False
    for l in asm[i:j].split('\n'):
        l = l.strip()
        if l.startswith(';;#ASMSTART'):
            in_asm = True
            continue
        if l.startswith(';;#ASMEND'):
            in_asm = False
            continue
        if not l or l.startswith((';', '.')):
            continue
        ops = l.split(';')[0].replace(',', ' ').split()
        if not ops:
            continue
        op = ops[0]
        if op == 's_waitcnt':
            vm = _retire(vm, l, 'vmcnt')
            lgkm = _retire(lgkm, l, 'lgkmcnt')
            continue
        live = set().union(*vm, *lgkm) if (vm or lgkm) else set()
        srcs = ops[1:]
        if op.startswith(('buffer_load', 'global_load')):
            # an LDS-DMA load (`... lds`) writes LDS, not its first operand (the address)
            dst = set() if ops[-1] == 'lds' else regs(ops[1])
            srcs = ops[1:] if ops[-1] == 'lds' else ops[2:]
            if (dst | set().union(*[regs(t) for t in srcs])) & live:
                hits.append(l)
            vm.append(dst if in_asm else set())
            continue
        if op.startswith('ds_read') or op.startswith('ds_load'):
            dst = regs(ops[1])
            if (dst | set().union(*[regs(t) for t in ops[2:]])) & live:
                hits.append(l)
            lgkm.append(dst if in_asm else set())
            continue
        if op.startswith('s_') or op.endswith(':'):
            continue
        if any(regs(t) & live for t in srcs):
            hits.append(l)
    return hits


# kernels whose fragment / operand loads are inline asm with hand-counted waits
ASM_RING_KERNELS = r'(wgrad_p16_kernel|gemm_kernel|wgrad_taps_kernel|conv0_kernel|rowconv_fwd_kernel)'


def kernels(asm, pattern=ASM_RING_KERNELS):
    return [n for n in re.findall(r'^(_ZN4niti\w+):', asm, flags=re.M) if re.search(pattern, n)]


if __name__ == '__main__':
    bad = 0
    for path in sys.argv[1:]:
        asm = open(path).read()
        for name in kernels(asm):
            h = scan(asm, name)
            if h:
                print(name, len(h), h[:3])
            bad += len(h)
        print(path, len(kernels(asm)), 'asm-ring kernels scanned')
    sys.exit(1 if bad else 0)
