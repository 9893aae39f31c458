"""Scan gfx950 assembly for instructions that touch a register an inline-asm load is still writing.

Kernels with asm load rings (the P16 weight gradient's buffer_load ring, the GEMM / tap-sharing /
first-layer kernels' ds_read fragment rings) count their own waits: hipcc does not know when such
a load lands, and may hand the destination of a load whose result it believes dead (the last
look-ahead loads of a ring) to another value while the load is still in flight -- the fault found
in round 2.  The scan tracks every load in issue order: loads between hipcc's ;;#ASMSTART /
;;#ASMEND markers hold their destination registers until an s_waitcnt retires them (vmcnt for
buffer / global loads, lgkmcnt for ds_read, in order); compiler-issued loads only take a place in
the counters.  Any other instruction naming a held register is a hit.

The scan follows the instruction order of the file, except that a block only entered by
forward branches (the previous instruction is an unconditional s_branch) starts from the merged
state of those branches rather than from the unrelated code above it.  A block with a
fall-through keeps the fall-through state: the waits of an if/else wait ladder (a dynamic
count) are all taken as executed, so the scan is optimistic there.  Back edges are not
followed, so a hit at a loop head may be a false alarm, and SMEM loads (which retire lgkmcnt
out of order) are not modelled.  A clean
scan is what every asm-ring kernel must show.
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


def _merge(a, b):
    """Two pending lists aligned at their most recent load; a waitcnt(n) keeps the last n of each."""
    n = max(len(a), len(b))
    a = [set()] * (n - len(a)) + a
    b = [set()] * (n - len(b)) + b
    return [x | y for x, y in zip(a, b)]


def scan(asm, name):
    i = asm.index(name + ':')
    j = asm.index('.Lfunc_end', i)
    vm, lgkm, hits = [], [], []
    in_asm = False
    at_label = {}           # label -> (vm, lgkm) merged over the forward branches seen so far
    no_fall = False         # the previous instruction never falls through
    for l in asm[i:j].split('\n'):
        l = l.strip()
        m = re.match(r'(\.LBB\w+):', l)
        if m:
            got = at_label.pop(m.group(1), None)
            if got is not None and no_fall:
                vm, lgkm = list(got[0]), list(got[1])
            no_fall = False
            continue
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
        if op.startswith(('s_branch', 's_cbranch')) and len(ops) > 1 and ops[1].startswith('.LBB'):
            old = at_label.get(ops[1])
            at_label[ops[1]] = (list(vm), list(lgkm)) if old is None else \
                (_merge(old[0], vm), _merge(old[1], lgkm))
            no_fall = op == 's_branch'
            continue
        no_fall = op in ('s_endpgm', 's_setpc_b64')
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
