#!/usr/bin/env python3
"""Scan the gfx950 machine code inside libnicnes.so for the store-data hazard of DESIGN.md section 8.

On gfx950 a vector-memory store of more than 8 bytes (dwordx3 / dwordx4: buffer, global, flat, scratch)
reads its data registers after it issues. A VALU instruction that writes one of those registers too soon
after the store changes what is stored. The compiler does not pad this case; in round 4 it put the zeroing
of a sampled-pick block sum right behind the 16-byte record store and ~450 of 10.5 M picks went wrong until
`s_nop 1` wait states were placed by hand (csrc/decode_kernel.hip, the record stores).

The rule checked here: after such a store, a VALU write of any of its data VGPRs needs at least
MIN_WAIT_STATES wait states in between, where every other instruction counts one and `s_nop N` counts N + 1.
The window is followed in program order (the fall-through path of a conditional branch; an unconditional
branch ends it).

    python scripts/isa_hazard.py [path/to/libnicnes.so]      # prints the hits, exit 1 if any

Used by tests/test_isa_hazards.py on every CPU test run.
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = '/opt/rocm/lib/llvm/bin'
BUNDLE_MAGIC = b'__CLANG_OFFLOAD_BUNDLE__'
MIN_WAIT_STATES = 2          # what the hand-placed `s_nop 1` provides
ARCH = 'gfx950'

_STORE = re.compile(r'^\s*(buffer|global|flat|scratch)_store_dwordx([34])\s+(.*)$')
_FUNC = re.compile(r'^[0-9a-f]+ <(.+)>:$')
_INSN = re.compile(r'^\s+([a-z_0-9]+)(?:\s+(.*?))?\s*(?://.*)?$')


sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'nes-img-captioning_amd'))
from nicnes.codeobj import code_objects, disassemble  # noqa: E402,F401  (the library's gfx950 code objects)


def vregs(tok):
    """VGPR numbers of an operand token (v7, v[4:7]); empty for anything else."""
    tok = tok.strip()
    m = re.match(r'^v\[(\d+):(\d+)\]$', tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'^v(\d+)$', tok)
    return {int(m.group(1))} if m else set()


def store_data_regs(kind, operands):
    ops = [o.strip() for o in operands.split(',')]
    # buffer_store vdata, vaddr|off, srsrc, soffset; global/flat/scratch_store vaddr|off, vdata, ...
    return vregs(ops[0]) if kind == 'buffer' else vregs(ops[1]) if len(ops) > 1 else set()


def scan(asm, min_wait=MIN_WAIT_STATES):
    """[(function, store line, offending line, wait states)] for every store whose data registers a VALU
    instruction writes with fewer than min_wait wait states in between."""
    lines = asm.splitlines()
    hits = []
    fn = None
    for i, line in enumerate(lines):
        m = _FUNC.match(line)
        if m:
            fn = m.group(1)
            continue
        m = _STORE.match(line.split('//')[0])
        if not m:
            continue
        data = store_data_regs(m.group(1), m.group(3))
        if not data:
            continue
        waits, j = 0, i + 1
        while j < len(lines) and waits < min_wait:
            im = _INSN.match(lines[j].split('//')[0] + ' ')
            j += 1
            if not im or not lines[j - 1].startswith('\t'):
                if _FUNC.match(lines[j - 1]):
                    break
                continue
            op, args = im.group(1), im.group(2) or ''
            if op == 's_nop':
                waits += int(args.split()[0], 0) + 1 if args else 1
                continue
            if op.startswith('v_') and args:
                dst = args.split(',')[0]
                if vregs(dst) & data:
                    hits.append((fn, line.split('//')[0].strip(), lines[j - 1].split('//')[0].strip(), waits))
                    break
            if op == 's_branch' or op in ('s_endpgm', 's_setpc_b64'):
                break                       # (a conditional branch's fall-through path is followed)
            waits += 1
    return hits


def wide_stores(asm):
    """How many dwordx3 / dwordx4 stores the listing holds (the scan's coverage)."""
    return sum(1 for line in asm.splitlines() if _STORE.match(line.split('//')[0]))


def scan_library(so_path, counts=None):
    """Hits over every gfx950 code object of a library or relocatable object; `counts` (a dict), when
    given, receives the number of code objects and of wide stores scanned."""
    hits, n_co, n_st = [], 0, 0
    for _, code in code_objects(so_path):
        asm = disassemble(code)
        hits += scan(asm)
        n_co += 1
        n_st += wide_stores(asm)
    if counts is not None:
        counts.update(code_objects=n_co, wide_stores=n_st)
    return hits


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(
        __file__))), 'nes-img-captioning_amd', 'nicnes', 'libnicnes.so')
    counts = {}
    hits = scan_library(so, counts)
    for fn, st, bad, w in hits:
        print('%s\n    %s\n    %s   (%d wait states)' % (fn, st, bad, w))
    print('%d hazard(s) in %s (%d code objects, %d wide stores)' % (len(hits), so, counts['code_objects'],
                                                                  counts['wide_stores']))
    return 1 if hits else 0


if __name__ == '__main__':
    sys.exit(main())
