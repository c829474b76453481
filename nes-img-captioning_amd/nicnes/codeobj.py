"""The gfx950 machine code inside libnicnes.so (measurement bookkeeping, not the compute path).

A committed rocprofv3 PMC profile measures one kernel's machine code. bench.py reports its counters only while the
library it runs holds the same code for that kernel: kernel_isa_sha256 hashes the kernel's disassembled
instructions (addresses and encodings dropped; branch targets are function-relative), so a source edit that leaves
a kernel's instructions unchanged keeps its profile valid and any change to them invalidates it.
scripts/isa_hazard.py scans the same code objects for the store-data hazard.
Needs the ROCm LLVM tools (/opt/rocm/lib/llvm/bin), present wherever the library is built or run."""
import hashlib
import os
import re
import struct
import subprocess
import tempfile

LLVM = '/opt/rocm/lib/llvm/bin'
BUNDLE_MAGIC = b'__CLANG_OFFLOAD_BUNDLE__'
ARCH = 'gfx950'
_FUNC = re.compile(r'^[0-9a-f]+ <(.+)>:$')


def code_objects(so_path):
    """The gfx950 code objects of every offload bundle in the library's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, 'fatbin')
        subprocess.check_call([os.path.join(LLVM, 'llvm-objcopy'), '--dump-section', '.hip_fatbin=' + fb, so_path,
                               os.path.join(td, 'lib.so')])
        with open(fb, 'rb') as f:
            data = f.read()
    out = []
    start = data.find(BUNDLE_MAGIC)
    while start >= 0:
        n = struct.unpack_from('<Q', data, start + len(BUNDLE_MAGIC))[0]
        p = start + len(BUNDLE_MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from('<QQQ', data, p)
            p += 24
            triple = data[p:p + tlen].decode()
            p += tlen
            if triple.endswith('--' + ARCH) and size:
                out.append((triple, data[start + off:start + off + size]))
        start = data.find(BUNDLE_MAGIC, start + 1)
    return out


def disassemble(code):
    with tempfile.NamedTemporaryFile(suffix='.co') as f:
        f.write(code)
        f.flush()
        return subprocess.check_output([os.path.join(LLVM, 'llvm-objdump'), '-d', '--mcpu=' + ARCH, f.name],
                                       text=True)


def kernel_listings(so_path):
    """{mangled function name: normalised instruction text} over every gfx950 code object of the library."""
    out = {}
    for _, code in code_objects(so_path):
        fn, lines = None, []
        for line in disassemble(code).splitlines():
            m = _FUNC.match(line)
            if m:
                if fn is not None:
                    out[fn] = '\n'.join(lines)
                fn, lines = m.group(1), []
                continue
            if fn is None or not line.startswith('\t'):
                continue
            ins = line.split('//')[0].strip()
            if ins:
                lines.append(re.sub(r'\s+', ' ', ins))
        if fn is not None:
            out[fn] = '\n'.join(lines)
    return out


def kernel_isa_sha256(so_path, symbol, listings=None):
    """SHA-256 of one kernel's normalised instructions (None when the library has no such kernel)."""
    lst = listings if listings is not None else kernel_listings(so_path)
    txt = lst.get(symbol)
    return hashlib.sha256(txt.encode()).hexdigest() if txt is not None else None
