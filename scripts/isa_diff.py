"""Dev tool: per-kernel gfx950 ISA of a HIP source, normalised so two builds can be compared function by function
(the round-6 knob clean-up of decode_kernel.hip had to leave every product kernel's instructions unchanged).

    python scripts/isa_diff.py dump SRC OUT.json [extra hipcc flags...]   # {kernel: normalised instruction text}
    python scripts/isa_diff.py diff A.json B.json                         # kernels added / removed / changed

Normalisation: comments and blank lines dropped, basic-block labels renumbered per function (.LBB<f>_<n> ->
.LBB_<n>: the function index shifts when other kernels are removed); the kernel descriptor (.amdhsa_* lines:
VGPR / SGPR counts, LDS, scratch) is kept as part of the function."""
import json
import re
import subprocess
import sys

FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-ffp-contract=off', '-fPIC', '-x', 'hip', '--cuda-device-only',
         '-S', '-o', '-']


def dump(src, out, extra):
    r = subprocess.run(['/opt/rocm/bin/hipcc'] + FLAGS + extra + [src], capture_output=True, text=True, check=True)
    funcs, cur, name = {}, None, None
    desc = {}
    dname = None
    for raw in r.stdout.splitlines():
        line = raw.split(';')[0].rstrip()
        if not line.strip():
            continue
        m = re.match(r'^([A-Za-z_][\w.$]*):\s*$', line)
        if m and not line.startswith('.'):
            name = m.group(1)
            cur = funcs.setdefault(name, [])
            continue
        if line.strip().startswith('.Lfunc_end'):
            name, cur = None, None
            continue
        m = re.match(r'^\s*\.amdhsa_kernel\s+(\S+)', line)
        if m:
            dname = m.group(1)
            desc[dname] = []
            continue
        if line.strip() == '.end_amdhsa_kernel':
            dname = None
            continue
        if dname is not None:
            desc[dname].append(line.strip())
            continue
        if cur is not None:
            cur.append(re.sub(r'\.LBB\d+_(\d+)', r'.LBB_\1', line.strip()))
    out_d = {k: '\n'.join(v + desc.get(k, [])) for k, v in funcs.items() if k.startswith('_Z')}
    with open(out, 'w') as f:
        json.dump(out_d, f, indent=0, sort_keys=True)
    print('%d kernels/functions' % len(out_d))


def diff(a, b):
    A, B = json.load(open(a)), json.load(open(b))
    only_a, only_b = sorted(set(A) - set(B)), sorted(set(B) - set(A))
    changed = sorted(k for k in set(A) & set(B) if A[k] != B[k])
    same = sorted(k for k in set(A) & set(B) if A[k] == B[k])
    demangle = lambda ks: subprocess.run(['c++filt'], input='\n'.join(ks), capture_output=True, text=True).stdout.split('\n')
    for title, ks in (('only in A', only_a), ('only in B', only_b), ('CHANGED', changed), ('identical', same)):
        print('%s (%d):' % (title, len(ks)))
        for k in demangle(ks):
            if k:
                print('   ', k)
    return 1 if changed else 0


if __name__ == '__main__':
    if sys.argv[1] == 'dump':
        dump(sys.argv[2], sys.argv[3], sys.argv[4:])
    else:
        sys.exit(diff(sys.argv[2], sys.argv[3]))
