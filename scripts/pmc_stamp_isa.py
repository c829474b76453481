"""Dev tool: add the machine-code stamp (kernel_symbol, kernel_isa_sha256) to PMC profiles that were recorded with the
decode SOURCES' hash only (rounds <= 5), so that a later source edit which leaves the kernel's instructions unchanged
keeps them valid for bench.py (load_pmc).

The stamp is taken from a library built from the commit the profiles measured, never from the current tree: the
commit's decode sources must hash to the profile's recorded source_sha256, else the profile is left alone.

    git worktree add /tmp/wt <commit> && make -C /tmp/wt/nes-img-captioning_amd
    python scripts/pmc_stamp_isa.py --worktree /tmp/wt --commit <commit> profiles/r05_pmc_*.json
"""
import argparse
import hashlib
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'nes-img-captioning_amd'))
import bench  # noqa: E402
from nicnes import codeobj  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--worktree', required=True)
    ap.add_argument('--commit', required=True)
    ap.add_argument('profiles', nargs='+')
    a = ap.parse_args()
    h = hashlib.sha256()
    for f in bench.KERNEL_SOURCES:
        with open(os.path.join(a.worktree, f), 'rb') as fh:
            h.update(fh.read())
    src_sha = h.hexdigest()
    lib = os.path.join(a.worktree, 'nes-img-captioning_amd', 'nicnes', 'libnicnes.so')
    listings = codeobj.kernel_listings(lib)
    keys = {v: k for k, v in bench.PMC_KEYS.items()}
    for path in a.profiles:
        m = re.match(r'r\d+_pmc_([a-z0-9]+)_p\d+_b\d+\.json$', os.path.basename(path))
        if not m or m.group(1) not in keys:
            print('skip (not a decode profile):', path)
            continue
        with open(path) as f:
            rec = json.load(f)
        if rec.get('source_sha256') != src_sha:
            print('skip (measured other sources than %s):' % a.commit, path)
            continue
        key = m.group(1)
        symbol = bench.PMC_SYMBOLS[(key, key != 'sampled')]      # the bench's default instantiation
        rec['kernel_symbol'] = symbol
        rec['kernel_isa_sha256'] = codeobj.kernel_isa_sha256(lib, symbol, listings)
        rec['isa_stamp'] = {'library_built_from_commit': a.commit,
                            'note': 'machine code of the measured instantiation in a library built from the commit whose '
                                    'decode sources hash to source_sha256 (scripts/pmc_stamp_isa.py)'}
        with open(path, 'w') as f:
            json.dump(rec, f, indent=1)
        print('stamped', path, symbol, rec['kernel_isa_sha256'][:12])


if __name__ == '__main__':
    main()
