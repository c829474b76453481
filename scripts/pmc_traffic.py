"""HBM bytes per launch of one kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): the counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced read, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
Counter values are taken per dispatch of the kernel (dispatches whose name matches and whose grid
is the largest seen for it -- the bench's sigma = 0 single-member setup evaluate is dropped --
minus the first `--skip` ones) and averaged.

usage: python scripts/pmc_traffic.py --fetch DIR --write DIR --kernel nicnes_decode_step_kernel \
           --algorithmic-bytes N --out profiles/r01_decode_pmc.json
"""
import argparse
import csv
import glob
import json
import os


def per_dispatch(root, counter, kernel):
    files = glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        raise SystemExit('no counter_collection.csv under %s' % root)
    vals = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get('Counter_Name') != counter or kernel not in row.get('Kernel_Name', ''):
                    continue
                key = (fn, int(row['Dispatch_Id']))
                grid = int(row.get('Grid_Size', 0) or 0)
                g, v = vals.get(key, (grid, 0.0))
                vals[key] = (g, v + float(row['Counter_Value']))
    if not vals:
        return []
    gmax = max(g for g, _ in vals.values())
    return [vals[k][1] for k in sorted(vals) if vals[k][0] == gmax]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--fetch', required=True)
    ap.add_argument('--write', required=True)
    ap.add_argument('--kernel', default='nicnes_decode_step_kernel')
    ap.add_argument('--skip', type=int, default=0)
    ap.add_argument('--algorithmic-bytes', type=float, default=None)
    ap.add_argument('--out', required=True)
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch, 'FETCH_SIZE', a.kernel)[a.skip:]
    write = per_dispatch(a.write, 'WRITE_SIZE', a.kernel)[a.skip:]
    if not fetch or not write:
        raise SystemExit('no dispatches of %s after skipping %d' % (a.kernel, a.skip))
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    hbm = (2.0 * f_kib + w_kib) * 1024.0
    out = {'kernel': a.kernel, 'dispatches_fetch': len(fetch), 'dispatches_write': len(write),
           'fetch_size_kib_per_launch': f_kib, 'write_size_kib_per_launch': w_kib,
           'hbm_bytes_per_launch': hbm, 'formula': '(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count)',
           'algorithmic_bytes_per_launch': a.algorithmic_bytes}
    if a.algorithmic_bytes:
        out['traffic_over_algorithmic'] = hbm / a.algorithmic_bytes
    with open(a.out, 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
