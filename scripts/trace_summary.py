"""Per-kernel launch summary of a rocprofv3 --kernel-trace run, restricted to full-population launches.

The bench's first evaluate is a sigma = 0, single-member setup decode (it derives the synthetic
references); its launches have a smaller grid. This script keeps the launches whose grid equals
the largest grid seen for that kernel, so the averages are over exactly the launches the bench's
HIP events time, and writes them next to the unfiltered rocprofv3 --stats averages.

usage: python scripts/trace_summary.py --trace DIR --out profiles/r01_decode_launches.json
"""
import argparse
import csv
import glob
import json
import os


def grid_of(row):
    x, y, z = (int(row.get(k, 1) or 1) for k in ('Grid_Size_X', 'Grid_Size_Y', 'Grid_Size_Z'))
    return (x * y * z, x, y, z)          # the largest total grid first (a split launch has a wide x)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--trace', required=True)
    ap.add_argument('--out', required=True)
    ap.add_argument('--prefix', default='nicnes_')
    ap.add_argument('--command', default='')
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.trace, '**', '*kernel_trace.csv'), recursive=True)
    if not files:
        raise SystemExit('no kernel_trace.csv under %s' % a.trace)
    launches = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                name = row['Kernel_Name'].split('(')[0]
                if a.prefix not in name:
                    continue
                dur = (int(row['End_Timestamp']) - int(row['Start_Timestamp'])) / 1e6
                launches.setdefault(name, []).append((int(row['Dispatch_Id']), grid_of(row), dur))
    out = {'command': a.command, 'kernels': {}}
    for name, rows in sorted(launches.items()):
        rows.sort()
        gmax = max(r[1] for r in rows)
        full = [r[2] for r in rows if r[1] == gmax]
        out['kernels'][name] = {
            'launches_all': len(rows), 'mean_ms_all': sum(r[2] for r in rows) / len(rows),
            'launches_full_grid': len(full), 'mean_ms_full_grid': sum(full) / len(full),
            'total_ms_full_grid': sum(full), 'grid': list(gmax),
        }
    with open(a.out, 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
