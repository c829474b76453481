"""Per-launch PMC summary of one kernel from several rocprofv3 --pmc passes.

Each pass directory holds a counter_collection.csv. For the kernel (substring of Kernel_Name), the
dispatches with the largest grid are kept (the bench's sigma = 0 single-member setup evaluate is
dropped), every counter is summed over its instances per dispatch and averaged over dispatches.
Derived figures (MI355X_MICROARCH.md: HBM section, rocprofv3 PMC slots, DVFS item):
  hbm_bytes        = (2 * FETCH_SIZE + WRITE_SIZE) * 1024   (gfx950 FETCH_SIZE half-count, KiB units)
  gpu_cycles       = GRBM_GUI_ACTIVE / 8                    (rocprofv3 sums the 8 XCDs)
  mfma_busy        = SQ_VALU_MFMA_BUSY_CYCLES / (gpu_cycles * CUs * 4 SIMDs)
  valu_mfma_coexec = SQ_VALU_MFMA_COEXEC_CYCLES / SQ_VALU_MFMA_BUSY_CYCLES
  wave_wait / wave_issue_stall / wave_active = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  clock_ghz        = gpu_cycles / kernel duration (from --duration-ms)

usage: python scripts/pmc_summary.py --kernel nicnes_decode_step_kernel --pass DIR [--pass DIR ...]
           [--duration-ms 2.66] [--cus 256] [--algorithmic-bytes N] [--algorithmic-flop N] --out FILE
"""
import argparse
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (kernel_source_sha256: the profile records which decode sources it measured)


def per_dispatch(root, kernel):
    files = glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        raise SystemExit('no counter_collection.csv under %s' % root)
    vals = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if kernel not in row.get('Kernel_Name', ''):
                    continue
                key = (fn, int(row['Dispatch_Id']))
                grid = int(row.get('Grid_Size', 0) or 0)
                d = vals.setdefault(key, {'grid': grid, 'c': {}})
                name = row['Counter_Name']
                d['c'][name] = d['c'].get(name, 0.0) + float(row['Counter_Value'])
    if not vals:
        return {}
    gmax = max(d['grid'] for d in vals.values())
    keep = [vals[k]['c'] for k in sorted(vals) if vals[k]['grid'] == gmax]
    out = {}
    for name in keep[0]:
        xs = [c[name] for c in keep if name in c]
        out[name] = (sum(xs) / len(xs), len(xs))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--kernel', required=True)
    ap.add_argument('--pass', dest='passes', action='append', required=True)
    ap.add_argument('--duration-ms', type=float, default=None)
    ap.add_argument('--cus', type=int, default=256)
    ap.add_argument('--algorithmic-bytes', type=float, default=None)
    ap.add_argument('--algorithmic-flop', type=float, default=None)
    ap.add_argument('--note', default='')
    ap.add_argument('--symbol', default=None, help='mangled name of the measured instantiation: the profile records '
                    'its machine-code hash in the tree\'s library (bench.load_pmc checks it)')
    ap.add_argument('--out', required=True)
    a = ap.parse_args()
    counters, dispatches = {}, {}
    for p in a.passes:
        for name, (v, n) in per_dispatch(p, a.kernel).items():
            counters[name] = v
            dispatches[name] = n
    c = counters
    out = {'kernel': a.kernel, 'note': a.note, 'source_sha256': bench.kernel_source_sha256(),
           'counters_per_launch': c, 'dispatches': dispatches}
    if a.symbol:
        out['kernel_symbol'] = a.symbol
        out['kernel_isa_sha256'] = bench.library_kernel_sha(a.symbol)
    d = {}
    if 'FETCH_SIZE' in c and 'WRITE_SIZE' in c:
        d['hbm_bytes_per_launch'] = (2.0 * c['FETCH_SIZE'] + c['WRITE_SIZE']) * 1024.0
        if a.algorithmic_bytes:
            d['traffic_over_algorithmic'] = d['hbm_bytes_per_launch'] / a.algorithmic_bytes
    if 'GRBM_GUI_ACTIVE' in c:
        cyc = c['GRBM_GUI_ACTIVE'] / 8.0
        d['gpu_cycles_per_launch'] = cyc
        if a.duration_ms:
            d['clock_ghz'] = cyc / (a.duration_ms * 1e-3) / 1e9
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in c:
            d['mfma_busy'] = c['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * a.cus * 4)
    if 'SQ_VALU_MFMA_BUSY_CYCLES' in c and 'SQ_INSTS_MFMA' in c and c['SQ_INSTS_MFMA']:
        d['mfma_busy_cycles_per_mfma'] = c['SQ_VALU_MFMA_BUSY_CYCLES'] / c['SQ_INSTS_MFMA']
    if 'SQ_VALU_MFMA_COEXEC_CYCLES' in c and c.get('SQ_VALU_MFMA_BUSY_CYCLES'):
        d['valu_mfma_coexec_frac'] = c['SQ_VALU_MFMA_COEXEC_CYCLES'] / c['SQ_VALU_MFMA_BUSY_CYCLES']
    if 'SQ_INSTS_VALU' in c and c.get('SQ_INSTS_MFMA'):
        d['valu_insts_per_mfma'] = (c['SQ_INSTS_VALU'] - c['SQ_INSTS_MFMA']) / c['SQ_INSTS_MFMA']
    if c.get('SQ_WAVE_CYCLES'):
        for k in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_LDS',
                  'SQ_ACTIVE_INST_VMEM'):
            if k in c:
                d[k.lower().replace('sq_', '') + '_over_wave_cycles'] = c[k] / c['SQ_WAVE_CYCLES']
    if a.algorithmic_flop and a.duration_ms:
        d['achieved_tflops'] = a.algorithmic_flop / (a.duration_ms * 1e-3) / 1e12
    out['derived'] = d
    with open(a.out, 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(d))


if __name__ == '__main__':
    main()
