"""Per-kernel VGPR / SGPR / spill / scratch figures of the decode kernels (hipcc's
-Rpass-analysis=kernel-resource-usage remarks), one line per kernel. A spilling hot kernel is a
regression to catch before any GPU run.
usage: python scripts/kernel_resources.py [source.hip ...]"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
srcs = sys.argv[1:] or [os.path.join(REPO, 'nes-img-captioning_amd', 'csrc', 'decode_kernel.hip')]
for src in srcs:
    r = subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-ffp-contract=off',
                        '-fPIC', '-x', 'hip', '-c', src, '-o', '/dev/null', '-Rpass-analysis=kernel-resource-usage'],
                       capture_output=True, text=True)
    cur, rows = None, []
    for line in r.stderr.splitlines():
        m = re.search(r'remark:\s+(.*?) \[-Rpass', line)
        if not m:
            continue
        txt = m.group(1)
        if txt.startswith('Function Name:'):
            cur = {'name': txt.split(':', 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ':' in txt:
            k, v = txt.split(':', 1)
            cur[k.strip()] = v.strip()
    for d in rows:
        name = subprocess.run(['c++filt', d['name']], capture_output=True, text=True).stdout.strip()
        print('%-62s VGPR %4s AGPR %3s SGPR %3s spillV %3s spillS %3s scratch %4s occ %s' % (
            name[:62], d.get('VGPRs', '?'), d.get('AGPRs', '?'), d.get('TotalSGPRs', '?'), d.get('VGPRs Spill', '?'),
            d.get('SGPRs Spill', '?'), d.get('ScratchSize [bytes/lane]', '?'), d.get('Occupancy [waves/SIMD]', '?')))
