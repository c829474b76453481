"""bench.py --gpus 2 with no external launcher, on a one-GPU box: both ranks time-share cuda:0 over gloo
(NICNES_BENCH_SHARE_GPU=1, NICNES_BENCH_BACKEND=gloo). The line must say 2 GPUs, what the collective
saw (2 ranks) and both ranks' member ranges."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_launches_two_ranks_itself():
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        env.pop(k, None)
    env.update({'NICNES_BENCH_SHARE_GPU': '1', 'NICNES_BENCH_BACKEND': 'gloo'})
    p = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', '2', '--steps', '2', '--warmup', '1',
                        '--population', '64', '--noise-len', str(1 << 25)], env=env, cwd=REPO, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout                  # rank 0 alone prints the line
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == 2 and rec['config']['members_per_gpu'] == 32
    assert rec['config']['collective']['world_size'] == 2
    assert rec['config']['shared_gpu_rehearsal'] is True
    assert [r['members'] for r in rec['ranks']] == [[0, 32], [32, 64]]
    assert [r['rank'] for r in rec['ranks']] == [0, 1]
    for r in rec['ranks']:
        assert r['evaluate_ms'] > 0 and r['update_ms'] > 0 and r['exchange_ms'] >= 0
    assert rec['value'] > 0 and rec['cpu_baseline'] is None
