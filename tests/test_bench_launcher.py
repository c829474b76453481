"""bench.py --gpus N (CPU only): the rank launcher's argument -> rank-environment mapping, the refusal to
report a WORLD_SIZE that differs from --gpus, and the launcher's exit status. The ranks stop before any
GPU work (NICNES_BENCH_DRY_RANKS=1), so this runs anywhere; the GPU leg is tests/test_gpu_bench_ranks.py."""
import json
import os
import subprocess
import sys

import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_resolve_world_without_a_launcher():
    assert bench.resolve_world(None, {}) == (1, False)
    assert bench.resolve_world(1, {}) == (1, False)
    assert bench.resolve_world(2, {}) == (2, True)
    assert bench.resolve_world(8, {}) == (8, True)


def test_resolve_world_under_a_launcher():
    assert bench.resolve_world(4, {'WORLD_SIZE': '4'}) == (4, False)
    assert bench.resolve_world(None, {'WORLD_SIZE': '2'}) == (2, False)
    with pytest.raises(SystemExit) as e:
        bench.resolve_world(8, {'WORLD_SIZE': '1'})
    assert e.value.code == 2


def test_rank_environments_match_torch_distributed_run():
    envs = bench.rank_environments(4, 29555, {'PATH': '/bin', 'HSA_ENABLE_IPC_MODE_LEGACY': '0'})
    assert [e['RANK'] for e in envs] == ['0', '1', '2', '3']
    assert [e['LOCAL_RANK'] for e in envs] == ['0', '1', '2', '3']
    for e in envs:
        assert e['WORLD_SIZE'] == '4' and e['LOCAL_WORLD_SIZE'] == '4'
        assert e['MASTER_ADDR'] == '127.0.0.1' and e['MASTER_PORT'] == '29555'
        assert e['PATH'] == '/bin' and e['HSA_ENABLE_IPC_MODE_LEGACY'] == '0'


def _run(args, extra_env, timeout=120):
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    env.pop('RANK', None)
    env.update(extra_env)
    return subprocess.run([sys.executable, os.path.join(REPO, 'bench.py')] + args, env=env, cwd=REPO,
                          capture_output=True, text=True, timeout=timeout)


def test_world_size_mismatch_exits_nonzero():
    p = _run(['--gpus', '8'], {'WORLD_SIZE': '1', 'RANK': '0'})
    assert p.returncode == 2
    assert 'WORLD_SIZE=1' in p.stderr and not p.stdout.strip()


def test_launcher_starts_n_ranks():
    p = _run(['--gpus', '3', '--no-cpu-baseline'], {'NICNES_BENCH_DRY_RANKS': '1', 'NICNES_BENCH_SHARE_GPU': '1'})
    assert p.returncode == 0, p.stderr
    out = [json.loads(l) for l in p.stdout.splitlines() if l.startswith('{')]
    assert [d['RANK'] for d in out] == ['0']            # stdout carries rank 0's line only
    seen = sorted(out + [json.loads(l) for l in p.stderr.splitlines() if l.startswith('{')], key=lambda d: d['RANK'])
    assert [d['RANK'] for d in seen] == ['0', '1', '2']
    assert {d['WORLD_SIZE'] for d in seen} == {'3'}
    assert [d['LOCAL_RANK'] for d in seen] == ['0', '1', '2']
    assert len({d['MASTER_PORT'] for d in seen}) == 1 and {d['MASTER_ADDR'] for d in seen} == {'127.0.0.1'}


def test_launcher_returns_a_failing_ranks_status():
    p = _run(['--gpus', '2'], {'NICNES_BENCH_DRY_RANKS': '1', 'NICNES_BENCH_SHARE_GPU': '1',
                               'NICNES_BENCH_DRY_FAIL_RANK': '1'})
    assert p.returncode == 3


def test_launcher_refuses_more_ranks_than_gpus():
    # this container has no GPU: two ranks on two GPUs cannot start (status 2, nothing printed)
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip('enough GPUs here')
    p = _run(['--gpus', '2'], {'NICNES_BENCH_DRY_RANKS': '1'})
    assert p.returncode == 2 and 'GPUs are visible' in p.stderr
