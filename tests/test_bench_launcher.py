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
    if 'NICNES_BENCH_KFD_TOPOLOGY' in extra_env:       # a stub node: its GPUs, not this container's device mask
        for v in bench.VISIBLE_DEVICE_VARS:
            env.pop(v, None)
    env.update(extra_env)
    return subprocess.run([sys.executable, os.path.join(REPO, 'bench.py')] + args, env=env, cwd=REPO,
                          capture_output=True, text=True, timeout=timeout)


def test_world_size_mismatch_exits_nonzero():
    p = _run(['--gpus', '8'], {'WORLD_SIZE': '1', 'RANK': '0'})
    assert p.returncode == 2
    assert 'WORLD_SIZE=1' in p.stderr and not p.stdout.strip()


def test_launcher_starts_n_ranks():
    p = _run(['--gpus', '3', '--population', '384', '--no-cpu-baseline'], {'NICNES_BENCH_DRY_RANKS': '1', 'NICNES_BENCH_SHARE_GPU': '1'})
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


def test_launcher_refuses_more_ranks_than_gpus(tmp_path):
    # a stub node with one GPU: two ranks on two GPUs cannot start (status 2, nothing printed)
    topo, dri = _stub_node(tmp_path, 1)
    p = _run(['--gpus', '2'], {'NICNES_BENCH_DRY_RANKS': '1', 'NICNES_BENCH_KFD_TOPOLOGY': topo,
                               'NICNES_BENCH_DRI': dri})
    assert p.returncode == 2 and 'GPUs are visible' in p.stderr and not p.stdout.strip()
    # no readable topology at all: status 2 as well (the launcher never falls back to a HIP call)
    p = _run(['--gpus', '2'], {'NICNES_BENCH_DRY_RANKS': '1', 'NICNES_BENCH_KFD_TOPOLOGY': str(tmp_path / 'none')})
    assert p.returncode == 2 and 'KFD topology' in p.stderr


def _stub_node(tmp_path, n_gpu, hidden=()):
    """A KFD topology like an MI355X node's: node 0 a CPU (no SIMDs), nodes 1..n_gpu GPUs with render minors
    128.., each with a render-node file (absent for the `hidden` GPUs, as a cgroup-restricted container has)."""
    topo, dri = tmp_path / 'nodes', tmp_path / 'dri'
    dri.mkdir()
    for k in range(n_gpu + 1):
        d = topo / str(k)
        d.mkdir(parents=True)
        if k == 0:
            (d / 'properties').write_text('cpu_cores_count 128\nsimd_count 0\ndrm_render_minor 0\n')
            continue
        (d / 'properties').write_text('cpu_cores_count 0\nsimd_count 1024\ngfx_target_version 90500\n'
                                      'drm_render_minor %d\n' % (127 + k))
        if k - 1 not in hidden:
            (dri / ('renderD%d' % (127 + k))).write_text('')
    return str(topo), str(dri)


def test_usable_gpu_count_reads_sysfs_only(tmp_path):
    topo, dri = _stub_node(tmp_path, 8, hidden=(3,))
    assert bench.usable_gpu_count({}, topo, dri) == 7
    assert bench.usable_gpu_count({'HIP_VISIBLE_DEVICES': '0,1'}, topo, dri) == 2
    assert bench.usable_gpu_count({}, str(tmp_path / 'missing'), dri) is None


@pytest.mark.parametrize('preset, per_rank, bu', [('metric', 64, False), ('configs3', 256, False),
                                                  ('configs4', 64, True)])
def test_launcher_eight_ranks_on_an_eight_gpu_node(tmp_path, preset, per_rank, bu):
    """bench.py --gpus 8 as the driver runs it on an 8-GPU node: the launcher counts the GPUs
    from sysfs (stub topology), starts 8 rank environments, and the ranks' member ranges tile the population
    (configs[3]: 256 per rank of 2048; configs[4] and the metric: 64 per rank of 512)."""
    topo, dri = _stub_node(tmp_path, 8)
    p = _run(['--gpus', '8', '--preset', preset, '--no-cpu-baseline'],
             {'NICNES_BENCH_DRY_RANKS': '1', 'NICNES_BENCH_KFD_TOPOLOGY': topo, 'NICNES_BENCH_DRI': dri})
    assert p.returncode == 0, p.stderr
    out = [json.loads(l) for l in p.stdout.splitlines() if l.startswith('{')]
    assert [d['RANK'] for d in out] == ['0']
    seen = sorted(out + [json.loads(l) for l in p.stderr.splitlines() if l.startswith('{')], key=lambda d: int(d['RANK']))
    assert [int(d['RANK']) for d in seen] == list(range(8)) and [d['LOCAL_RANK'] for d in seen] == [str(r) for r in range(8)]
    assert {d['WORLD_SIZE'] for d in seen} == {'8'} and len({d['MASTER_PORT'] for d in seen}) == 1
    assert [d['members'] for d in seen] == [[r * per_rank, (r + 1) * per_rank] for r in range(8)]
    assert {d['population'] for d in seen} == {8 * per_rank} and {d['bu'] for d in seen} == {bu}
    assert {d['scaling'] for d in seen} == {'strong'}
