"""The torch-CPU restatement of the reference worker (oracle/ref_worker.py, bench.py's cpu_baseline)
must decode exactly like the imported reference FCModel did when the golden vectors were made."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle import ref_worker


@pytest.mark.parametrize('name', ['decode_tiny_xavier', 'decode_tiny_wc', 'decode_full_wc', 'decode_full_xavier'])
def test_port_decode_bit_exact_vs_reference(golden_dir, name):
    torch.set_num_threads(1)
    z = np.load('%s/%s.npz' % (golden_dir, name))
    V, E, R, F, T = (int(v) for v in z['dims'])
    d = O.Dims(V, E, R, F, T)
    theta = z['theta'] if 'theta' in z else O.make_theta(d, int(z['theta_seed']), float(z['gain']),
                                                         float(z['bias_std']))
    fc = z['fc'] if 'fc' in z else np.random.Generator(np.random.PCG64(int(z['fc_seed']))).standard_normal(
        (int(z['B']), d.F)).astype(np.float32)
    m = ref_worker.FCModelRef(V, E, R, F, T)
    torch.nn.utils.vector_to_parameters(torch.from_numpy(theta), m.parameters())
    with torch.no_grad():
        seq, lp = m.sample(torch.from_numpy(fc))
    assert np.array_equal(seq.numpy(), z['seq'])
    assert np.array_equal(lp.numpy(), z['logprobs'])


def test_port_worker_fitness_pair():
    d = O.Dims(vocab_size=63, E=32, R=32, F=64)
    theta = O.make_theta(d, 2, 4.0, 0.1)
    fc = np.random.default_rng(0).standard_normal((4, d.F)).astype(np.float32)
    gts = [np.random.default_rng(i).integers(1, 64, (5, 16)).astype(np.int32) for i in range(4)]
    w = ref_worker.RefWorker(theta, fc, gts, {}, 100, 5, 63)
    w.model = ref_worker.FCModelRef(63, 32, 32, 64, 16)
    delta = (np.float32(0.01) * np.random.default_rng(1).standard_normal(d.D)).astype(np.float32)
    f = w.fitness(delta)
    assert f.shape == (2,) and np.all(f >= 0)
