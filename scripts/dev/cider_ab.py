"""Dev: CIDEr-D image-kernel time (HIP events, nicnes_kernel_times) of variant libraries, interleaved in one
process: python scripts/dev/cider_ab.py DIR POP ROUNDS"""
import glob
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'nes-img-captioning_amd'))
import torch  # noqa: E402
import nicnes  # noqa: E402
import nicnes.synthetic as S  # noqa: E402

d, pop, rounds = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
libs = sorted(glob.glob(os.path.join(d, 'libnicnes_*.so')))
noise = torch.from_numpy(S.noise_table(1 << 27)).cuda()
engs = {}
ref = None
for p in libs:
    e = nicnes.Engine(max_batch=128, max_members=pop, noise_len=1 << 27, lib_path=p)
    S.setup_engine_workload(e, B=128, noise=noise)
    e.set_timing(True)
    engs[os.path.basename(p)[10:-3]] = e
res = {k: [] for k in engs}
for r in range(rounds):
    for k, e in engs.items():
        f = e.evaluate(r + 1, 0, pop, 0.01)
        res[k].append(e.kernel_times()[1])
        if r == 0:
            if ref is None:
                ref = f.cpu().numpy()
            print(k, 'fitness == first:', bool(np.array_equal(ref, f.cpu().numpy())))
for k, v in res.items():
    print('%-10s cider ms median %.4f min %.4f' % (k, np.median(v), np.min(v)))
