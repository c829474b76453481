"""bench.py's algorithmic work per unit against SURVEY.md 8(d) (CPU only): the roofline's
`achieved` and `algorithmic_bytes_per_launch` are built from these."""
import os

import bench


def test_flops_per_member_match_survey():
    # 2 [F E + 17 (2 E 5 R) + 16 R V1] = 44,957,696 FLOP per row and decode
    assert bench.decode_flops_per_member(1) == 2 * 44957696
    assert abs(bench.decode_flops_per_member(128) / 1e9 - 11.509) < 5e-4
    # the step kernel does everything but the image projection
    assert bench.decode_flops_per_member(128) - bench.step_flops_per_member(128) == 2 * 128 * 2 * 2048 * 128


def test_noise_bytes_per_member():
    logit = 9488 * 129 * 4
    cell = 2 * 640 * 129 * 4
    assert bench.step_noise_bytes_per_member(128) == 16 * logit + 17 * cell + 15 * 2 * 128 * 128 * 4 + 512
    # 512 members over 18 launches: ~2.6 GB per launch
    assert abs(bench.step_noise_bytes_per_member(128) * 512 / 18 / 1e9 - 2.603) < 1e-3


def test_stale_pmc_profiles_are_not_reported(tmp_path, monkeypatch):
    """bench.py reports a PMC profile's counter figures only while the decode sources hash as recorded."""
    import json
    import os
    prof = tmp_path / 'profiles'
    prof.mkdir()
    for f in bench.KERNEL_SOURCES:
        os.makedirs(tmp_path / os.path.dirname(f), exist_ok=True)
        with open(os.path.join(bench.REPO, f), 'rb') as src, open(tmp_path / f, 'wb') as dst:
            dst.write(src.read())
    monkeypatch.setattr(bench, 'REPO', str(tmp_path))
    sha = bench.kernel_source_sha256()
    rec = {'kernel': 'nicnes_decode_steps_kernel', 'derived': {'hbm_bytes_per_launch': 1.0}}
    (prof / 'r02_pmc_steps_p512_b128.json').write_text(json.dumps(dict(rec, source_sha256='0' * 64)))
    got, why = bench.load_pmc('nicnes_decode_steps_kernel', 512, 128)
    assert got is None and 'r02_pmc_steps_p512_b128.json' in why
    (prof / 'r03_pmc_steps_p512_b128.json').write_text(json.dumps(dict(rec, source_sha256=sha)))
    got, why = bench.load_pmc('nicnes_decode_steps_kernel', 512, 128)
    assert why is None and got['file'] == os.path.join('profiles', 'r03_pmc_steps_p512_b128.json')
    # an edit of the kernel makes the newest profile stale too
    with open(tmp_path / bench.KERNEL_SOURCES[0], 'ab') as f:
        f.write(b'\n// edit\n')
    got, why = bench.load_pmc('nicnes_decode_steps_kernel', 512, 128)
    assert got is None and why
    assert bench.load_pmc('no such kernel', 512, 128) == (None, None)


def test_presets_name_the_baseline_configs():
    import json
    with open(os.path.join(bench.REPO, 'BASELINE.json')) as f:
        cfgs = json.load(f)['configs']
    assert bench.PRESETS['metric'][0] == 512 and bench.PRESETS['configs2'][:2] == (512, 128)
    assert bench.PRESETS['configs1'][0] == 64 and 'pop=64' in cfgs[1]
    assert bench.PRESETS['configs3'][0] == 2048 and 'pop=2048' in cfgs[3]
    assert bench.PRESETS['configs4'][2] and 'bu' in cfgs[4] and 'pop=512' in cfgs[4]


def test_committed_pmc_profiles_match_the_decode_sources():
    """The bench line's counter figures (traffic, MFMA busy) come from committed PMC profiles: every shape the
    bench reports (the fused kernel at 512 and 256 members per GPU, the coop kernel at 128 and 64, the sampled
    kernel) has one measured on the machine code the built library holds now for that instantiation (round 6:
    kernel_isa_sha256 of the symbol, nicnes.codeobj; a source edit that leaves the instructions unchanged keeps it)."""
    for kernel, P in (('nicnes_decode_steps_kernel', 512), ('nicnes_decode_coop_kernel<2>', 128),
                      ('nicnes_decode_coop_kernel<4>', 64), ('nicnes_decode_steps_kernel<sample>', 512)):
        rec, why = bench.load_pmc(kernel, P, 128)
        assert rec is not None, why
        assert rec['derived']['hbm_bytes_per_launch'] > 0 and 0 < rec['derived']['mfma_busy'] < 1


def test_sampled_slot_bytes_follow_the_slot_layout():
    """bench.py's sampled algorithmic bytes: per workgroup, logit step and 64-row stage 72 KiB (8 logit words and
    the {P, r} record, 9 x 64 lanes x 16 B per wave, 8 waves) plus 8 KiB per block of 8 stages."""
    nst = (9488 + 63) // 64
    assert nst == 149 and 9 * 64 * 16 * 8 == 73728
    src = open(os.path.join(bench.REPO, 'bench.py')).read()
    assert 'nst * 73728 + (nst + 7) // 8 * 8192' in src
