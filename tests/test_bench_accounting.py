"""bench.py's algorithmic work per unit against SURVEY.md 8(d) (CPU only): the roofline's
`achieved` and `algorithmic_bytes_per_launch` are built from these."""
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
