"""CPU checks of the QSC step's launch geometry (ops/qsc.py)."""
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.qsc import balanced_grid


def test_balanced_grid_gives_every_wave_the_same_samples():
    # the flagship step: 2304 samples, 4 waves per workgroup, at most 256 workgroups -> 3 samples per wave
    assert balanced_grid(2304, 4, 256) == 192
    for samples in (32, 100, 288, 2304, 4608, 9216):
        for waves, cap in ((4, 256), (2, 256), (4, 128)):
            g = balanced_grid(samples, waves, cap)
            assert 1 <= g <= cap
            busiest_cap = -(-samples // (waves * cap))
            # the same samples per wave as the capped grid's busiest wave, and every sample covered
            assert -(-samples // (waves * g)) == busiest_cap
            assert g * waves * busiest_cap >= samples
            # and no smaller grid keeps that load
            assert g == 1 or (g - 1) * waves * busiest_cap < samples
