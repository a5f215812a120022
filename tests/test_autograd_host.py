"""CPU: host-side logic of gpsig_amd.autograd (no GPU calls)."""
from gpsig_amd import autograd as ag


def test_fold_blocks_single_launch_for_comparable_sides():
    assert ag._fold_blocks(1024, 512, 5) == (1024, 512)
    assert ag._fold_blocks(50, 50, 5) == (50, 50)


def test_fold_blocks_cut_lopsided_shapes():
    """n1 = 4096, n2 = 64 at one launch is (4160^2 / 2) / (4096 * 64) = 33x the useful pairs and a
    (M+1) * 4160^2 fp64 weight tensor; the blocks keep every launch within ~2x and the weight budget."""
    b1, b2 = ag._fold_blocks(4096, 64, 5)
    assert (b1, b2) == (128, 64)
    pairs = ((4096 + b1 - 1) // b1) * ((64 + b2 - 1) // b2) * (b1 + b2) ** 2 / 2
    assert pairs <= 2.5 * 4096 * 64
    b1, b2 = ag._fold_blocks(64, 4096, 5)
    assert (b1, b2) == (64, 128)


def test_fold_blocks_respect_weight_budget():
    b1, b2 = ag._fold_blocks(20000, 20000, 5, budget=1 << 30)
    assert 12 * 6 * (b1 + b2) ** 2 <= 1 << 30 and b1 == b2 >= 1
