"""Result files in the reference's format (optimize_pregrasp.py:1016-1020). CPU only."""
import numpy as np

from compliancedex_amd.results import NAMES, load_results, save_results


def test_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    E = 6
    arrs = [rng.random((E, 4, 3)), rng.random((E, 4, 3)), rng.random((E, 6)), rng.random((E, 4)), rng.random((E, 16))]
    paths = save_results("banana", *arrs, data_dir=str(tmp_path))
    assert [p.split("/")[-1] for p in paths] == [f"{n}_banana.npy" for n in NAMES]
    back = load_results("banana", data_dir=str(tmp_path))
    for n, a in zip(NAMES, arrs):
        assert back[n].dtype == np.float64 and np.array_equal(back[n], a)
    # verify_pregrasp.py:154 reads compliance as kp.repeat(3).reshape(-1, 3)
    assert back["compliance"].repeat(3).reshape(-1, 3).shape == (E * 4, 3)
