"""The distCUDA2 oracle (oracle/knn_oracle.py) against scipy's KD-tree, an independent exact
3-NN, and its edge cases (CPU)."""
import numpy as np
import pytest

import knn_oracle


@pytest.mark.parametrize("P,seed", [(50, 0), (700, 1), (3000, 2)])
def test_oracle_matches_kdtree(P, seed):
    from scipy.spatial import cKDTree
    rng = np.random.default_rng(seed)
    pts = rng.normal(size=(P, 3)).astype(np.float32) * np.float32(3.0)
    pts[: P // 10] = pts[P // 10: 2 * (P // 10)]            # duplicates: distance 0 neighbours
    got = knn_oracle.mean_dist(pts)
    d, _ = cKDTree(pts.astype(np.float64)).query(pts.astype(np.float64), k=4)
    # k=4 includes the point itself at 0 (or a duplicate): drop exactly one zero per row
    ref = (d[:, 1:] ** 2).mean(axis=1)
    np.testing.assert_allclose(got, ref, rtol=2e-5, atol=1e-6)


def test_oracle_small_sets():
    assert knn_oracle.mean_dist(np.zeros((0, 3), np.float32)).shape == (0,)
    one = knn_oracle.mean_dist(np.ones((1, 3), np.float32))
    assert np.isinf(one[0])
    four = np.array([[0, 0, 0], [1, 0, 0], [0, 2, 0], [0, 0, 3]], np.float32)
    # squared distances: A-B 1, A-C 4, A-D 9, B-C 5, B-D 10, C-D 13
    np.testing.assert_allclose(knn_oracle.mean_dist(four), [14 / 3, 16 / 3, 22 / 3, 32 / 3], rtol=1e-6)
