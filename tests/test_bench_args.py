"""bench.py's argument handling (CPU): the --early-views batch list and the number of binning
batches (= compositor launch pairs per step) the timed-region check expects, and the defaults the
driver's plain `python bench.py` run gets."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_early_views_parsing(bench):
    assert bench._early_views("3") == 3
    assert bench._early_views("1,2") == (1, 2)
    assert bench._early_views("2, 3, 3") == (2, 3, 3)
    import argparse
    with pytest.raises(argparse.ArgumentTypeError):
        bench._early_views("-1")
    with pytest.raises(argparse.ArgumentTypeError):
        bench._early_views("")


@pytest.mark.parametrize("early,V,n", [(3, 8, 2), (0, 8, 1), (8, 8, 1), (9, 8, 1), (1, 8, 2), ((1, 2), 8, 3),
                                       ((2, 3), 8, 3), ((2, 3, 3), 8, 3), ((1, 1, 1), 5, 4), ((3, 5), 8, 2)])
def test_binning_batches(bench, early, V, n):
    """Batches: the early views, then side batches of the listed sizes while views remain, then
    the rest (native_view_renderer's cuts)."""
    assert bench._n_binning_batches(early, V) == n


def test_defaults(bench):
    a = bench.parse_args([])
    assert a.gpus == 1 and a.early_views == 2 and a.order_on_side and a.binning == "sort"
    assert a.main_priority == 0 and a.side_priority == 0
    assert not bench.parse_args(["--no-order-on-side"]).order_on_side
    assert bench.parse_args(["--order-on-side"]).order_on_side
    assert bench.parse_args(["--binning", "bucket", "--early-views", "2,3"]).early_views == (2, 3)
