"""Tile-bucket binning (tilebin.hip: lsr_forward_preprocess_views_tb_async,
lsr_forward_instance_scan_views_async, lsr_forward_binning_views_tb) against the sort path
(depth sort + instance emission + stable 13-bit tile sort), which the parity suite pins to the
oracle: the same instance count, the same tile ranges and point-list words (ids and quadrant bits,
in the same (depth, id) order), hence bit-identical forward outputs, final T and n_contrib, and
backward gradients equal up to the float atomics' order (the deterministic backward: bit for bit).
Upstream semantics: the per-tile lists of rasterizer_impl.cu (duplicateWithKeys + SortPairs +
identifyTileRanges), ordered by (tile, depth) with ties in Gaussian order."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # CPU container: the driver only runs these on the MI355X box
    pytest.skip("needs a GPU", allow_module_level=True)

import diff_gaussian_rasterization as dgr  # noqa: E402
import synthetic  # noqa: E402
from helpers import small_case  # noqa: E402
from lsr_testutil import decode_img, decode_point_words, grad_err, raster_settings  # noqa: E402


def _render(rss, dev, tile_bucket, order_first=None):
    kw = dict(scales=dev.scales, rotations=dev.rotations, shs=dev.shs)
    side = torch.cuda.Stream() if order_first is not None else None
    pfs = dgr.preprocess_views_native(rss, dev.means3D, dev.opacities, language_feature=dev.lang,
                                      tile_bucket=tile_bucket, order_first=order_first, order_stream=side, **kw)
    if order_first is not None:
        dgr.binning_views_native(pfs[:order_first])
        dgr.binning_views_native(pfs[order_first:])
    else:
        dgr.binning_views_native(pfs)
    return dgr.render_views_native(pfs)


def _case(name):
    if name == "views10":   # an 8-view and a 2-view launch set; view 3 sees nothing (K = 0)
        sc, _ = small_case(P=3000, W=96, H=64, C=6, seed=12, big_frac=0.05)
        cams = synthetic.camera_batch(10, 96, 64, seed=12)
        rss = [raster_settings(c, bg=(0.3, 0.6, 0.9)) for c in cams]
        away = cams[3].world_view_transform.clone()
        away[3, 2] -= 1000.0
        rss[3] = rss[3]._replace(viewmatrix=away.to("cuda"))
        return sc, rss
    if name == "long_buckets":   # 6 tiles, buckets of several thousand: the LDS-chunk + merge fallback
        sc, _ = small_case(P=30000, W=48, H=32, C=4, seed=3, big_frac=0.02, logscale_mean=-3.0)
        cams = synthetic.camera_batch(2, 48, 32, seed=3)
        return sc, [raster_settings(c) for c in cams]
    if name == "headline":   # 1352 x 1014 (5,440 tiles), C = 32
        sc = synthetic.make_scene(300_000, C=32, seed=4)
        cams = synthetic.camera_batch(2, 1352, 1014, seed=4)
        return sc, [raster_settings(c) for c in cams]
    raise ValueError(name)


@pytest.mark.parametrize("name", ["views10", "long_buckets", "headline"])
def test_tile_bucket_lists_equal_sort_path(name):
    sc, rss = _case(name)
    dev = sc.to("cuda")
    ref = _render(rss, dev, False)
    got = _render(rss, dev, True)
    longest = 0
    for v, (a, b) in enumerate(zip(ref, got)):
        sa, sb = a[4], b[4]
        assert sa.num_rendered == sb.num_rendered, v
        for x, y in zip(a[:4], b[:4]):
            assert torch.equal(x, y), v
        ia, ib = decode_img(sa), decode_img(sb)
        for x, y in zip(ia, ib):
            assert np.array_equal(x, y), v
        if sa.num_rendered:
            ranges = ia[0]
            n = int(ranges[:, 1].max())
            assert n > 0
            assert np.array_equal(decode_point_words(sa)[:n], decode_point_words(sb)[:n]), v
            longest = max(longest, int((ranges[:, 1] - ranges[:, 0]).max()))
    if name == "views10":
        assert ref[3][4].num_rendered == 0
    if name == "long_buckets":
        assert longest > 2 * 2048, longest   # at least two merge passes past the LDS chunks
    g = torch.Generator(device="cpu").manual_seed(9)
    H, W = rss[0].image_height, rss[0].image_width
    C = dev.lang.shape[1]
    gcs = [torch.randn(3, H, W, generator=g).cuda() for _ in rss]
    gls = [torch.randn(C, H, W, generator=g).cuda() for _ in rss]
    ga = dgr.backward_views_native([r[4] for r in ref], gcs, gls)
    gb = dgr.backward_views_native([r[4] for r in got], gcs, gls)
    for k in ga:
        if ga[k] is not None:
            assert grad_err(gb[k].cpu().numpy(), ga[k].cpu().numpy()) <= 1e-5, k
    # the deterministic backward addresses its per-(Gaussian, tile) records through the instance
    # offsets, which the two paths make differently (depth-ranked scan scattered by id vs id order)
    for v in range(min(2, len(rss))):
        if ref[v][4].num_rendered == 0:
            continue
        da = dgr.backward_native(ref[v][4], gcs[v], gls[v], deterministic=True)
        db = dgr.backward_native(got[v][4], gcs[v], gls[v], deterministic=True)
        for k in da:
            if da[k] is not None:
                assert torch.equal(da[k], db[k]), (v, k)


def test_tile_bucket_split_scans_and_row_chunks():
    """The instance scans of the later views on a second stream (order_first) and the preprocess in
    row chunks give the same lists as one batch."""
    sc, rss = _case("views10")
    dev = sc.to("cuda")
    ref = _render(rss, dev, True)
    got = _render(rss, dev, True, order_first=3)
    kw = dict(scales=dev.scales, rotations=dev.rotations, shs=dev.shs)
    P = dev.means3D.shape[0]
    chunks = [(0, 1024, None), (1024, 2048, None), (2048, P, None)]
    pfs = dgr.preprocess_views_native(rss, dev.means3D, dev.opacities, language_feature=dev.lang, tile_bucket=True,
                                      row_chunks=chunks, **kw)
    dgr.binning_views_native(pfs)
    rows = dgr.render_views_native(pfs)
    for other in (got, rows):
        for v, (a, b) in enumerate(zip(ref, other)):
            assert a[4].num_rendered == b[4].num_rendered, v
            for x, y in zip(a[:4], b[:4]):
                assert torch.equal(x, y), v
            if a[4].num_rendered:
                n = int(decode_img(a[4])[0][:, 1].max())
                assert np.array_equal(decode_point_words(a[4])[:n], decode_point_words(b[4])[:n]), v


@pytest.mark.parametrize("tile_bucket", [True, False])
def test_row_chunks_rejected_before_any_launch(tile_bucket):
    """Invalid row chunks (a gap, r1 < r0, an unaligned start, short coverage) raise ValueError before
    any preprocess launch or before() wait is enqueued, on both binning paths."""
    sc, rss = _case("views10")
    dev = sc.to("cuda")
    kw = dict(scales=dev.scales, rotations=dev.rotations, shs=dev.shs, language_feature=dev.lang,
              tile_bucket=tile_bucket)
    P = dev.means3D.shape[0]
    called = []
    mark = lambda: called.append(1)   # noqa: E731
    for chunks in ([(0, 1024, mark), (2048, P, mark)], [(0, 1024, mark), (1024, 512, mark), (512, P, mark)],
                   [(0, 1000, mark), (1000, P, mark)], [(0, 1024, mark)]):
        with pytest.raises(ValueError, match="row_chunks"):
            dgr.preprocess_views_native(rss[:2], dev.means3D, dev.opacities, row_chunks=chunks, **kw)
    assert not called


def test_tile_bucket_single_view_render_native():
    """render_native of an unbinned tile-bucket view bins it the tile-bucket way first."""
    sc, rss = _case("views10")
    dev = sc.to("cuda")
    kw = dict(scales=dev.scales, rotations=dev.rotations, shs=dev.shs)
    ref = dgr.forward_native(rss[0], dev.means3D, dev.opacities, language_feature=dev.lang, **kw)
    pf = dgr.preprocess_views_native(rss[:1], dev.means3D, dev.opacities, language_feature=dev.lang,
                                     tile_bucket=True, **kw)[0]
    got = dgr.render_native(pf)
    for x, y in zip(ref[:4], got[:4]):
        assert torch.equal(x, y)
