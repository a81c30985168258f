"""The GPU kernel tests enumerate only valid (tile variant, shape) pairs at
collection time (tests/tile_support.py); this pins that Python mirror to the
native launchers' own validation (``zk_igemm_*_supported``: host-only dry
runs, no GPU needed) and states the rejected combinations explicitly."""

import itertools

import pytest

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import tile_support as ts  # noqa: E402

SHAPES = [(cin, cout, s, hw) for cin, cout in itertools.product([64, 128, 192, 256, 512], repeat=2)
          for s, hw in [(1, 7), (1, 12), (2, 12), (2, 9)]]


@pytest.fixture(scope="module")
def lib():
    from zookeeper_amd.ops import _native

    if not _native.available():
        pytest.skip(f"native library not built: {_native.load_error()}")
    return _native.lib()


def _geom(cin, cout, s, hw):
    from zookeeper_amd.nn.layers import same_padding

    pt, pb = same_padding(hw, 3, s)
    ho = (hw + pt + pb - 3) // s + 1
    return pt, ho


def test_dgrad_rule_matches_native(lib):
    for (cin, cout, s, hw), v in itertools.product(SHAPES, ts.DGRAD):
        pt, ho = _geom(cin, cout, s, hw)
        native = bool(lib.zk_igemm_dgrad_supported(3, hw, hw, cin, ho, ho, cout, 3, 3, s, pt, pt, v))
        assert native == ts.dgrad_ok(v, cin, cout, s), (v, cin, cout, s, hw)


def test_fwd_rule_matches_native(lib):
    for (cin, cout, s, hw), v in itertools.product(SHAPES, ts.FWD):
        pt, ho = _geom(cin, cout, s, hw)
        native = bool(lib.zk_igemm_fwd_supported(3, hw, hw, cin, cout, 3, 3, s, pt, pt, ho, ho, 0,
                                                 v, 0))
        assert native == ts.fwd_ok(v, cin, cout, s), (v, cin, cout, s, hw)


def test_wgrad_rule_matches_native(lib):
    for (cin, cout, s, hw), v in itertools.product(SHAPES, list(ts.WGRAD) + [31]):
        pt, ho = _geom(cin, cout, s, hw)
        native = lib.zk_igemm_wgrad_ws_bytes(3, cin, hw, hw, ho, ho, cout, 3, 3, s, pt, pt, 256,
                                             v) >= 0
        assert native == ts.wgrad_ok(v, cin, cout, s), (v, cin, cout, s, hw)


def test_rejected_sets_are_the_expected_ones():
    """The combinations the GPU tests no longer generate, stated by rule:
    conv3 tiles (variant >= 20) need stride 1; a tile must divide the GEMM N
    (Cin for dgrad, Cout for fwd / wgrad); the row-window dgrad (variant 50)
    takes 64 -> 64 channels only."""
    shapes = [(64, 64, 1), (64, 128, 2), (128, 128, 1), (256, 512, 2), (128, 64, 1),
              (128, 256, 2), (64, 64, 1), (256, 256, 1)]
    for v, cin, cout, s in ts.rejected(ts.dgrad_ok, ts.DGRAD, shapes):
        bn, _, c3 = ts.DGRAD[v]
        if v == 50:  # the row-window kernel: 64 -> 64 channels only
            assert s != 1 or (cin, cout) != (64, 64)
            continue
        assert (c3 and s != 1) or cin % bn != 0
    for v, cin, cout, s in ts.rejected(ts.wgrad_ok, ts.WGRAD, shapes):
        bm, bn, c3 = ts.WGRAD[v]
        if v == 51:  # the row-window kernel: Cin = Cout in {64, ..., 512} only
            assert s != 1 or cin != cout
            continue
        assert (c3 and s != 1) or cout % bm != 0 or (cin if c3 else 9 * cin) % bn != 0
    # every variant is exercised by at least one generated shape
    assert {p[0] for p in ts.pairs(ts.dgrad_ok, ts.DGRAD, shapes)} == set(ts.DGRAD)
