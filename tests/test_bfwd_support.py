"""Which convolutions the persistent binary forward (``bfwd.hip``, variant 40
of ``zk_igemm_fwd_fp4``) takes, and that the fp4 forward's default picks it
for exactly the 64 -> 64 / 128 -> 128 stride-1 'same' layers it supports --
host-only queries (dry runs), no GPU needed.  The numerics are pinned on the
GPU by ``tests/gpu/test_fp4_forward.py``."""

import pytest


@pytest.fixture(scope="module")
def lib():
    from zookeeper_amd.ops import _native

    if not _native.available():
        pytest.skip(f"native library not built: {_native.load_error()}")
    return _native.lib()


@pytest.mark.parametrize("B,hw,cin,cout,stride,pad,ok", [
    (1536, 56, 64, 64, 1, 1, True),     # E18 stage 1
    (1536, 28, 128, 128, 1, 1, True),   # E18 stage 2
    (3, 9, 64, 64, 1, 1, True),
    (3, 9, 128, 64, 1, 1, True),        # one 64-channel output slice
    (3, 9, 64, 192, 1, 1, True),        # three slices
    (8, 60, 64, 64, 1, 1, True),        # widest 64-channel image
    (8, 61, 64, 64, 1, 1, False),
    (8, 32, 128, 128, 1, 1, True),      # widest 128-channel image
    (8, 33, 128, 128, 1, 1, False),
    (8, 14, 256, 256, 1, 1, False),     # the weight image would not fit LDS
    (8, 14, 64, 96, 1, 1, False),       # Cout not a multiple of 64
    (8, 28, 64, 128, 2, 0, False),      # stride 2
    (6000, 56, 64, 64, 1, 1, False),    # 2^24 flattened pixels or more
])
def test_bfwd_supported(lib, B, hw, cin, cout, stride, pad, ok):
    assert bool(lib.zk_bfwd_supported(B, hw, hw, cin, cout, 3, 3, stride, pad, pad)) == ok
    ho = (hw + 2 * pad - 3) // stride + 1
    # variant 40 accepts the same set (the igemm dispatch also needs Ho == H)
    v40 = bool(lib.zk_igemm_fwd_supported(B, hw, hw, cin, cout, 3, 3, stride, pad, pad, ho, ho, 0,
                                          40, 1))
    assert v40 == (ok and ho == hw)


def test_default_picks_bfwd_for_e18_stages_1_2(lib):
    # the default (-1) accepts these shapes; variant 40 is what it runs there
    # (the in-step profiles show bfwd_kernel<BfCfg<64, ...>> / <BfCfg<128, ...>>)
    for B, hw, c in [(1536, 56, 64), (1536, 28, 128), (256, 56, 64)]:
        assert lib.zk_igemm_fwd_supported(B, hw, hw, c, c, 3, 3, 1, 1, 1, hw, hw, 0, -1, 1)
        assert lib.zk_igemm_fwd_supported(B, hw, hw, c, c, 3, 3, 1, 1, 1, hw, hw, 0, 40, 1)
