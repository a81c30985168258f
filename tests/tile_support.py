"""Which implicit-GEMM tile variants (``igemm.hip``) accept which conv
geometry — a Python mirror of the launchers' validation, so the GPU kernel
tests generate only valid (variant, shape) pairs at collection time instead
of skipping at run time.  ``tests/test_tile_support.py`` checks this mirror
against the library's own ``zk_igemm_*_supported`` / ``zk_igemm_wgrad_ws_bytes``
queries (host-only, no GPU) over a grid of shapes.

Geometry of a 3x3 'same' conv (the only kind these tests build):
``pt = pl = (stride == 1) ? 1 : same_padding(...)``.
"""

from __future__ import annotations

from typing import Dict, Iterable, List, Tuple

# dgrad: variant -> (BN = Cin tile, CB = K bytes per stage row, conv3 family)
DGRAD: Dict[int, Tuple[int, int, bool]] = {
    0: (128, 128, False), 1: (128, 64, False), 2: (128, 128, False), 3: (256, 128, False),
    4: (64, 128, False), 5: (64, 128, False), 6: (64, 128, False), 7: (64, 64, False),
    8: (64, 64, False), 9: (64, 128, False), 10: (128, 128, False), 11: (128, 64, False),
    12: (256, 64, False), 13: (256, 64, False), 14: (256, 128, False),
    15: (256, 64, False), 16: (128, 64, False), 17: (256, 64, False),
    20: (64, 128, True), 21: (64, 64, True), 22: (64, 128, True), 23: (128, 64, True),
    24: (128, 64, True), 25: (256, 64, True), 26: (128, 64, True), 27: (64, 64, True),
    28: (64, 32, True), 29: (64, 32, True), 30: (64, 32, True),
    32: (64, 64, True), 33: (128, 32, True), 34: (128, 32, True),
    # row-window kernel (conv3rw.hip): 64 -> 64 only, stride 1
    50: (64, 64, True),
    # phased 256x256 kernel (deep_gemm.hip): Cin % 256 == 0
    60: (256, 128, True),
    # LDS-staged (coalesced) epilogue variants
    40: (128, 128, False), 41: (128, 64, False), 42: (64, 128, False), 43: (64, 64, False),
    44: (128, 128, False), 45: (256, 128, False), 46: (128, 64, False), 47: (256, 64, False),
    48: (64, 128, False),
}

# bf16 forward: variant -> (BN = Cout tile, CB, conv3)
FWD: Dict[int, Tuple[int, int, bool]] = {
    0: (128, 128, False), 1: (128, 64, False), 2: (128, 128, False), 3: (256, 128, False),
    4: (64, 128, False), 5: (64, 128, False), 6: (64, 128, False), 7: (64, 64, False),
    8: (64, 64, False), 9: (64, 128, False), 10: (128, 128, False), 11: (128, 64, False),
    12: (256, 64, False), 13: (256, 64, False), 14: (256, 128, False),
    20: (64, 128, True), 21: (64, 64, True), 22: (64, 128, True), 23: (128, 64, True),
    24: (128, 64, True), 25: (256, 64, True), 26: (128, 64, True), 27: (64, 64, True),
}

# wgrad: variant -> (BM = Cout tile, BN = K tile (taps*Cin or Cin for conv3), conv3);
# variant 31 does not exist (always rejected).
WGRAD: Dict[int, Tuple[int, int, bool]] = {
    0: (128, 128, False), 1: (128, 128, False), 2: (128, 192, False), 3: (64, 192, False),
    4: (128, 128, False), 5: (64, 128, False), 6: (128, 256, False), 7: (64, 64, False),
    8: (256, 256, False), 9: (256, 256, False), 10: (256, 128, False), 11: (128, 256, False),
    12: (256, 256, False),
    20: (64, 64, True), 21: (64, 64, True), 22: (128, 64, True), 23: (128, 128, True),
    24: (64, 128, True), 25: (64, 64, True), 26: (128, 128, True), 27: (64, 64, True),
    28: (128, 64, True), 29: (64, 64, True), 30: (64, 64, True), 32: (128, 64, True),
    33: (64, 64, True), 34: (128, 64, True),
    # phased 256x256 kernel (deep_gemm.hip): stride 1, Cin and Cout % 256 == 0
    60: (256, 256, True),
}


def same_pad(hw: int, stride: int) -> Tuple[int, int]:
    out = -(-hw // stride)
    total = max((out - 1) * stride + 3 - hw, 0)
    return total // 2, out


def conv3_ok(stride: int) -> bool:  # 3x3 'same' geometry is implied
    return stride == 1


def dgrad_ok(v: int, cin: int, cout: int, stride: int) -> bool:
    if v not in DGRAD:
        return False
    bn, cb, c3 = DGRAD[v]
    if v == 50:
        return stride == 1 and cin == 64 and cout == 64
    if v == 60:
        return stride <= 2 and cin % 256 == 0 and cout % 64 == 0
    if c3 and not conv3_ok(stride):
        return False
    return (2 * cout) % cb == 0 and cin % bn == 0 and stride <= 2


def fwd_ok(v: int, cin: int, cout: int, stride: int) -> bool:
    if v not in FWD:
        return False
    bn, cb, c3 = FWD[v]
    if c3 and not conv3_ok(stride):
        return False
    return (2 * cin) % cb == 0 and cout % bn == 0


def wgrad_ok(v: int, cin: int, cout: int, stride: int) -> bool:
    if v not in WGRAD:
        return False
    bm, bn, c3 = WGRAD[v]
    if v == 60:
        return stride == 1 and cin % 256 == 0 and cout % 256 == 0
    if c3:
        return conv3_ok(stride) and cout % bm == 0 and cin % bn == 0
    return cout % bm == 0 and (9 * cin) % bn == 0 and cin % 8 == 0


def pairs(rule, variants: Iterable[int], shapes: Iterable[tuple], key=lambda s: s[:3]) -> List[tuple]:
    """``(variant, *shape)`` for every pair the rule accepts (``key`` picks
    ``(cin, cout, stride)`` out of a shape tuple)."""
    return [(v, *s) for s in shapes for v in variants if rule(v, *key(s))]


def rejected(rule, variants: Iterable[int], shapes: Iterable[tuple], key=lambda s: s[:3]):
    return [(v, *s) for s in shapes for v in variants if not rule(v, *key(s))]
