"""Loader for the in-tree native library ``zookeeper_amd/_zkamd.so``.

The library holds the hand-written HIP kernels for gfx950 and the C++ runtime
pieces (pinned host ring / gather pool).  It exports a plain C ABI — every
entry point takes raw device pointers, sizes and a ``hipStream_t`` — and is
bound with ``ctypes``.  The library links against ``libamdhip64.so.7``; torch
is imported first so the process shares torch's already-loaded HIP runtime
(same SONAME) and kernels launch on torch's current stream.

Build: ``python -m zookeeper_amd.csrc.build`` (or ``__graft_entry__.build()``).

If a GPU is present but the library is missing or fails to load, ``lib()``
raises: GPU code paths never fall back silently.  Set ``ZK_NATIVE=0`` to
force the pure-PyTorch path deliberately.

Provenance: the build embeds a digest of every kernel / runtime source and
header (``zk_build_digest``, ``csrc/build.py:source_digest``).  A library
whose digest differs from the sources next to it is refused (not loaded):
a stale ``.so`` cannot run kernels other than the ones in the tree.
"""

from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_HERE, "_zkamd.so")

_lib: Optional[ctypes.CDLL] = None
_load_error: Optional[str] = None
_tried = False


def _declare(lib: ctypes.CDLL) -> None:
    from zookeeper_amd.ops import _signatures

    for name, (restype, argtypes) in _signatures.SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = restype
        fn.argtypes = argtypes


def _load() -> None:
    global _lib, _load_error, _tried
    if _tried:
        return
    _tried = True
    if os.environ.get("ZK_NATIVE", "1") == "0":
        _load_error = "disabled by ZK_NATIVE=0"
        return
    if not os.path.exists(LIB_PATH):
        _load_error = f"{LIB_PATH} not built (run `python -m zookeeper_amd.csrc.build`)"
        return
    try:
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:
        _load_error = str(e)
        return
    stale = _digest_mismatch(lib)
    if stale:
        _load_error = stale
        return
    _declare(lib)
    _lib = lib


def _digest_mismatch(lib: ctypes.CDLL) -> Optional[str]:
    """Why ``lib`` does not match the sources in the tree, or None."""
    from zookeeper_amd.csrc import build as _build

    tree = _build.source_digest()
    if tree is None:  # no sources shipped next to the package: nothing to compare
        return None
    fn = getattr(lib, "zk_build_digest", None)
    if fn is None:
        return f"{LIB_PATH} has no build digest (built before provenance checks); rebuild it"
    fn.restype = ctypes.c_char_p
    fn.argtypes = []
    built = fn().decode()
    if built != tree:
        return (f"{LIB_PATH} is stale: built from sources with digest {built[:16]}, the tree has "
                f"{tree[:16]} (run `python -m zookeeper_amd.csrc.build`)")
    return None


def build_digest() -> Optional[str]:
    """The source digest the loaded library was built from (None: not loaded)."""
    if not available():
        return None
    return _lib.zk_build_digest().decode()


def native_disabled() -> bool:
    """True if the native path was switched off on purpose (``ZK_NATIVE=0``)."""
    return os.environ.get("ZK_NATIVE", "1") == "0"


def available() -> bool:
    """True if the native library is loaded (GPU kernels need a GPU too)."""
    _load()
    return _lib is not None


def load_error() -> Optional[str]:
    _load()
    return _load_error


def lib() -> ctypes.CDLL:
    _load()
    if _lib is None:
        raise RuntimeError(f"zookeeper_amd native library unavailable: {_load_error}")
    return _lib


def stream_ptr(device: Optional[torch.device] = None) -> int:
    """Raw ``hipStream_t`` of torch's current stream."""
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


def direct_grad(p, channels_last: bool = False):
    """The gradient buffer a kernel may accumulate into directly, or None.

    Parameters managed by :class:`~zookeeper_amd.parallel.flat.FlatParams`
    carry ``_zk_direct_grad``: their ``.grad`` is a view into the flat fp32
    gradient buffer, zeroed once per step.  Kernels then add their
    contribution in place (no temporary, no framework accumulate kernel) and
    call :func:`grad_ready`; the autograd function returns ``None`` for them.
    """
    if p is None or not getattr(p, "_zk_direct_grad", False):
        return None
    g = p.grad
    if g is None or g.dtype != torch.float32:
        return None
    if channels_last and not g.is_contiguous(memory_format=torch.channels_last):
        return None
    if not channels_last and not g.is_contiguous():
        return None
    # claimed for this step: the data-parallel bucketer then ignores autograd's
    # post-accumulate call for p (it runs even though the op returns None) and
    # waits for the kernel's own grad_ready
    p._zk_direct_claim = True
    return g


def zeroed_scratch(owner, name: str, shape, dtype: torch.dtype,
                   device: torch.device) -> torch.Tensor:
    """A persistent accumulator kept on ``owner`` (a module), zero when handed
    out.  Only for accumulators whose consuming kernel re-zeroes them after
    reading (BN ``stats`` → ``zk_bn_finalize`` / ``zk_bn_finalize_f64``,
    BN-backward ``sums`` → ``zk_bn_bwd_coef``): that replaces a fill kernel
    per layer and step.  The owner's ``__dict__`` holds it, so it is not
    part of ``state_dict``."""
    cache = owner.__dict__.setdefault("_zk_scratch", {})
    shape = tuple(shape)
    buf = cache.get(name)
    if buf is None or buf.shape != shape or buf.dtype != dtype or buf.device != device:
        buf = torch.zeros(shape, dtype=dtype, device=device)
        cache[name] = buf
    return buf


# Arrival counters of the in-launch split-K trees (zk_wgrad_rows), one buffer
# per (device, stream): launches on one stream never overlap and every launch
# leaves its counters zero, so a stream's launches can share one buffer.
_COUNTERS: Dict[Tuple[int, int], torch.Tensor] = {}
_OLD_COUNTERS: List[torch.Tensor] = []  # outgrown buffers (queued kernels may still use them)


def tree_counters(nbytes: int, device: torch.device, stream: int) -> torch.Tensor:
    key = (device.index if device.index is not None else torch.cuda.current_device(), stream)
    buf = _COUNTERS.get(key)
    if buf is None or buf.numel() * 4 < nbytes:
        if buf is not None:
            _OLD_COUNTERS.append(buf)
        n = max(1024, (nbytes + 3) // 4)
        buf = torch.empty(n, dtype=torch.int32, device=device)
        check(lib().zk_zero(buf.data_ptr(), n * 4, stream), "zk_zero")
        _COUNTERS[key] = buf
    return buf


def wgrad_rows_ok(geom) -> bool:
    """Whether ``zk_wgrad_rows`` (row-streaming 3x3 weight gradient with the
    in-launch fixed-order split-K tree) takes this layer."""
    from zookeeper_amd.ops.options import OPTS

    B, H, W, Cin, Ho, Wo, Cout, kh, kw, s, pt, pl = geom
    if not (OPTS.wgrad_rows and kh == 3 and kw == 3 and s == 1 and pt == 1 and pl == 1
            and Ho == H and Wo == W):
        return False
    return lib().zk_wgrad_rows_plan(B, H, W, Cin, Cout, 0, None, None) == 0


_WGRAD_OPERANDS = {"image": 0, "sign": 1, "fp4": 2}


def igemm_wgrad(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, dw: torch.Tensor,
                geom, pad_ones: int, clip: float, stream: int, what: str = "zk_igemm_wgrad",
                variant: int = -1, operand: str = "image") -> None:
    """Implicit-GEMM weight gradient ``dw += mask(|w| <= clip) * dyᵀ ⊛ x``.

    * 3x3 stride-1 layers the row-streaming kernel takes (``wgrad_rows_ok``):
      ``zk_wgrad_rows``, split-K combined inside the launch by a fixed-order
      tree (no reduce launch);
    * otherwise ``zk_igemm_wgrad``: per-split slabs (plain stores) summed in a
      fixed order by ``wgrad_reduce_kernel``.

    Both are bit-reproducible.  ``operand``: ``"image"`` (``x`` is a bf16
    image: the +-1 sign image or a float activation), ``"sign"`` (``x`` is
    the bf16 activation and the kernel takes its sign; needs pad_ones) or
    ``"fp4"`` (``x`` is the e2m1 sign image [B][H][W][Cin/2]); the last two
    only on ``zk_wgrad_rows``.
    ``geom`` = (B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl)."""
    L = lib()
    B, H, W, Cin, Ho, Wo, Cout, kh, kw, s, pt, pl = geom
    op = _WGRAD_OPERANDS.get(operand)
    if op is None:
        raise ValueError(f"{what}: unknown operand {operand!r}")
    if variant < 0 and wgrad_rows_ok(geom) and (pad_ones or op != 1):
        sb, cb = ctypes.c_int64(0), ctypes.c_int64(0)
        check(L.zk_wgrad_rows_plan(B, H, W, Cin, Cout, 0, ctypes.byref(sb), ctypes.byref(cb)),
              what + " (plan)")
        slab = (torch.empty(sb.value // 4, dtype=torch.float32, device=dy.device)
                if sb.value > 0 else None)
        cnt = tree_counters(cb.value, dy.device, stream) if cb.value > 0 else None
        check(L.zk_wgrad_rows(dy.data_ptr(), x.data_ptr(), w.data_ptr() if w is not None else None,
                              dw.data_ptr(), slab.data_ptr() if slab is not None else None,
                              sb.value, cnt.data_ptr() if cnt is not None else None, cb.value,
                              B, H, W, Cin, Cout, int(pad_ones), op, float(clip), 0,
                              stream), what)
        return
    if op:
        raise ValueError(f"{what}: the {operand!r} operand needs zk_wgrad_rows")
    ws, ws_bytes = None, 0
    ws_bytes = max(int(L.zk_igemm_wgrad_ws_bytes(B, Cin, H, W, Ho, Wo, Cout, kh, kw, s, pt,
                                                 pl, 0, variant)), 0)
    if ws_bytes > 0:
        ws = torch.empty(ws_bytes // 4, dtype=torch.float32, device=dy.device)
    check(L.zk_igemm_wgrad(dy.data_ptr(), x.data_ptr(), w.data_ptr(), dw.data_ptr(), B, H, W,
                           Cin, Ho, Wo, Cout, kh, kw, s, pt, pl, int(pad_ones), float(clip), 0,
                           variant, ws.data_ptr() if ws is not None else None, ws_bytes, stream),
          what)


def slab_reduce() -> bool:
    """Split-K weight gradients through per-split slabs and a fixed-order
    reduce rather than fp32 atomics: the policy of every weight-gradient op
    (igemm, small-K convs, depthwise, stem), in every mode (fp32-atomic
    reductions measured slower in the E18 step and were removed,
    profiles/r4/removed_variants.md)."""
    return True


def zeroed(shape, device, dtype=torch.float32) -> torch.Tensor:
    """A zero-filled scratch tensor cleared by a runtime memset (no framework
    fill kernel in the training step)."""
    t = torch.empty(shape, dtype=dtype, device=device)
    if t.is_cuda and available():
        check(lib().zk_zero(t.data_ptr(), t.numel() * t.element_size(), stream_ptr(t.device)),
              "zk_zero")
    else:
        t.zero_()
    return t


def grad_ready(p) -> None:
    """Tell the data-parallel bucketer that ``p``'s gradient is complete."""
    cb = getattr(p, "_zk_grad_ready", None)
    if cb is not None:
        cb()


# ZK_DEBUG_SYNC=1: synchronise the device after every native launch so a
# kernel fault is reported at the launch that caused it (debugging only);
# ZK_DEBUG_SYNC=a,b: only after launches whose name contains a or b.
_DEBUG_SYNC_ENV = os.environ.get("ZK_DEBUG_SYNC", "0")
_DEBUG_SYNC = _DEBUG_SYNC_ENV not in ("", "0")
_DEBUG_SYNC_ONLY = (tuple(x for x in _DEBUG_SYNC_ENV.split(",") if x)
                    if _DEBUG_SYNC_ENV not in ("", "0", "1") else ())


def check(code: int, what: str = "kernel") -> None:
    if code != 0:
        raise RuntimeError(f"{what} failed with hipError {code}")
    if _DEBUG_SYNC and (not _DEBUG_SYNC_ONLY or any(x in what for x in _DEBUG_SYNC_ONLY)):
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:
            raise RuntimeError(f"{what}: device error after the launch: {e}") from None
        log = os.environ.get("ZK_DEBUG_SYNC_LOG")
        if log:
            with open(log, "a") as f:
                f.write(f"ok {what}\n")


def gather_rows(src: np.ndarray, idx: np.ndarray, dst: torch.Tensor, threads: int = 8) -> None:
    """Native multi-threaded row gather ``dst[i] = src[idx[i]]`` (host memory)."""
    l = lib()
    src = np.ascontiguousarray(src) if not src.flags.c_contiguous else src
    idx64 = np.ascontiguousarray(idx, dtype=np.int64)
    row_bytes = int(np.prod(src.shape[1:])) * src.itemsize
    rc = l.zk_gather_rows(
        src.ctypes.data, ctypes.c_int64(row_bytes), idx64.ctypes.data,
        ctypes.c_int64(len(idx64)), ctypes.c_void_p(dst.data_ptr()), ctypes.c_int(threads),
    )
    if rc != 0:
        raise RuntimeError(f"zk_gather_rows failed with code {rc}")
