"""Count the GPUs a job may use WITHOUT touching the HIP runtime.

Launcher parents (``bench.py --gpus N``, ``sweep``, ``--nproc``) fork rank
processes; they must never initialise the GPU themselves (a HIP-initialised
parent that forks, or execs, is unsafe on this pool).  On torch 2.10+rocm7.0
``torch.cuda.device_count()`` goes through amdsmi and falls back to
``hipGetDeviceCount`` -- a runtime init -- when amdsmi fails, so the count
comes from the environment and the kernel driver's sysfs topology instead:

* ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``
  (the first one set wins; an empty value means no device);
* otherwise the KFD topology: every ``/sys/class/kfd/kfd/topology/nodes/*``
  with a non-zero ``gpu_id`` is a GPU (CPU nodes report 0).
"""

from __future__ import annotations

import glob
import os
from typing import List, Optional

_VIS_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
_KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _parse_visible(val: str) -> List[str]:
    return [v.strip() for v in val.split(",") if v.strip()]


def kfd_gpu_count(root: str = _KFD_NODES) -> int:
    n = 0
    for node in glob.glob(os.path.join(root, "*")):
        try:
            with open(os.path.join(node, "gpu_id")) as f:
                if int(f.read().strip() or "0") != 0:
                    n += 1
        except (OSError, ValueError):
            continue
    return n


def visible_gpu_count(env: Optional[dict] = None, kfd_root: str = _KFD_NODES) -> int:
    """Number of GPUs this process would see, from env + sysfs only."""
    env = os.environ if env is None else env
    physical = kfd_gpu_count(kfd_root)
    for var in _VIS_VARS:
        if var in env:
            ids = _parse_visible(env[var])
            return min(len(ids), physical) if physical else len(ids)
    return physical


def visible_gpu_ids(env: Optional[dict] = None, kfd_root: str = _KFD_NODES) -> List[str]:
    """The device ids a launcher may hand out (``HIP_VISIBLE_DEVICES``
    entries if set, else ``0..n-1``)."""
    env = os.environ if env is None else env
    for var in _VIS_VARS:
        if var in env:
            return _parse_visible(env[var])
    return [str(i) for i in range(kfd_gpu_count(kfd_root))]


# Hardware queues per process (HIP's GPU_MAX_HW_QUEUES; HIP's default is 4).
# A training step here uses more streams than that -- compute, the
# weight-gradient side stream(s), the loader's copy stream, the gradient
# all-reduce's comm stream and RCCL's own -- and HIP maps streams onto the
# hardware queues round-robin.  A stream wait is a barrier packet in its
# queue, so two streams sharing a queue serialise: with 4 queues the comm
# stream's wait for the last gradient bucket (enqueued early, satisfied only
# at the end of the backward) held the loader's H2D copy of the next batch
# behind it, and the next forward waited for its input -- E18 b1536 with the
# bucketed all-reduce on (one rank, forced DP): 32.1-34.2 ms/step at 4
# queues, 32.4-33.6 at 8, 27.7 at 16 (= without DP: the device-resident data
# path, which has no copy stream, showed no DP cost at all).
HW_QUEUES = 16


def configure_hw_queues(n: int = HW_QUEUES) -> str:
    """Raise ``GPU_MAX_HW_QUEUES`` to at least ``n`` for this process (the
    MI355X boxes export HIP's default, 4, explicitly); ``ZK_HW_QUEUES`` picks
    an exact value instead.  Effective only before the HIP runtime
    initialises (call before the first GPU use; rank processes inherit it).
    Returns the value in effect."""
    want = os.environ.get("ZK_HW_QUEUES")
    cur = os.environ.get("GPU_MAX_HW_QUEUES")
    if want:
        os.environ["GPU_MAX_HW_QUEUES"] = str(int(want))
    elif cur is None or not cur.strip().isdigit() or int(cur) < n:
        os.environ["GPU_MAX_HW_QUEUES"] = str(int(n))
    return os.environ["GPU_MAX_HW_QUEUES"]
