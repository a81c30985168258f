"""Keep the GPU busy for ``seconds`` (matmul loop): a background load for
race diagnostics (scripts/diag_dp.py DIAG_BURN=1)."""
import sys
import time

import torch

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
t0 = time.time()
while time.time() - t0 < secs:
    for _ in range(20):
        b = a @ a
    torch.cuda.synchronize()
