"""Error map of the persistent 64 -> 64 binary forward (variant 40) against
the conv3 tile (variant 20) on a small shape: which pixels / channels
differ.  Diagnostic only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from zookeeper_amd.ops._native import lib, stream_ptr  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    hw = int(sys.argv[2]) if len(sys.argv) > 2 else 9
    L, st = lib(), stream_ptr()
    torch.manual_seed(7)
    x = torch.randn(B, hw, hw, 64, device="cuda").to(torch.bfloat16)
    w = torch.randn(64, 3, 3, 64, device="cuda")
    sx4 = torch.empty(B, hw, hw, 32, dtype=torch.uint8, device="cuda")
    L.zk_sign_pack(x.data_ptr(), None, None, None, sx4.data_ptr(), x.numel() // 32, 1.0, st)
    wf4 = torch.empty(9, 64, 32, dtype=torch.uint8, device="cuda")
    L.zk_weight_pack(w.data_ptr(), None, None, None, None, wf4.data_ptr(), 64, 9, 64, st)
    ys = {}
    for v in (20, 40):
        y = torch.full((B, hw, hw, 64), -12345, dtype=torch.int16, device="cuda")
        stats = torch.zeros(2, 64, dtype=torch.int64, device="cuda")
        rc = L.zk_igemm_fwd_fp4(sx4.data_ptr(), wf4.data_ptr(), y.data_ptr(), stats.data_ptr(), B,
                                hw, hw, 64, 64, 3, 3, 1, 1, 1, hw, hw, 0, 0, v, 1, st)
        torch.cuda.synchronize()
        assert rc == 0, rc
        ys[v] = (y.reshape(-1, 64).long().cpu(), stats.cpu())
    a, b = ys[20][0], ys[40][0]
    bad = (a != b)
    print("bad elements", int(bad.sum()), "of", bad.numel())
    pix = bad.any(1).nonzero().flatten().tolist()
    ch = bad.any(0).nonzero().flatten().tolist()
    print("bad pixels", len(pix), pix[:64])
    print("bad channels", len(ch), ch)
    for p in pix[:4]:
        print(p, "ref", a[p, :16].tolist())
        print(p, "got", b[p, :16].tolist())
    print("stats equal", torch.equal(ys[20][1], ys[40][1]))


if __name__ == "__main__":
    main()
