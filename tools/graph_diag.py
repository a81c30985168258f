"""Compare the HIP-graph replay of forward + backward with the eager run on
the same inputs and parameters (SGD with lr 0, so nothing moves): prints the
loss of both and the parameters whose gradients differ most.

    python tools/graph_diag.py [--hw 64] [--batch 8]
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", type=int, default=64)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--replays", type=int, default=6)
    args = ap.parse_args()
    from zookeeper_amd.core import configure
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.parallel import dist as zdist
    from zookeeper_amd.train import SGD, Trainer

    info = zdist.init()
    torch.manual_seed(1234)
    model = BinaryResNetE((args.hw, args.hw, 3), 10, 18, backend="hip")
    spec = SGD()
    configure(spec, {"learning_rate": 0.0, "momentum": 0.0})
    tr = Trainer(model, "sparse_categorical_crossentropy", spec, info, graph=True, graph_warmup=2)
    g = torch.Generator().manual_seed(3)

    def batch():
        x = torch.randn(args.batch, 3, args.hw, args.hw, generator=g).to(info.device, torch.bfloat16)
        y = torch.randint(0, 10, (args.batch,), generator=g).to(info.device)
        return x.contiguous(memory_format=torch.channels_last), y

    x0, y0 = batch()
    for _ in range(2):
        tr.train_step(x0, y0)
    for it in range(args.replays):
        x, y = batch()
        lg, _ = tr.train_step(x, y)
        lg = float(lg)
        gg = tr.flat.grad.clone()
        le, _ = tr._forward_backward(x, y)
        torch.cuda.synchronize()
        ge = tr.flat.grad.clone()
        rows = []
        for s in tr.flat.slots:
            a = gg[s.offset:s.offset + s.numel]
            b = ge[s.offset:s.offset + s.numel]
            rows.append((((a - b).norm() / b.norm().clamp_min(1e-30)).item(), s.name,
                         b.norm().item(), a.norm().item()))
        rows.sort(reverse=True)
        tot = ((gg - ge).norm() / ge.norm()).item()
        print(f"replay {it}: loss graph {lg:.6f} eager {float(le):.6f} grad rel {tot:.2e}",
              flush=True)
        for r, n, bn, an in rows[:8]:
            print(f"    {n:40s} rel {r:.2e} |eager| {bn:.3e} |graph| {an:.3e}", flush=True)


if __name__ == "__main__":
    main()
