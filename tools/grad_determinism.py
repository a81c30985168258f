"""Run the same forward + backward of a model several times from the same
state (one process, the HIP path) and report per-parameter gradient
differences between the repeats.  fp32 atomics in the split-K / statistics
reductions make the gradients vary in the last bits; anything larger points
at a race.

    python tools/grad_determinism.py [--model BinaryResNetE18] [--hw 64] [--batch 4] [--reps 4]
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", type=int, default=64)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--freeze", default="", help="comma list of parameter names to freeze")
    ap.add_argument("--no-handoff", action="store_true",
                    help="stem does not hand its sign images to the first block")
    args = ap.parse_args()
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.parallel.flat import FlatParams
    from zookeeper_amd.train.losses import get_loss
    from zookeeper_amd.train.trainer import prepare_model

    torch.manual_seed(1234)
    dev = torch.device("cuda", 0)
    model = prepare_model(BinaryResNetE((args.hw, args.hw, 3), 10, 18, backend="hip"), dev)
    model.train()
    if args.no_handoff:
        model.stem.sign_clip = None
    for n, p_ in model.named_parameters():
        if n in args.freeze.split(","):
            p_.requires_grad_(False)
    flat = FlatParams(model, dev)
    loss_fn = get_loss("sparse_categorical_crossentropy")
    g = torch.Generator().manual_seed(99)
    x = torch.randn(args.batch, 3, args.hw, args.hw, generator=g).to(dev, torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (args.batch,), generator=g).to(dev)
    grads, logits, stem_out = [], [], []
    model.stem.register_forward_hook(lambda m, i, o: stem_out.append(o.detach().clone()))
    for _ in range(args.reps):
        flat.zero_grad()
        out = model(x)
        logits.append(out.detach().float().clone())
        loss, _ = loss_fn(out, y)
        loss.backward()
        torch.cuda.synchronize()
        grads.append(flat.grad.clone())
    for i in range(1, args.reps):
        print(f"rep {i}: logits max |diff| vs rep 0: {(logits[i] - logits[0]).abs().max().item():.3g}"
              f"  stem output: {(stem_out[i].float() - stem_out[0].float()).abs().max().item():.3g}",
              flush=True)
    ref = grads[0]
    for i, gi in enumerate(grads[1:], 1):
        rows = []
        for s in flat.slots:
            a = gi[s.offset:s.offset + s.numel]
            b = ref[s.offset:s.offset + s.numel]
            rel = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
            rows.append((rel, s.name, b.norm().item()))
        rows.sort(reverse=True)
        print(f"rep {i}: worst", [(n, f"{r:.2e}", f"|g|={gn:.2e}") for r, n, gn in rows[:6]],
              flush=True)


if __name__ == "__main__":
    main()
