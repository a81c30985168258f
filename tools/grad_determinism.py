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
    ap.add_argument("--poison", type=int, default=-1,
                    help="before every repeat fill the allocator's free cached memory with this "
                         "byte (255 = NaN in bf16/fp32; -2 = a different byte per repeat): a "
                         "kernel reading memory it does not own then shows up in the gradients")
    ap.add_argument("--trace", action="store_true",
                    help="checksum every module's output and output gradient per repeat and "
                         "print the first ones that differ from repeat 0")
    ap.add_argument("--gc", action="store_true",
                    help="disable Python's cyclic GC and collect before every repeat (the "
                         "allocator then sees the same alloc/free sequence each time)")
    args = ap.parse_args()
    if args.gc:
        import gc

        gc.disable()
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
    trace = []  # per repeat: list of (kind, name, checksum)

    def _cs(t):  # device-side (no host synchronisation inside the step)
        t = t.detach().double()
        return torch.stack([t.sum(), t.abs().sum()])

    if args.trace:
        def fwd_hook(name):
            def h(mod, inp, out):
                if isinstance(out, torch.Tensor):
                    trace[-1].append(("fwd", name, _cs(out)))
                    if out.requires_grad:
                        out.register_hook(lambda g: trace[-1].append(("bwd", name, _cs(g))))
            return h
        for name, mod in model.named_modules():
            if name:
                mod.register_forward_hook(fwd_hook(name))
    def poison(byte):
        res0 = torch.cuda.memory_reserved()
        keep = []
        for sz in (1 << 26, 1 << 22, 1 << 20, 1 << 16, 1 << 12, 1 << 9):
            while True:
                t = torch.empty(sz, dtype=torch.uint8, device=dev)
                if torch.cuda.memory_reserved() > res0:
                    del t  # a new cached segment: the next (smaller) size fills it
                    res0 = torch.cuda.memory_reserved()
                    break
                keep.append(t)
        for t in keep:
            t.fill_(byte)
        n = sum(t.numel() for t in keep)
        del keep
        torch.cuda.synchronize()
        return n

    for rep in range(args.reps):
        if args.poison != -1:
            byte = args.poison if args.poison >= 0 else (37 * rep + 11) % 256
            print(f"rep {rep}: poisoned {poison(byte) / 2**20:.1f} MiB of free memory with {byte}",
                  flush=True)
        if args.gc:
            gc.collect()
        flat.zero_grad()
        trace.append([])
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
    if args.trace:
        for i in range(1, args.reps):
            diffs = [(k, n, a.tolist(), b.tolist()) for (k, n, a), (_, _, b) in zip(trace[0], trace[i])
                     if not torch.equal(a, b)]
            print(f"rep {i}: {len(diffs)} of {len(trace[0])} traced tensors differ from rep 0; "
                  "first ones (in execution order):", flush=True)
            for k, n, a, b in diffs[:12]:
                print(f"    {k} {n}: {a} vs {b}", flush=True)
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
        print(f"rep {i}: above 1e-5:", [(n, f"{r:.1e}") for r, n, gn in rows if r > 1e-5],
              flush=True)


if __name__ == "__main__":
    main()
