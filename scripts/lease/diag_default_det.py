"""Diagnostic: is the DEFAULT mode (runtime.deterministic=False) bit-reproducible
for E18 / QuickNet gradients now that the split-K reduction defaults to slabs and
the BN-backward sums are fixed-order in every mode?  Prints the number of
differing gradient elements over N repeated forward + backward passes."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "tests", "gpu"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import test_determinism as td  # noqa: E402


def _resnet_grads(steps_x, model_seed=1234):
    from zookeeper_amd.models.resnet import ResNetModule
    from zookeeper_amd.ops import streams
    from zookeeper_amd.parallel.flat import FlatParams
    from zookeeper_amd.train.losses import get_loss
    from zookeeper_amd.train.trainer import prepare_model

    torch.manual_seed(model_seed)
    dev = torch.device("cuda", 0)
    model = prepare_model(ResNetModule((64, 64, 3), 10, blocks=(1, 1, 1, 1)), dev).train()
    flat = FlatParams(model, dev)
    loss_fn = get_loss("sparse_categorical_crossentropy")
    x, y = steps_x
    flat.zero_grad()
    loss, _ = loss_fn(model(x), y)
    with streams.session(dev):
        loss.backward()
    torch.cuda.synchronize()
    return loss.detach().clone(), flat.grad.clone(), [b.clone() for b in model.buffers()]


def main():
    from zookeeper_amd.ops.options import set_options

    set_options(deterministic=False)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    for name, fn in (("e18", td._e18_grads), ("quicknet", td._quicknet_grads),
                     ("resnet", _resnet_grads)):
        batch = td._batch()
        l0, g0, _ = fn(batch)
        worst = 0
        for _ in range(reps):
            l1, g1, _ = fn(batch)
            worst = max(worst, int((g0 != g1).sum().item()))
        print(f"{name}: default mode, {reps} repeats: max differing gradient elements {worst} "
              f"of {g0.numel()}; loss equal {bool(torch.equal(l0, l1))}", flush=True)


if __name__ == "__main__":
    main()
