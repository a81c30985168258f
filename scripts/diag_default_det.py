"""Diagnostic: is the DEFAULT mode (runtime.deterministic=False) bit-reproducible
for E18 / QuickNet gradients now that the split-K reduction defaults to slabs and
the BN-backward sums are fixed-order in every mode?  Prints the number of
differing gradient elements over N repeated forward + backward passes."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tests", "gpu"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import test_determinism as td  # noqa: E402


def main():
    from zookeeper_amd.ops.options import set_options

    set_options(deterministic=False)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    for name, fn in (("e18", td._e18_grads), ("quicknet", td._quicknet_grads)):
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
