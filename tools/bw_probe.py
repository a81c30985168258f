import torch
n = 512*56*56*256
a = torch.empty(n, dtype=torch.bfloat16, device="cuda")
b = torch.empty(n, dtype=torch.bfloat16, device="cuda")
c = torch.empty(n//4, dtype=torch.bfloat16, device="cuda")
def t(f, reps=10):
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps): f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps
us = t(lambda: a.fill_(1.0)); print(f"fill 822MB: {us:.1f} us {n*2/us/1e6:.2f} TB/s")
us = t(lambda: b.copy_(a)); print(f"copy 822MB: {us:.1f} us {n*4/us/1e6:.2f} TB/s")
us = t(lambda: torch.add(a, b, out=b)); print(f"add (2r+1w): {us:.1f} us {n*6/us/1e6:.2f} TB/s")
us = t(lambda: a.sum()); print(f"sum read 822MB: {us:.1f} us {n*2/us/1e6:.2f} TB/s")
