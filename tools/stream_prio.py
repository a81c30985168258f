"""Print the HIP stream priority range torch exposes on this device."""
import torch

if __name__ == "__main__":
    print("priority_range", torch.cuda.Stream.priority_range())
    for p in (-2, -1, 0, 1):
        s = torch.cuda.Stream(priority=p)
        print("requested", p, "got", s.priority)
