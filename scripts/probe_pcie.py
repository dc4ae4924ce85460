"""Diagnostics: pinned-host <-> device copy rates, one direction at a time and both directions
at once on two streams (does this box overlap H2D with D2H?)."""
import time

import torch

n = 160 * 1024 * 1024
h_in = torch.empty(n, dtype=torch.uint8).pin_memory()
h_out = torch.empty(n, dtype=torch.uint8).pin_memory()
d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
d_out = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def h2d():
    with torch.cuda.stream(s1):
        d_in.copy_(h_in, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h_out.copy_(d_out, non_blocking=True)


def both():
    h2d()
    d2h()


a, b, c = t(h2d), t(d2h), t(both)
print(f"H2D {n / a / 1e9:.1f} GB/s  D2H {n / b / 1e9:.1f} GB/s  both at once {2 * n / c / 1e9:.1f} "
      f"GB/s aggregate ({c * 1e3:.2f} ms vs {(a + b) * 1e3:.2f} ms serial)", flush=True)
