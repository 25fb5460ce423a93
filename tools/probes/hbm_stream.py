"""Streaming-bandwidth floor for the update's activation traffic: write-only (fill),
read-only (sum) and read+write (copy) of bf16 buffers the size of one mini-batch's
activations (24,576 rows x 512 / 256 / 128 columns x 2 networks), timed with HIP events
over 50 back-to-back launches."""
import torch

dev = "cuda"
for cols in (512, 256, 128):
    n = 24576 * cols * 2
    x = torch.randn(n, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    mb = n * 2 / 1e6
    for name, fn, bytes_ in (("fill ", lambda: y.fill_(1.0), n * 2),
                             ("copy ", lambda: y.copy_(x), n * 4),
                             ("sum  ", lambda: x.sum(), n * 2)):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1e3
        print(f"{name} {mb:6.1f} MB buffer: {us:7.1f} us  {bytes_ / us / 1e6:6.2f} TB/s")
