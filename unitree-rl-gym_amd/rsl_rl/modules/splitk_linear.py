"""nn.Linear whose weight gradient is split over the batch (K) dimension.

PPO mini-batches are tall (24576 x <=512): the library GEMM for
dW = dY^T X puts the whole 24576-long reduction on a handful of output tiles
(a 512x256 dW is 16 tiles for 256 CUs).  Splitting K into chunks turns it into a
batched GEMM with chunks x tiles workgroups plus a small reduction.  Same
parameters and state_dict keys as nn.Linear (checkpoints interchange).
"""

import torch
import torch.nn as nn
import torch.nn.functional as F

SPLIT_MIN_ROWS = 8192
CHUNK = 512  # rows per split-K chunk (4096 -> 512 cut 1 ms off an H1 update)


class _SplitKLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = dy.mm(weight)
        if ctx.needs_input_grad[1]:
            m = x.shape[0]
            c = m // CHUNK
            if c >= 2 and m % CHUNK == 0:
                dw = torch.bmm(dy.view(c, CHUNK, -1).transpose(1, 2), x.view(c, CHUNK, -1)).sum(0)
            else:
                dw = dy.t().mm(x)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.sum(0)
        return dx, dw, db


class SplitKLinear(nn.Linear):
    def forward(self, x):
        if x.dim() == 2 and x.shape[0] >= SPLIT_MIN_ROWS and torch.is_grad_enabled() and x.is_cuda:
            return _SplitKLinearFn.apply(x, self.weight, self.bias)
        return F.linear(x, self.weight, self.bias)
