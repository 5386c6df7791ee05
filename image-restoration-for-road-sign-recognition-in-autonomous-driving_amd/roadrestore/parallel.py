"""Data parallelism: one process per GPU, gradients all-reduced over RCCL.

The reference trains on one device (14:19); the north star shards the batch
over the 8 GPUs of a node.  Each rank runs the full network on its own shard
(per-replica BatchNorm statistics, as torch DDP does) and the gradients are
summed across ranks.

The network's backward (roadrestore.engine) writes every parameter gradient
into one flat fp32 buffer laid out in the order the gradients become final
(final conv, dec1, up1, ..., enc1) and calls a ready-hook after each group.
``DataParallel`` cuts that buffer into ~``bucket_mb`` contiguous buckets and
launches each bucket's all-reduce (in place, no packing copy) on a side
stream as soon as its last gradient is written, so communication overlaps
the rest of the backward; the optimizer waits for the comm stream.  The
1/world_size average is folded into the loss gradient (``grad_scale``), the
exactly-zero gradients (conv biases before a train-mode BN) are not sent.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class DataParallel:
    def __init__(self, model, process_group=None, bucket_mb=25.0, broadcast_params=True):
        self.model = model
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.bucket_bytes = int(bucket_mb * 2 ** 20)
        layout = model.grad_layout()
        order, zero = model._grad_order()
        zs = {id(z) for z in zero}
        self.zero_ids = zs
        # bucket plan over the non-zero part of the flat layout (readiness order)
        self.buckets = []          # (start, end, param-id set)
        off = sum(p.numel() for p in layout if id(p) in zs)
        cur, cur_start, cur_bytes = set(), off, 0
        for p in layout:
            if id(p) in zs:
                continue
            cur.add(id(p))
            cur_bytes += p.numel() * 4
            off += p.numel()
            if cur_bytes >= self.bucket_bytes:
                self.buckets.append((cur_start, off, cur))
                cur, cur_start, cur_bytes = set(), off, 0
        if cur:
            self.buckets.append((cur_start, off, cur))
        self._pending = []
        self._done = set()
        self._launched = set()
        self.comm_stream = None
        if torch.cuda.is_available() and next(model.parameters()).is_cuda:
            self.comm_stream = torch.cuda.Stream()
        model.set_grad_ready_hook(self._on_ready)
        if broadcast_params and self.world > 1:
            with torch.no_grad():
                for t in list(model.parameters()) + list(model.buffers()):
                    dist.broadcast(t.data, src=0, group=self.pg)

    @property
    def grad_scale(self):
        return 1.0 / self.world

    def _on_ready(self, sink, params):
        if self.world == 1:
            return
        for p in params:
            self._done.add(id(p))
        for bi, (a, b, ids) in enumerate(self.buckets):
            if bi in self._launched or not ids <= self._done:
                continue
            self._launched.add(bi)
            view = sink.flat[a:b]
            if self.comm_stream is not None:
                self.comm_stream.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self.comm_stream):
                    work = dist.all_reduce(view, group=self.pg, async_op=True)
            else:
                work = dist.all_reduce(view, group=self.pg, async_op=True)
            self._pending.append(work)
        if len(self._launched) == len(self.buckets):
            self.finish()

    def finish(self):
        """Join every outstanding bucket (the optimizer reads the grads next)."""
        for w in self._pending:
            w.wait()
        if self.comm_stream is not None:
            torch.cuda.current_stream().wait_stream(self.comm_stream)
        self._pending = []
        self._done = set()
        self._launched = set()

    def __call__(self, x):
        return self.model(x)
