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
    def __init__(self, model, process_group=None, bucket_mb=25.0, tail_mb=4.0,
                 broadcast_params=True):
        self.model = model
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.bucket_bytes = int(bucket_mb * 2 ** 20)
        self.tail_bytes = int(tail_mb * 2 ** 20)
        layout = model.grad_layout()
        order, zero = model._grad_order()
        zs = {id(z) for z in zero}
        self.zero_ids = zs
        # bucket plan over the non-zero part of the flat layout (readiness
        # order), cut from the END: the last bucket only becomes ready when
        # the whole backward is done, so its all-reduce is exposed -- it is
        # kept to <= tail_mb (ResUNet: res3..enc1, 3.5 MB), the others to
        # ~bucket_mb (they overlap the rest of the backward)
        self.buckets = []          # (start, end, param-id set)
        start = sum(p.numel() for p in layout if id(p) in zs)
        items, off = [], start
        for p in layout:
            if id(p) in zs:
                continue
            items.append((off, off + p.numel(), id(p)))
            off += p.numel()
        rev, cur, cur_bytes, limit = [], [], 0, self.tail_bytes
        for it in reversed(items):
            nb = (it[1] - it[0]) * 4
            if cur and cur_bytes + nb > limit:
                rev.append(cur)
                cur, cur_bytes, limit = [], 0, self.bucket_bytes
            cur.append(it)
            cur_bytes += nb
        if cur:
            rev.append(cur)
        for b in reversed(rev):
            b = b[::-1]
            self.buckets.append((b[0][0], b[-1][1], {i for _, _, i in b}))
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
