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
the rest of the backward; the optimizer waits for the comm stream.  On GPUs
the all-reduces are bare ncclAllReduce calls on a communicator of our own
(``RcclComm``), so the whole step, bucket all-reduces included, is HIP-graph
capturable: the side stream forks from and joins the capturing stream and
the collectives are recorded into the graph (bench.py captures it at every N).  The
1/world_size average is folded into the loss gradient (``grad_scale``), the
exactly-zero gradients (conv biases before a train-mode BN) are not sent in
train mode.  In eval mode (a fine-tune with frozen BatchNorm statistics)
those biases have real gradients, so the zero section of the flat buffer goes
out as one more bucket once the backward is done.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from . import engine


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]     # NCCL_UNIQUE_ID_BYTES


def uid_to_bytes(uid):
    """The raw 128 bytes of an ncclUniqueId (reading the c_char field would
    stop at the first NUL)."""
    return ctypes.string_at(ctypes.addressof(uid), ctypes.sizeof(uid))


def uid_from_bytes(raw):
    if len(raw) != ctypes.sizeof(_UniqueId):
        raise RuntimeError("RcclComm: bad unique id")
    uid = _UniqueId()
    ctypes.memmove(ctypes.addressof(uid), raw, len(raw))
    return uid


class RcclComm:
    """A communicator of its own on the RCCL library torch ships (rccl.h:
    ncclGetUniqueId / ncclCommInitRank / ncclAllReduce), for the gradient
    all-reduce of the data-parallel step.

    Why not ``dist.all_reduce``: ProcessGroupNCCL's watchdog thread polls the
    completion event of every work it issues, and polling an event recorded
    into a HIP graph under capture is an error that kills the process.  A
    bare ncclAllReduce on the caller's stream has no such host-side state, so
    the whole step -- bucket all-reduces included -- captures into one HIP
    graph and replays at N > 1 as it does at N = 1.  The unique id travels
    over the existing torch process group (rank 0 -> all)."""

    NCCL_FLOAT32, NCCL_SUM = 7, 0

    def __init__(self, process_group=None, device=None):
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if not os.path.exists(path):
            path = "librccl.so"
        self.lib = lib = ctypes.CDLL(path)
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                         _UniqueId, ctypes.c_int]
        lib.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p]
        lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        self.rank = dist.get_rank(process_group)
        self.world = dist.get_world_size(process_group)
        uid = _UniqueId()
        if self.rank == 0:
            self._check(lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        obj = [uid_to_bytes(uid) if self.rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=process_group)
        uid = uid_from_bytes(obj[0])
        self.comm = ctypes.c_void_p()
        with torch.cuda.device(device):
            self._check(lib.ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank),
                        "ncclCommInitRank")

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.lib.ncclGetErrorString(rc).decode()} ({rc})")

    def all_reduce_(self, t, stream=None):
        """In-place sum of a contiguous fp32 device tensor over the ranks,
        enqueued on ``stream`` (default: the current stream)."""
        if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
            raise ValueError("RcclComm.all_reduce_ takes a contiguous fp32 device tensor")
        st = stream if stream is not None else torch.cuda.current_stream(t.device)
        self._check(self.lib.ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(),
                                           self.NCCL_FLOAT32, self.NCCL_SUM, self.comm,
                                           st.cuda_stream), "ncclAllReduce")

    def close(self):
        if self.comm:
            self.lib.ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()


class DataParallel:
    def __init__(self, model, process_group=None, bucket_mb=25.0, tail_mb=4.0,
                 broadcast_params=True, force_comm=False, comm=None):
        self.model = model
        # force_comm: launch the bucket all-reduces even at world size 1 (a
        # 1-GPU rehearsal of the N > 1 step, e.g. its HIP-graph capture)
        self.force_comm = force_comm
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
        self.zero_span = (0, start)
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
        # comm: "rccl" = RcclComm (graph-capturable, the default on GPUs with
        # an RCCL process group), "torch" = dist.all_reduce (gloo on CPU)
        if comm is None:
            comm = os.environ.get("RR_DP_COMM")
        if comm is None:
            comm = ("rccl" if self.comm_stream is not None and dist.is_initialized()
                    and dist.get_backend(process_group) == "nccl" else "torch")
        self.rccl = None
        if comm == "rccl" and (self.world > 1 or force_comm):
            self.rccl = RcclComm(process_group, next(model.parameters()).device)
        model.set_grad_ready_hook(self._on_ready)
        if broadcast_params and self.world > 1:
            with torch.no_grad():
                for t in list(model.parameters()) + list(model.buffers()):
                    dist.broadcast(t.data, src=0, group=self.pg)

    @property
    def grad_scale(self):
        return 1.0 / self.world

    def _on_ready(self, sink, params):
        if self.world == 1 and not self.force_comm:
            return
        for p in params:
            self._done.add(id(p))
        for bi, (a, b, ids) in enumerate(self.buckets):
            if bi in self._launched or not ids <= self._done:
                continue
            self._launched.add(bi)
            self._reduce(sink.flat[a:b])
        if len(self._launched) == len(self.buckets):
            # eval mode: the conv biases feeding a BN have real gradients
            # (written during the backward, which is complete once the last
            # bucket is ready), so the zero section is exchanged too
            a, b = self.zero_span
            if b > a and not self.model.training:
                self._reduce(sink.flat[a:b])
            self.finish()

    def _reduce(self, view):
        # the bucket's weight grads are final once the weight-grad reduces
        # forked onto the reduce stream so far have run (engine.reduce_stream)
        if self.rccl is not None:
            self.comm_stream.wait_stream(torch.cuda.current_stream())
            engine.join_wgrad_reduces(self.comm_stream)
            self.rccl.all_reduce_(view, self.comm_stream)   # joined in finish()
        elif self.comm_stream is not None:
            self.comm_stream.wait_stream(torch.cuda.current_stream())
            engine.join_wgrad_reduces(self.comm_stream)
            with torch.cuda.stream(self.comm_stream):
                self._pending.append(dist.all_reduce(view, group=self.pg, async_op=True))
        else:
            if view.is_cuda:
                engine.join_wgrad_reduces()
            self._pending.append(dist.all_reduce(view, group=self.pg, async_op=True))

    def finish(self):
        """Join every outstanding bucket (the optimizer reads the grads next)."""
        for w in self._pending:
            w.wait()
        if self.comm_stream is not None:
            torch.cuda.current_stream().wait_stream(self.comm_stream)
        self._pending = []
        self._done = set()
        self._launched = set()

    def close(self):
        if self.rccl is not None:
            self.rccl.close()
            self.rccl = None

    def __call__(self, x):
        return self.model(x)
