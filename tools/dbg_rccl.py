"""Step-by-step check of RcclComm on one GPU (world-size-1 RCCL group)."""
import faulthandler, os, socket, sys
faulthandler.enable()
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
import torch
import torch.distributed as dist
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
with socket.socket() as sk:
    sk.bind(("127.0.0.1", 0)); port = sk.getsockname()[1]
store = dist.TCPStore("127.0.0.1", port, 1, True)
dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
print("pg up", flush=True)
from roadrestore.parallel import RcclComm
c = RcclComm(None, dev)
print("comm up", c.comm, flush=True)
t = torch.arange(1000, device=dev, dtype=torch.float32)
c.all_reduce_(t)
torch.cuda.synchronize()
print("allreduce ok", t[:4].tolist(), flush=True)
x = torch.randn(10, device=dev)
print("torch op ok", x.sum().item(), flush=True)
with torch.autograd.profiler.record_function("x"):
    pass
print("record_function ok", flush=True)
c.close()
dist.destroy_process_group()
print("done", flush=True)
