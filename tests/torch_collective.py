"""keto_collective over torch.distributed (test / bench harness, not product): the object
partition's all-to-alls on a gloo process group (CPU tests, ranks sharing one GPU) or RCCL
(bench.py, one rank per GPU).  Host buffers in and out, as keto_collective specifies; with
device_buffers=True also keto_collective.alltoallv_device: the library's device buffers on its
own stream -- over RCCL straight GPU to GPU (the collective runs on the library's stream through
torch.cuda.ExternalStream), over gloo staged through host memory on this side."""
import numpy as np
import torch
import torch.distributed as dist


class _DevBytes:
    """a device byte range as a torch tensor (no copy): __cuda_array_interface__"""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3}


class TorchCollective:
    def __init__(self, group=None, device_buffers: bool = False):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
        self.device_buffers = device_buffers  # False: the library stages through host memory itself

    def alltoallv_device(self, send_ptr: int, send_bytes, recv_ptr: int, recv_bytes, stream: int):
        ns, nr = int(sum(send_bytes)), int(sum(recv_bytes))
        with torch.cuda.ExternalStream(stream):
            s = torch.as_tensor(_DevBytes(send_ptr, ns), device="cuda") if ns else torch.zeros(0, dtype=torch.uint8, device="cuda")
            r = torch.as_tensor(_DevBytes(recv_ptr, nr), device="cuda") if nr else torch.zeros(0, dtype=torch.uint8, device="cuda")
            if self.dev == "cuda":  # RCCL: device to device on the library's stream
                dist.all_to_all_single(r, s, [int(x) for x in recv_bytes], [int(x) for x in send_bytes], group=self.group)
            else:  # gloo: staged here
                hr = torch.empty(nr, dtype=torch.uint8)
                dist.all_to_all_single(hr, s.cpu(), [int(x) for x in recv_bytes], [int(x) for x in send_bytes],
                                       group=self.group)
                r.copy_(hr.to("cuda"))

    def alltoall_u64(self, send: np.ndarray) -> np.ndarray:
        s = torch.from_numpy(send.astype(np.int64)).to(self.dev)
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s, group=self.group)
        return r.cpu().numpy().astype(np.uint64)

    def alltoallv(self, send: np.ndarray, send_bytes, recv: np.ndarray, recv_bytes):
        s = torch.from_numpy(send).to(self.dev)
        r = torch.empty(int(sum(recv_bytes)), dtype=torch.uint8, device=self.dev)
        dist.all_to_all_single(r, s, [int(x) for x in recv_bytes], [int(x) for x in send_bytes], group=self.group)
        recv[:] = r.cpu().numpy()

    def allreduce_max_u64(self, v: int) -> int:
        t = torch.tensor([int(v)], dtype=torch.int64, device=self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())
